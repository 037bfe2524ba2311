set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for f in 0 4 0 4; do
  echo "== XFORM=$f"; VLOG_AMD_XFORM=$f XB_ABL="0,7" XB_F8=0 timeout -k 10 120 ./abtmp/xattn_bench 150 3 || exit 1
done 2>&1 | tee gpurun_out/xattn_ab_r05_b.txt
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-variable"
for f in 0 4 0 4; do
  VLOG_AMD_XFORM=$f timeout -k 10 300 $B > gpurun_out/ab_x$f.json 2> gpurun_out/ab_x$f.err || { tail -5 gpurun_out/ab_x$f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_x$f.json')); print('XFORM=$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['config']['token_crc32'], d['stages_s_per_step'])" | tee -a gpurun_out/bench_ab_r05_b.txt
done
VLOG_AMD_XFORM=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_xattn.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
