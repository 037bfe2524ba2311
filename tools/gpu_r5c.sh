set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do XB_ABL="0,7,16" XB_F8=0 timeout -k 10 120 ./abtmp/xattn_bench 150 3 || exit 1; done 2>&1 | tee gpurun_out/xattn_blocked_r05_c.txt
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-variable"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/ab_blk$i.json 2> gpurun_out/ab_blk$i.err || { tail -5 gpurun_out/ab_blk$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_blk$i.json')); print('blocked', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['config']['token_crc32'], d['stages_s_per_step'])" | tee -a gpurun_out/bench_blk_r05_c.txt
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_xattn.py tests/test_gpu_words.py tests/test_gpu_fp8.py tests/test_gpu_parity.py tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r5c.log 2>&1; rc=$?; tail -3 gpurun_out/t_r5c.log; exit $rc
