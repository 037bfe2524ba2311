set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_words.py "tests/test_gpu_gates.py::test_config5_alignment_large_v3_vs_oracle" 2>&1 | tee gpurun_out/t_r5s.txt | tail -4 || exit 1
for v in 1 0 1; do
  echo "== align_fused $v"; VLOG_AMD_ALIGN_FUSED=$v timeout -k 10 300 python3 tools/prof_align.py 2>&1 | tail -2 || exit 1
done 2>&1 | tee gpurun_out/ab_align_fused.txt
for v in 0 1; do
  echo "== c5 align_fused $v"; VLOG_AMD_ALIGN_FUSED=$v timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['token_crc32'], d['stages_s_per_step'])" || exit 1
done 2>&1 | tee -a gpurun_out/ab_align_fused.txt
