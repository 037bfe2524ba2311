set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for f in 1 0 1 0; do
  echo "== fold $f"; VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], k['dec_gemm']['ms'], k['cross_attn']['ms'])" || exit 1
done 2>&1 | tee gpurun_out/fold_ab3.txt
for f in 1 0; do
  echo "== c5 fold $f"; VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], k['dec_gemm']['ms'], k['cross_attn']['ms'])" || exit 1
done 2>&1 | tee gpurun_out/c5_fold_ab3.txt
timeout -k 10 300 python3 -u tools/diag_fold.py 2>&1 | tee gpurun_out/diag_fold3.txt | tail -5 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_logprobs.py tests/test_gpu_big_rows.py 2>&1 | tee gpurun_out/t_r5l.txt | tail -5
