set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in dgb_old dgb_new; do
  echo "== $b"; VLOG_AMD_RING_LDS=72 timeout -k 10 200 ./abtmp/$b 200 750 2>&1 | grep -E "rows= 64 cols=64 pad= 0|empty" | grep -v "kr=1280" || exit 1
done 2>&1 | tee gpurun_out/dgb_ab2.txt
echo "== config5" | tee gpurun_out/c5.txt
timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variable 2>&1 | tee -a gpurun_out/c5.txt | tail -3 || exit 1
for f in 1 0; do
  echo "== fold $f"; VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 || exit 1
done 2>&1 | tee gpurun_out/fold_ab2.txt
timeout -k 10 300 python3 -u tools/diag_fold.py 2>&1 | tee gpurun_out/diag_fold2.txt | tail -5 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_logprobs.py tests/test_gpu_split.py tests/test_gpu_words.py 2>&1 | tee gpurun_out/t_r5j.txt | tail -5
