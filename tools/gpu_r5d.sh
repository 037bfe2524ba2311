set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/diag_fold.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/diag_fold.txt || exit 1
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-variable"
for f in 1 0 1 0; do
  VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 300 $B > gpurun_out/ab_f$f.json 2> gpurun_out/ab_f$f.err || { tail -15 gpurun_out/ab_f$f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_f$f.json')); k=d['kernels_one_step']; print('FOLD=$f', d['value'], d['ms_per_step'], d['config']['token_crc32'], d['stages_s_per_step']['decode'], {n: k[n]['ms'] for n in ('dec_gemm','dec_other','cross_comb') if n in k})" | tee -a gpurun_out/ab_fold_r05_d.txt
done
export VLOG_AMD_PARITY_OUT=$GRAFT_REPO_ROOT/gpurun_out/parity_r5d.jsonl
timeout -k 10 1500 python -u -m pytest tests/test_gpu_logprobs.py tests/test_gpu_split.py tests/test_gpu_big_rows.py tests/test_gpu_gates.py -x -v --timeout 900 --timeout-method thread > gpurun_out/t_r5d.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/t_r5d.log | tail -30; exit $rc
