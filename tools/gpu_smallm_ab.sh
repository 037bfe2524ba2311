# small-M decoder GEMM (decode_gemv) on the GPU: its parity tests, then an A/B on the sequential worker call
# (beam 5 = 5 rows, engine event profiler), arms alternated on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemv.py tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_gemv.log 2>&1
rc=$?; tail -3 gpurun_out/tests_gemv.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " gpurun_out/tests_gemv.log | head -30; exit $rc; }
for cfg in "" "decode_gemv=0" "" "decode_gemv=0"; do
  timeout -k 10 300 python tools/prof_worker_seq.py large-v3 "$cfg" >> gpurun_out/smallm.jsonl 2>> gpurun_out/smallm.err || { tail -20 gpurun_out/smallm.err; exit 1; }
  tail -1 gpurun_out/smallm.jsonl | cut -c1-900
done
