# Round-2 feature check: word timestamps, throughput-mode worker call, the full GPU suite, and the worker-call bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-feat}
export VLOG_AMD_PARITY_OUT=$R/gpurun_out/parity_$TAG.jsonl
rm -f $VLOG_AMD_PARITY_OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests_$TAG.log | tail -80
tail -5 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$WORKER_BENCH" ]; then
  timeout -k 10 900 python -u tools/bench_worker_call.py $WORKER_BENCH > gpurun_out/worker_call_$TAG.json 2> gpurun_out/worker_call_$TAG.err
  rc2=$?
  cat gpurun_out/worker_call_$TAG.json; [ $rc2 -ne 0 ] && tail -20 gpurun_out/worker_call_$TAG.err
  exit $(( rc > rc2 ? rc : rc2 ))
fi
exit $rc
