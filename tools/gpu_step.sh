# One gpurun call for iteration: selected GPU tests (TESTS, default the gate tests), then optionally the bench
# (BENCH_ARGS; BENCH=0 skips it).  Every GPU step under its own time limit, chained with &&.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-step}
TESTS=${TESTS:-tests/test_gpu_gates.py}
export VLOG_AMD_PARITY_OUT=$R/gpurun_out/parity_$TAG.jsonl VLOG_AMD_PROGRESS=$R/gpurun_out/progress_$TAG.log
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -x -v --durations=15 --timeout 600 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/tests_$TAG.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " gpurun_out/tests_$TAG.log | head -30; exit $rc; }
fi
[ "${BENCH:-1}" = "0" ] && exit 0
timeout -k 10 ${BENCH_LIMIT:-600} python3 bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
