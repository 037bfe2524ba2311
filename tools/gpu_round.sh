# round artifacts in one gpurun call: full GPU suite, default bench (with the CPU baseline), rocprof kernel
# stats of one bench step, PMC traffic of the dominant kernel.  Each GPU step time-limited and && chained.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-round}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && tail -3 gpurun_out/gpu_tests_$TAG.log &&
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
TAG=$TAG bash tools/gpu_prof.sh &&
bash tools/pmc_traffic.sh
rc=$?
[ $rc -ne 0 ] && tail -30 gpurun_out/gpu_tests_$TAG.log gpurun_out/bench_$TAG.err 2>/dev/null
exit $rc
