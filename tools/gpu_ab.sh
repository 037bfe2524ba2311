# GPU tests + bench A/B on an env knob (one gpurun call); every GPU step time-limited, chained with &&
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-ab}
KNOB=${KNOB:-VLOG_AMD_DEC_SPLIT=0}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && tail -3 gpurun_out/gpu_tests_$TAG.log &&
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
env $KNOB timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_b.json 2> gpurun_out/bench_${TAG}_b.err && cat gpurun_out/bench_${TAG}_b.json
rc=$?
[ $rc -ne 0 ] && tail -30 gpurun_out/gpu_tests_$TAG.log gpurun_out/bench_$TAG.err gpurun_out/bench_${TAG}_b.err 2>/dev/null
exit $rc
