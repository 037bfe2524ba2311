# full GPU tests + bench A/B on a knob + rocprof stats (one gpurun call; each GPU step time-limited, && chained)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && tail -3 gpurun_out/gpu_tests_$TAG.log &&
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
{ [ -z "$KNOB" ] || { env $KNOB timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_b.json 2> gpurun_out/bench_${TAG}_b.err && cat gpurun_out/bench_${TAG}_b.json; }; } &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 &&
head -30 $(ls $R/gpurun_out/prof_$TAG/*kernel_stats.csv | head -1)
rc=$?
[ $rc -ne 0 ] && tail -30 $R/gpurun_out/gpu_tests_$TAG.log $R/gpurun_out/bench_$TAG.err $R/gpurun_out/prof_$TAG.log 2>/dev/null
exit $rc
