# Round evidence in one gpurun call, every GPU step under its own time limit and chained with &&:
#   1. the GPU suite as the driver runs it (python -m pytest tests -m gpu), log under gpurun_out/
#   2. the driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5), with its wall time
#   3. rocprofv3 --kernel-trace --stats of a short bench run (same kernels)
#   4. PMC HBM-traffic passes of the dominant kernel (tools/pmc_traffic.sh)
# SKIP_TESTS=1 / SKIP_BENCH=1 / SKIP_PROF=1 / NO_PMC=1 drop steps; WORKER=1 appends the worker-call lines
# (tools/bench_worker_call.py: margin model, and random weights at T=0 as round 2 measured).  TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-r03}
export VLOG_AMD_PROGRESS=$R/gpurun_out/progress_$TAG.log
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=20 --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -30; exit $rc; }
fi
[ -n "$SKIP_BENCH" ] && exit 0
t0=$(date +%s.%N)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
t1=$(date +%s.%N)
echo "{\"cmd\": \"python3 bench.py --gpus 1 --steps 20 --warmup 5\", \"wall_s\": $(python3 -c "print(round($t1-$t0,1))")}" > gpurun_out/bench_${TAG}_wall.json
cat gpurun_out/bench_$TAG.json gpurun_out/bench_${TAG}_wall.json
[ -n "$SKIP_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-variable > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
head -25 $(ls $R/gpurun_out/prof_$TAG/*kernel_stats.csv | head -1) | cut -d, -f1-5
tail -1 $R/gpurun_out/prof_$TAG.log
if [ -z "$NO_PMC" ]; then
  BENCH_ARGS=--no-variable bash $R/tools/pmc_traffic.sh || exit 1
fi
[ -z "$WORKER" ] && exit 0
cd $R
timeout -k 10 600 python tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_$TAG.json 2> gpurun_out/worker_$TAG.err || { tail -20 gpurun_out/worker_$TAG.err; exit 1; }
cat gpurun_out/worker_$TAG.json
timeout -k 10 600 python tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 --random-weights --temperature 0 > gpurun_out/worker_${TAG}_random_t0.json 2> gpurun_out/worker_${TAG}_random_t0.err || { tail -20 gpurun_out/worker_${TAG}_random_t0.err; exit 1; }
cat gpurun_out/worker_${TAG}_random_t0.json
