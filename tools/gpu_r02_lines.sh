# Builder-run lines beside the headline: config 5 (beam 5 + word timestamps), the worker's exact call at T=0
# and as written, each step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-lines}
timeout -k 10 600 python bench.py --beam 5 --word-timestamps --no-cpu-baseline --no-parity > gpurun_out/bench_${TAG}_cfg5.json 2> gpurun_out/bench_${TAG}_cfg5.err || { tail -20 gpurun_out/bench_${TAG}_cfg5.err; exit 1; }
cat gpurun_out/bench_${TAG}_cfg5.json
timeout -k 10 500 python -u tools/bench_worker_call.py --temperature 0 --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_${TAG}_t0.json 2> gpurun_out/worker_${TAG}_t0.err || { tail -20 gpurun_out/worker_${TAG}_t0.err; exit 1; }
cat gpurun_out/worker_${TAG}_t0.json
