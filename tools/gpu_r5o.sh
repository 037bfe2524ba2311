set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BENCH_ARGS=--no-variable bash tools/pmc_traffic.sh || exit 1
cd $R
timeout -k 10 400 python3 -u tools/shard_balance.py 2 150 2 > gpurun_out/shard_balance_r05.json 2> gpurun_out/shard_balance_r05.err || { tail -20 gpurun_out/shard_balance_r05.err; exit 1; }
cat gpurun_out/shard_balance_r05.json
timeout -k 10 600 python3 tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_call_r05.json 2> gpurun_out/worker_call_r05.err || { tail -20 gpurun_out/worker_call_r05.err; exit 1; }
head -c 1500 gpurun_out/worker_call_r05.json
