set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VLOG_AMD_BENCH_SHARE_GPU=1 VLOG_AMD_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_r05_rehearsal_2ranks.json 2> gpurun_out/bench_r05_rehearsal_2ranks.err || { tail -30 gpurun_out/bench_r05_rehearsal_2ranks.err; exit 1; }
head -c 1500 gpurun_out/bench_r05_rehearsal_2ranks.json
