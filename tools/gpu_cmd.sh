set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VLOG_AMD_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_r06_rehearsal_2ranks.json 2> gpurun_out/bench_r06_rehearsal_2ranks.err || { tail -30 gpurun_out/bench_r06_rehearsal_2ranks.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_rehearsal_2ranks.json')); print(d['value'], d['n_gpus'], d['ranks'], d['config'].get('gpus_shared'), d.get('parity',{}).get('identical'))"
grep -ci "nccl\|rccl" gpurun_out/bench_r06_rehearsal_2ranks.err || true
