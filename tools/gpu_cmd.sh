set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r06.log 2>&1 || { tail -20 gpurun_out/smoke_r06.log; exit 1; }
tail -2 gpurun_out/smoke_r06.log
VLOG_AMD_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_r06_rehearsal_2ranks.json 2> gpurun_out/bench_r06_rehearsal_2ranks.err || { tail -30 gpurun_out/bench_r06_rehearsal_2ranks.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_rehearsal_2ranks.json')); print(d['value'], d['n_gpus'], d['ranks'], d['config'].get('gpus_shared'), d.get('parity',{}).get('identical'))"
echo "rccl/nccl mentions in rank logs: $(grep -ci 'nccl\|rccl' gpurun_out/bench_r06_rehearsal_2ranks.err || true)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-variable > $R/gpurun_out/prof_r06.log 2>&1 || { tail -30 $R/gpurun_out/prof_r06.log; exit 1; }
head -12 $(ls $R/gpurun_out/prof_r06/*kernel_stats.csv | head -1) | cut -d, -f1-5
tail -1 $R/gpurun_out/prof_r06.log
BENCH_ARGS=--no-variable bash $R/tools/pmc_traffic.sh
