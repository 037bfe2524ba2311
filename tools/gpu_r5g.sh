set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for f in 0 1; do
VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 600 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/bench_r05_c5_f$f.json 2> gpurun_out/bench_r05_c5_f$f.err || { tail -20 gpurun_out/bench_r05_c5_f$f.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r05_c5_f$f.json')); k=d['kernels_one_step']
print('c5 fold=$f', d['value'], d['ms_per_step'], d['config']['token_crc32'], d['stages_s_per_step'])
print({n: (v['ms'], v['launches']) for n, v in k.items()})"
done
cd /tmp && export TMPDIR=/tmp
VLOG_AMD_DEC_LN_FOLD=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --beam 5 --word-timestamps --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_c5.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_c5.log; exit 1; }
head -25 $(ls $GRAFT_REPO_ROOT/gpurun_out/prof_c5/*kernel_stats.csv | head -1) | cut -d, -f1-5
