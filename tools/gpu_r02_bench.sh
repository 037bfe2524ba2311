# Round-2 evidence: the default bench line (as the driver runs it), a rocprofv3 kernel-trace --stats pass of the
# same command, and the PMC HBM-traffic passes of the dominant kernel.  Each GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
head -25 $(ls $R/gpurun_out/prof_$TAG/*kernel_stats.csv | head -1) | cut -d, -f1-5
tail -1 $R/gpurun_out/prof_$TAG.log
[ -n "$NO_PMC" ] && exit 0
bash $R/tools/pmc_traffic.sh
