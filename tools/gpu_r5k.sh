set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 0; do
  VLOG_AMD_DEC_LN_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf$f -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-variable > gpurun_out/pf$f.log 2>&1 || exit 1
done


find gpurun_out/pf0 gpurun_out/pf1 -type f ! -name "*kernel_stats.csv" -delete; du -sh gpurun_out
