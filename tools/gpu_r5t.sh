set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_align -o run -- python3 $R/tools/prof_align.py > $R/gpurun_out/prof_align.log 2>&1 || { tail -20 $R/gpurun_out/prof_align.log; exit 1; }
find $R/gpurun_out/prof_align -type f ! -name "*kernel_stats.csv" -delete
tail -1 $R/gpurun_out/prof_align.log
