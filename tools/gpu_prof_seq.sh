set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_worker_seq.py > gpurun_out/prof_seq.json 2> gpurun_out/prof_seq.err && cat gpurun_out/prof_seq.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_seq -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_worker_seq.py > $GRAFT_REPO_ROOT/gpurun_out/prof_seq_rocprof.log 2>&1 && head -30 $(ls $GRAFT_REPO_ROOT/gpurun_out/prof_seq/*kernel_stats.csv | head -1) | cut -d, -f1-5
