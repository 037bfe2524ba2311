set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/prof_worker_host.py > gpurun_out/prof_worker_host.txt 2>&1 || { tail -20 gpurun_out/prof_worker_host.txt; exit 1; }
head -3 gpurun_out/prof_worker_host.txt
