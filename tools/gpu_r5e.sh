set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/diag_fold.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/diag_fold.txt
