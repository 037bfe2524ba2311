set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_8p.txt 2>&1 && head -7 gpurun_out/gemm_8p.txt &&
VLOG_AMD_GEMM_8P=2 timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_8p2.txt 2>&1 && head -7 gpurun_out/gemm_8p2.txt &&
timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_8p.txt 2>&1 && head -7 gpurun_out/gemm_8p.txt
