set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_a.txt 2>&1 && head -7 gpurun_out/gemm_a.txt &&
VLOG_AMD_GEMM_8P=2 timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_b.txt 2>&1 && head -7 gpurun_out/gemm_b.txt &&
timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/gemm_a2.txt 2>&1 && head -7 gpurun_out/gemm_a2.txt
