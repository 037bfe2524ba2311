set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DGB_BIG=1 timeout -k 10 120 ./tools/dec_gemm_bench 100 750 > gpurun_out/dgb_r6_750b.txt 2>&1 &&
DGB_BIG=1 timeout -k 10 120 ./tools/dec_gemm_bench 100 384 > gpurun_out/dgb_r6_384b.txt 2>&1 &&
DGB_BIG=1 timeout -k 10 120 ./tools/dec_gemm_bench 100 640 > gpurun_out/dgb_r6_640b.txt 2>&1
rc=$?; grep -v unsupp gpurun_out/dgb_r6_750b.txt | tail -80; exit $rc
