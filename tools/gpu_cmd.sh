set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DGB_LC=1 DGB_COPIES=40 DGB_ACOPIES=8 timeout -k 10 150 ./tools/dec_gemm_bench 50 750 > gpurun_out/dgb_r6_lcwb_750.txt 2>&1 || { tail -20 gpurun_out/dgb_r6_lcwb_750.txt; exit 1; }
grep -E "LCWB|LC   bm=128 bn=128|LC   bm= 64 bn= 64" gpurun_out/dgb_r6_lcwb_750.txt | sed -E 's/ +/ /g'
DGB_LC=1 DGB_COPIES=40 DGB_ACOPIES=8 timeout -k 10 150 ./tools/dec_gemm_bench 50 150 > gpurun_out/dgb_r6_lcwb_150.txt 2>&1 || { tail -20 gpurun_out/dgb_r6_lcwb_150.txt; exit 1; }
grep -E "LCWB|LC   bm= 64 bn= 64|LC   bm= 96" gpurun_out/dgb_r6_lcwb_150.txt | sed -E 's/ +/ /g'
