set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 1 0 1; do
  echo "== 4W=$v"; VLOG_AMD_GEMM_4W=$v timeout -k 10 120 ./tools/gb4w 10 || exit 1
done 2>&1 | grep -v "dec\.\|tiny" | tee gpurun_out/gemm4w_ab.txt
