set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 1 0 1; do
  echo "== PERSIST=$v"; VLOG_AMD_GEMM_PERSIST=$v GEMM_ONLY="150 win" timeout -k 10 200 ./tools/gbx 10 || exit 1
done 2>&1 | tee gpurun_out/gemm_persist_ab.txt
