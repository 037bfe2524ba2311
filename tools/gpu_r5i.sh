set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in dgb_old dgb_new dgb_old dgb_new; do
  echo "== $b"; VLOG_AMD_RING_LDS=72 timeout -k 10 200 ./abtmp/$b 200 750 2>&1 | grep -E "rows= 64 cols=64 pad= 0|empty" | grep -v "kr=1280" || exit 1
done 2>&1 | tee gpurun_out/dgb_ab.txt
