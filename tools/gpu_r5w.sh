set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for a in 7 39 7 39 0; do
  echo "== abl $a"; XB_F8=0 XB_ABL=$a timeout -k 10 200 ./tools/xbx 150 3 || exit 1
done 2>&1 | tee gpurun_out/xattn_depth2.txt
