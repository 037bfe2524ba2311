# Diagnostic: the beam parity test under each VLOG_AMD_SEL_ABL setting of logits_select_kernel (bit 0 plain row
# loads, bit 1 K-round top-k); assertion failures continue, any crash/timeout stops the script
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for a in ${ABLS:-0 1 2 3}; do
  VLOG_AMD_SEL_ABL=$a timeout -k 10 300 python -u -m pytest ${SEL_TEST:-tests/test_gpu_decode.py::test_beam_search_matches_oracle} -x -q --timeout 200 --timeout-method thread > gpurun_out/sel_abl$a.log 2>&1
  rc=$?
  echo "abl=$a rc=$rc $(tail -1 gpurun_out/sel_abl$a.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
