# Diagnostic: tools/diag_xattn_beam.py under each environment arm (";"-separated NAME=VALUE, "" = defaults)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
IFS=';' read -ra arms <<< "${ARMS:-}"
[ ${#arms[@]} -eq 0 ] && arms=("")
for arm in "${arms[@]}"; do
  echo "== arm [$arm]"
  env $arm timeout -k 10 300 python tools/diag_xattn_beam.py ${MODEL:-tiny} > gpurun_out/diag_xattn.out 2> gpurun_out/diag_xattn.err
  rc=$?
  cat gpurun_out/diag_xattn.out
  [ $rc -ne 0 ] && { tail -20 gpurun_out/diag_xattn.err; exit $rc; }
done
