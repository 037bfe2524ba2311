# The worker's sequential beam-5 call on the GPU: beam parity tests first (TESTS), then the engine event profile
# for each arm in ARMS (";"-separated: engine options "k=v,k=v", "env:NAME=VALUE" for an environment variable,
# "" = defaults; tools/prof_worker_seq.py) and a rocprofv3 kernel-trace of the default arm
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-seq}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_gemv.py tests/test_gpu_decode.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/tests_$TAG.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " gpurun_out/tests_$TAG.log | head -30; exit $rc; }
fi
IFS=';' read -ra arms <<< "${ARMS:-}"
[ ${#arms[@]} -eq 0 ] && arms=("")
for arm in "${arms[@]}"; do
  envs=(); opt="$arm"
  if [[ "$arm" == env:* ]]; then envs=("${arm#env:}"); opt=""; fi
  env "${envs[@]}" timeout -k 10 300 python tools/prof_worker_seq.py large-v3 "$opt" >> gpurun_out/prof_$TAG.jsonl 2>> gpurun_out/prof_$TAG.err || { tail -20 gpurun_out/prof_$TAG.err; exit 1; }
  echo "arm [$arm]: $(tail -1 gpurun_out/prof_$TAG.jsonl | cut -c1-120)"
done
[ -n "$NO_ROCPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rp_$TAG -o run -- python3 $R/tools/prof_worker_seq.py large-v3 > $R/gpurun_out/rp_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/rp_$TAG.log; exit 1; }
python3 $R/tools/rp_summary.py $R/gpurun_out/rp_$TAG/run_kernel_stats.csv 24
