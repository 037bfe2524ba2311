# A/B of an engine env knob on the bench (no parity / cpu baseline), then the config parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-parity --no-cpu-baseline > gpurun_out/bench_${TAG}_a.json 2> gpurun_out/bench_${TAG}_a.err && python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_a.json'));print('A',d['value'],d['stages_s_per_step'],{k:v['ms'] for k,v in d['kernels_one_step'].items()})" &&
env $KNOB timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-parity --no-cpu-baseline > gpurun_out/bench_${TAG}_b.json 2> gpurun_out/bench_${TAG}_b.err && python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_b.json'));print('B',d['value'],d['stages_s_per_step'],{k:v['ms'] for k,v in d['kernels_one_step'].items()})" || exit $?
if [ -n "$TESTS" ]; then
  export VLOG_AMD_PARITY_OUT=$R/gpurun_out/parity_$TAG.jsonl
  rm -f $VLOG_AMD_PARITY_OUT
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?
  tail -15 gpurun_out/tests_$TAG.log
  exit $rc
fi
