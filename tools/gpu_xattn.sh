# factored cross-attention: its GPU tests first, then the whole GPU suite, then bench A/B (factored vs projected)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 600 python -u -m pytest ${FIRST:-tests/test_gpu_xattn.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}_first.log 2>&1; rc=$?; tail -30 gpurun_out/t_${TAG}_first.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NOALL" ]; then timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}_all.log 2>&1; rc=$?; tail -15 gpurun_out/t_${TAG}_all.log; [ $rc -ne 0 ] && exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
if [ -n "$AB" ]; then VLOG_AMD_CROSS_MODE=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_proj.json 2> gpurun_out/bench_${TAG}_proj.err || { tail -20 gpurun_out/bench_${TAG}_proj.err; exit 1; }; cat gpurun_out/bench_${TAG}_proj.json; fi
for kv in $SWEEP; do env $kv timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$kv.json 2> gpurun_out/bench_${TAG}_$kv.err || { tail -20 gpurun_out/bench_${TAG}_$kv.err; exit 1; }; echo "== $kv"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(d['value'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/bench_${TAG}_$kv.json; done
