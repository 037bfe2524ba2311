# Persistent encoder GEMM: bit-identity test first (short limit), gemm_bench with it on / off, bench.py A/B,
# then the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-pp}
timeout -k 10 240 python -u -m pytest tests/test_gpu_gemm_persist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_t.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do echo "PERSIST=$v"; VLOG_AMD_GEMM_PERSIST=$v timeout -k 10 120 ./tools/gemm_bench 10 2>&1 | head -5; done > gpurun_out/${TAG}_gemm.txt || exit 1; cat gpurun_out/${TAG}_gemm.txt
i=0
for kv in "BASE=1" "VLOG_AMD_GEMM_PERSIST=0" "BASE=1" "VLOG_AMD_GEMM_PERSIST=0"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
[ -n "$NOFULL" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
exit 0
