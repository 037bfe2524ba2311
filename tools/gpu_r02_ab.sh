# bench.py A/B of env-knob arms (ARMS, ':' joins variables of one arm), then (unless NOFULL) the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-ab}
i=0
for kv in $ARMS; do
  i=$((i+1))
  env ${kv//:/ } timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
[ -n "$NOFULL" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
exit 0
