# Full GPU suite on the current defaults, then bench.py A/B of decoder ring-GEMM tile plans (env knobs; ':' joins
# several variables of one arm).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-dec}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
fi
i=0
for kv in ${ARMS:-"BASE=1" "VLOG_AMD_DEC_GEMM=fc2=64:VLOG_AMD_DEC_COLS=fc2=64" "VLOG_AMD_DEC_GEMM=qkv=64:VLOG_AMD_DEC_COLS=qkv=64" "VLOG_AMD_DEC_GEMM=fc2=64,qkv=64:VLOG_AMD_DEC_COLS=fc2=64,qkv=64" "BASE=1" "VLOG_AMD_DEC_GEMM=fc2=64,qkv=64:VLOG_AMD_DEC_COLS=fc2=64,qkv=64"}; do
  i=$((i+1))
  env ${kv//:/ } timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
