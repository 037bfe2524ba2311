# Infinity Cache residency probe: the first K windows' encoder output loaded with the default policy, the rest
# non-temporal.  xattn_bench (back-to-back launches) then bench.py arms.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-keep}
for k in 0 40 60 150 0 40 60 150; do XB_KEEP=$k XB_ABL=0 XB_F8=0 timeout -k 10 60 ./tools/xattn_bench 150 3 | sed "s/^/keep=$k /" >> gpurun_out/${TAG}_micro.txt 2>&1 || exit 1; done
cat gpurun_out/${TAG}_micro.txt
i=0
for kv in ${ARMS:-BASE=1 VLOG_AMD_XKEEP=30 VLOG_AMD_XKEEP=45 VLOG_AMD_XKEEP=60 VLOG_AMD_XKEEP=150 BASE=1 VLOG_AMD_XKEEP=45}; do
  i=$((i+1))
  env ${kv//:/ } timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
