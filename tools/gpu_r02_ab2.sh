# same-box A/B of env knobs on the bench (no cpu baseline / parity), printing RTFx and per-class ms
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-ab2}
i=0
for kv in "BASE=1" $KNOBS; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
