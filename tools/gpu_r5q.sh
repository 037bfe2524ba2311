set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for S in 3 4 2 5 3 6 4; do
  echo "== splits $S"; VLOG_AMD_XSPLITS=$S timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], 'xattn', k['cross_attn']['ms'], 'comb', k['cross_comb']['ms'], 'frac', d['roofline']['frac'])" || exit 1
done 2>&1 | tee gpurun_out/ab_xsplits.txt
