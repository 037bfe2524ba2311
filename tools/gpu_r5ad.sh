set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in 16 4 6 16 4 8; do
  echo "== xsplits max $c"; VLOG_AMD_XSPLITS_MAX=$c timeout -k 10 300 python3 bench.py --workload variable --steps 4 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'xattn', k['cross_attn']['ms'], 'comb', k['cross_comb']['ms'], d['stages_s_per_step']['decode'])" || exit 1
done 2>&1 | tee gpurun_out/ab_xsplits_max.txt
