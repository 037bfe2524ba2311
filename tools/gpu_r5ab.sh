set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in 5 6 7 4 5 6; do
  echo "== compact $c/8"; VLOG_AMD_COMPACT_8THS=$c timeout -k 10 300 python3 bench.py --workload variable --steps 4 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'passes', c.get('decoder_steps'), 'rowsteps', c.get('decoder_row_steps'), 'xattn', k['cross_attn']['ms'], 'dec_gemm', k['dec_gemm']['ms'], d['stages_s_per_step'])" || exit 1
done 2>&1 | tee gpurun_out/ab_compact.txt
