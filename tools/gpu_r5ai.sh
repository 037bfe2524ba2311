set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in 1 0 1 0; do
  echo "== variable decode_graph $g"; VLOG_AMD_DEC_GRAPH=$g timeout -k 10 300 python3 bench.py --workload variable --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-profile 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['token_crc32'], d['stages_s_per_step'])" || exit 1
  echo "== uniform decode_graph $g"; VLOG_AMD_DEC_GRAPH=$g timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variable --no-profile 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['token_crc32'], d['stages_s_per_step'])" || exit 1
done 2>&1 | tee gpurun_out/ab_dec_graph.txt
