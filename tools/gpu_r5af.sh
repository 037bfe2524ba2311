set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in 0 16 0 16; do
  for W in 1 4; do
    echo "== cap env $c (0 = default 8), $W windows"; VLOG_AMD_XSPLITS_MAX=$c timeout -k 10 300 python3 bench.py --windows $W --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], 'decode', d['stages_s_per_step']['decode'], 'xattn', k['cross_attn']['ms'], 'comb', k['cross_comb']['ms'])" || exit 1
  done
done 2>&1 | tee gpurun_out/ab_xsplits_small.txt
for c in 0 16; do
  echo "== variable cap env $c"; VLOG_AMD_XSPLITS_MAX=$c timeout -k 10 300 python3 bench.py --workload variable --steps 4 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'xattn', k['cross_attn']['ms'], 'comb', k['cross_comb']['ms'])" || exit 1
done 2>&1 | tee -a gpurun_out/ab_xsplits_small.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_split.py 2>&1 | tail -2
