set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_split.py "tests/test_gpu_logprobs.py::test_row_set_decode_every_step" 2>&1 | tee gpurun_out/t_r5ae.txt | tail -2 || exit 1
for c in 0 16 0 16; do
  echo "== xsplits max env $c (0 = the rule)"; VLOG_AMD_XSPLITS_MAX=$c timeout -k 10 300 python3 bench.py --workload variable --steps 4 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'xattn', k['cross_attn']['ms'], 'comb', k['cross_comb']['ms'], d['stages_s_per_step']['decode'])" || exit 1
done 2>&1 | tee -a gpurun_out/ab_xsplits_max.txt
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('uniform', d['value'], d['config']['token_crc32'])" | tee -a gpurun_out/ab_xsplits_max.txt
