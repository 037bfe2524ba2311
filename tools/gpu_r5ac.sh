set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread "tests/test_gpu_logprobs.py::test_row_set_decode_every_step" "tests/test_gpu_gates.py::test_config4_variable_length_gates_and_row_set_decode" tests/test_gpu_failure.py "tests/test_gpu_gates.py::test_config5_beam_compaction_variable_length" 2>&1 | tee gpurun_out/t_r5ac.txt | tail -3 || exit 1
for c in 7 5 7; do
  echo "== compact $c/8"; VLOG_AMD_COMPACT_8THS=$c timeout -k 10 300 python3 bench.py --workload variable --steps 4 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'rowsteps', c.get('decoder_row_steps'), 'xattn', k['cross_attn']['ms'], d['stages_s_per_step'])" || exit 1
done 2>&1 | tee -a gpurun_out/ab_compact.txt
