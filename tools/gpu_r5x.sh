# Every-window parity sweep on the final tree: the large-v3 per-step records at stride 1 (every window, greedy /
# fp8 / beam 5 and the fold opt-in) and the variable-length gates at stride 1; results appended to
# gpurun_out/parity_r5_full.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export VLOG_AMD_PARITY_OUT=$PWD/gpurun_out/parity_r5_full.jsonl VLOG_AMD_RECORDS_STRIDE=1 VLOG_AMD_GATE_STRIDE=1
rm -f $VLOG_AMD_PARITY_OUT
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread \
  "tests/test_gpu_logprobs.py::test_config4_5_large_v3_greedy_beam_fp8_every_step" \
  "tests/test_gpu_gates.py::test_config4_variable_length_gates_and_row_set_decode" > gpurun_out/parity_r5_full.log 2>&1
rc=$?; tail -5 gpurun_out/parity_r5_full.log; exit $rc
