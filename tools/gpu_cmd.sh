set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export VLOG_AMD_PARITY_OUT=$PWD/gpurun_out/parity_r6_d.jsonl VLOG_AMD_PROGRESS=$PWD/gpurun_out/progress_r6_d.log
VLOG_AMD_ATTN_V=4 timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_attention.py > gpurun_out/tests_r6_attn4.log 2>&1 || { tail -30 gpurun_out/tests_r6_attn4.log; exit 1; }
tail -2 gpurun_out/tests_r6_attn4.log
timeout -k 10 300 python tools/attn_enc_ab.py --forms 2,4,2,4,2,4 > gpurun_out/attn_ab_r6.jsonl 2>&1 || { tail -20 gpurun_out/attn_ab_r6.jsonl; exit 1; }
cat gpurun_out/attn_ab_r6.jsonl
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_big_rows.py \
  "tests/test_gpu_gates.py::test_config5_beam5_identical_to_oracle_beam" "tests/test_gpu_gates.py::test_config5_alignment_large_v3_vs_oracle" \
  "tests/test_gpu_gates.py::test_config5_beam_compaction_variable_length" \
  "tests/test_gpu_logprobs.py::test_config4_5_large_v3_greedy_beam_fp8_every_step" tests/test_gpu_words.py::test_large_v3_beam5_word_timestamps_128_windows > gpurun_out/tests_r6_d.log 2>&1 || { tail -40 gpurun_out/tests_r6_d.log; exit 1; }
tail -3 gpurun_out/tests_r6_d.log
timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --steps 8 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_r06_c5.json 2> gpurun_out/bench_r06_c5.err || { tail -20 gpurun_out/bench_r06_c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_c5.json')); k=d['kernels_one_step']
print(d['value'], d['ms_per_step'], d['config']['token_crc32'], {n: k[n]['ms'] for n in k})"
