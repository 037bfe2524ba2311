set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_words.py "tests/test_gpu_gates.py::test_config5_alignment_large_v3_vs_oracle" tests/test_gpu_multi.py 2>&1 | tail -2 || exit 1
timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 > gpurun_out/bench_r05_c5_final.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r05_c5_final.json')); print(d['value'], d['config']['token_crc32'], d['stages_s_per_step'])"
