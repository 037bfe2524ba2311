set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_vtt_e2e.py tests/test_gpu_words.py tests/test_gpu_multi.py "tests/test_gpu_gates.py::test_config1_tiny_en_vtt_identical_to_cpu_oracle" 2>&1 | tee gpurun_out/t_r5z.txt | tail -3 || exit 1
timeout -k 10 600 python3 tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_call_r05_b.json 2> gpurun_out/worker_call_r05_b.err || { tail -20 gpurun_out/worker_call_r05_b.err; exit 1; }
head -c 1200 gpurun_out/worker_call_r05_b.json
