set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_logprobs.py tests/test_gpu_split.py tests/test_gpu_sampling.py tests/test_gpu_big_rows.py tests/test_gpu_gates.py 2>&1 | tee gpurun_out/t_r5m.txt | tail -5
