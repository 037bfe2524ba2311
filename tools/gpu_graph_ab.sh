set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/split_g.log 2>&1; rc=$?; tail -3 gpurun_out/split_g.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/split_g.log | head -20; exit $rc; }
timeout -k 10 600 python tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_g1.json 2> gpurun_out/worker_g1.err && cat gpurun_out/worker_g1.json &&
timeout -k 10 600 python tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 --no-graph > gpurun_out/worker_g0.json 2> gpurun_out/worker_g0.err && cat gpurun_out/worker_g0.json &&
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-profile --no-cpu-baseline --no-parity > gpurun_out/bench_g1.json 2>/dev/null && head -c 600 gpurun_out/bench_g1.json && echo &&
VLOG_AMD_DEC_GRAPH=0 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-profile --no-cpu-baseline --no-parity > gpurun_out/bench_g0.json 2>/dev/null && head -c 600 gpurun_out/bench_g0.json &&
timeout -k 10 900 python tools/bench_product.py --hours 1 10 > gpurun_out/product.json 2> gpurun_out/product.err && cat gpurun_out/product.json && timeout -k 10 300 python tools/blas_probe.py > gpurun_out/blas_probe.txt 2>&1 && cat gpurun_out/blas_probe.txt
