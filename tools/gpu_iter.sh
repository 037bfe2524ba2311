# iteration: targeted GPU tests, decoder GEMM microbench, full bench (one gpurun call; each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-iter}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_attention.py tests/test_gpu_parity.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -25 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$DEC" ]; then timeout -k 10 150 ./tools/dec_gemm_bench 200 150 > gpurun_out/dec_$TAG.txt 2>&1 || exit 1; grep -E "RING|launch_gemm|empty" gpurun_out/dec_$TAG.txt; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
