# microbench + GPU tests + bench (one gpurun call); every GPU step time-limited, chained with &&
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/gemm_bench 5 > gpurun_out/gemm_bench.txt 2>&1 && cat gpurun_out/gemm_bench.txt &&
VLOG_AMD_GEMM_BIG=0 VLOG_AMD_GEMM_SKINNY=0 timeout -k 10 120 ./tools/gemm_bench 5 > gpurun_out/gemm_bench_tiled.txt 2>&1 && cat gpurun_out/gemm_bench_tiled.txt &&
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 && tail -2 gpurun_out/gpu_tests.log &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err && cat gpurun_out/bench_new.json
rc=$?
[ $rc -ne 0 ] && tail -30 gpurun_out/gpu_tests.log gpurun_out/bench_new.err 2>/dev/null
exit $rc
