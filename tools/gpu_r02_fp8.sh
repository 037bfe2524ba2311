# fp8 cross memory: its GPU tests, the opt-in bench line, rocprof stats and PMC traffic of its xattn kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-fp8}
export VLOG_AMD_PARITY_OUT=$R/gpurun_out/parity_$TAG.jsonl
rm -f $VLOG_AMD_PARITY_OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_configs.py -k "fp8" -v --timeout 500 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/tests_$TAG.log
timeout -k 10 600 python bench.py --cross-fp8 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --cross-fp8 --no-cpu-baseline --no-parity > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
head -8 $(ls $R/gpurun_out/prof_$TAG/*kernel_stats.csv | head -1) | cut -d, -f1-5
BENCH_ARGS=--cross-fp8 bash $R/tools/pmc_traffic.sh
