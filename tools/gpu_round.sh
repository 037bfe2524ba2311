set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err || { tail -20 gpurun_out/bench_new.err; exit 1; }
cat gpurun_out/bench_new.json
VLOG_AMD_GEMM_BIG=0 VLOG_AMD_GEMM_SKINNY=0 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err || { tail -20 gpurun_out/bench_old.err; exit 1; }
cat gpurun_out/bench_old.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/prof2.log 2>&1 || { tail -20 $R/gpurun_out/prof2.log; exit 1; }
head -25 $(ls $R/gpurun_out/prof2/*kernel_stats.csv | head -1)
