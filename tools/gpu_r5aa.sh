set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 tools/prof_bench_host.py 5 1 0 > gpurun_out/prof_bench_host_c5.txt 2>&1 || { tail -20 gpurun_out/prof_bench_host_c5.txt; exit 1; }
timeout -k 10 400 python3 tools/prof_bench_host.py 1 0 0 > gpurun_out/prof_bench_host_c4.txt 2>&1 || { tail -20 gpurun_out/prof_bench_host_c4.txt; exit 1; }
grep "^step" gpurun_out/prof_bench_host_c5.txt gpurun_out/prof_bench_host_c4.txt
