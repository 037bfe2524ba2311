# Round-end evidence on the final tree: the full GPU suite, then tools/gpu_r02_bench.sh (default bench line,
# rocprofv3 --kernel-trace --stats of the same command, PMC traffic passes).  Each GPU step time-limited.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-r02_g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/gpu_tests_$TAG.log | head -20; exit $rc; }
TAG=$TAG bash $R/tools/gpu_r02_bench.sh
