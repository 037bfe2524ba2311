set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_r05_u.log 2>&1
rc=$?; tail -45 gpurun_out/gpu_tests_r05_u.log; exit $rc
