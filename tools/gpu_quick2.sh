set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 && tail -2 gpurun_out/gpu_tests.log &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err && cat gpurun_out/bench_new.json &&
timeout -k 10 600 python bench.py --no-cpu-baseline --beam 5 --windows 60 --steps 1 > gpurun_out/bench_beam5.json 2> gpurun_out/bench_beam5.err && cat gpurun_out/bench_beam5.json
rc=$?
[ $rc -ne 0 ] && tail -30 gpurun_out/gpu_tests.log gpurun_out/bench_new.err gpurun_out/bench_beam5.err 2>/dev/null
exit $rc
