# Round-2 calibration run: the BASELINE-config parity tests (no -x: every config reports), then the bench with
# its parity sample.  Each GPU step is time-limited and the steps are && chained.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r02a}
export VLOG_AMD_PARITY_OUT=$R/gpurun_out/parity_$TAG.jsonl
rm -f $VLOG_AMD_PARITY_OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_vtt_e2e.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/cfg_tests_$TAG.log 2>&1
rc1=$?
tail -15 gpurun_out/cfg_tests_$TAG.log
# a fault / abort / timeout ends the call here
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then exit $rc1; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json
rc2=$?
[ $rc2 -ne 0 ] && tail -20 gpurun_out/bench_$TAG.err
exit $(( rc1 > rc2 ? rc1 : rc2 ))
