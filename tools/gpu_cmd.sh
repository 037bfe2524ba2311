set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export VLOG_AMD_PARITY_OUT=$PWD/gpurun_out/parity_r6_suite.jsonl VLOG_AMD_PROGRESS=$PWD/gpurun_out/progress_r6_suite.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 600 --timeout-method thread --deselect tests/test_gpu_gates.py --ignore tests/test_gpu_gates.py --ignore tests/test_gpu_logprobs.py > gpurun_out/gpu_tests_r06_a2.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r06_a2.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r06_a2.log | head -30; exit $rc; }
t0=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r06_a.json 2> gpurun_out/bench_r06_a.err || { tail -30 gpurun_out/bench_r06_a.err; exit 1; }
t1=$(date +%s.%N)
echo "{\"cmd\": \"python3 bench.py --gpus 1 --steps 20 --warmup 5\", \"wall_s\": $(python3 -c "print(round($t1-$t0,1))")}" > gpurun_out/bench_r06_a_wall.json
cat gpurun_out/bench_r06_a_wall.json; python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_a.json')); print(d['value'], d['ms_per_step'], d['config']['workload'], d['roofline']['frac'], d['roofline'].get('traffic_source','')[:60], d['variable'].get('value'))"
