# Worker-call evidence on one box: decode parity tests, the unchanged worker's call (tools/bench_worker_call.py,
# sequential beam 5 + VAD on 2 min, throughput mode on 30 min) and a short bench.py line (headline unchanged?)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-w}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_gemv.py tests/test_gpu_split.py tests/test_gpu_decode.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 600 python tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_$TAG.json 2> gpurun_out/worker_$TAG.err || { tail -20 gpurun_out/worker_$TAG.err; exit 1; }
cat gpurun_out/worker_$TAG.json
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-profile --no-cpu-baseline --no-parity > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
head -c 700 gpurun_out/bench_$TAG.json
