set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/bench_r05_c5.json 2> gpurun_out/bench_r05_c5.err || { tail -20 gpurun_out/bench_r05_c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r05_c5.json')); k=d['kernels_one_step']
print('c5', d['value'], d['ms_per_step'], d['config']['token_crc32'], d['stages_s_per_step'])
print({n: (v['ms'], v['launches']) for n, v in k.items()})"
timeout -k 10 600 python3 tools/bench_worker_call.py --minutes-seq 2 --minutes-tp 10 > gpurun_out/worker_r05_f.json 2> gpurun_out/worker_r05_f.err || { tail -20 gpurun_out/worker_r05_f.err; exit 1; }
cat gpurun_out/worker_r05_f.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_gemv.py tests/test_gpu_words.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
