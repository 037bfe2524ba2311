# Builder-run side lines on the final tree: config 5 (beam 5 + batched word timestamps) and the opt-in fp8 cross memory.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --beam 5 --word-timestamps --no-cpu-baseline --no-parity > gpurun_out/cfg5_i.json 2> gpurun_out/cfg5_i.err || { tail -20 gpurun_out/cfg5_i.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/cfg5_i.json')); print('cfg5', d['value'], d['stages_s_per_step'])"
timeout -k 10 300 python bench.py --cross-fp8 --no-cpu-baseline > gpurun_out/fp8_i.json 2> gpurun_out/fp8_i.err || { tail -20 gpurun_out/fp8_i.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/fp8_i.json')); print('fp8', d['value'], d['roofline']['avg_launch_us'], d.get('parity',{}).get('windows_eps_consistent'))"
