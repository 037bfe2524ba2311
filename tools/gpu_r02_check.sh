# bench.py A/B of the host poll interval of the decode loop (steps between live-count syncs)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
i=0
for c in 8 4 2 1 8 4 2; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --check-every $c > gpurun_out/chk_$i.json 2> gpurun_out/chk_$i.err || { tail -20 gpurun_out/chk_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print('check_every', sys.argv[2], d['value'], d['ms_per_step'], d['config']['decoder_steps'], d['stages_s_per_step'])" gpurun_out/chk_$i.json $c
done
