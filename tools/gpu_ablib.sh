# same-box A/B of library variants: bench.py with VLOG_AMD_LIB=<each .so given in LIBS>, in order
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
i=0
for L in $LIBS; do
  i=$((i+1))
  VLOG_AMD_LIB=$L timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['stages_s_per_step'], round(d['kernels_one_step']['cross_attn']['ms'],1))" gpurun_out/ab_$i.json $L
done
