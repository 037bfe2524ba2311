# sweep env knobs over the bench (one gpurun call): CONFIGS="A=1,B=2 A=0" (space-separated, comma-joined vars)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1 || { tail -30 gpurun_out/sweep_tests.log; exit 1; }; tail -2 gpurun_out/sweep_tests.log; fi
for c in $CONFIGS; do
  envs=$(echo $c | tr ',' ' ')
  env $envs timeout -k 10 400 python bench.py --no-cpu-baseline --steps ${STEPS:-1} > gpurun_out/sweep_$c.json 2> gpurun_out/sweep_$c.err || { tail -20 gpurun_out/sweep_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/sweep_$c.json')); k=d.get('kernels_one_step',{})
print('$c', d['value'], 'decode', d['stages_s_per_step']['decode'], 'cross', k.get('cross_attn',{}).get('ms'), 'gemm', k.get('dec_gemm',{}).get('ms'))"
done
