set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
summ() { python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; v=d.get('variable') or {}
kv=v.get('kernels_one_step',{})
print(d['value'], d['config']['token_crc32'], 'xattn', k['cross_attn']['ms'], 'frac', d['roofline']['frac'], '| var', v.get('value'), v.get('token_crc32'), 'xattn', kv.get('cross_attn',{}).get('ms'), 'frac', (v.get('roofline') or {}).get('frac'))"; }
for L in old new old new; do
  echo "== $L"; VLOG_AMD_LIB=$PWD/abtmp/$L.so timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-parity --variable-steps 4 2>&1 | tail -1 | summ || exit 1
done 2>&1 | tee gpurun_out/ab_xcd_interleave.txt
for L in old new; do
  echo "== c5var $L"; VLOG_AMD_LIB=$PWD/abtmp/$L.so timeout -k 10 400 python3 bench.py --beam 5 --word-timestamps --workload variable --steps 3 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], 'cross', k['cross_attn']['ms'], d['stages_s_per_step'])" || exit 1
done 2>&1 | tee -a gpurun_out/ab_xcd_interleave.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_split.py tests/test_gpu_words.py tests/test_gpu_gates.py 2>&1 | tee gpurun_out/t_r5p.txt | tail -4
