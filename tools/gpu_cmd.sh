set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_big_rows.py > gpurun_out/tests_r6_c.log 2>&1 || { tail -30 gpurun_out/tests_r6_c.log; exit 1; }
tail -3 gpurun_out/tests_r6_c.log
for arm in 0 512 0 512; do
  VLOG_AMD_DEC_BIG128=$arm timeout -k 10 300 python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/c5_big128_$arm.json 2> gpurun_out/c5_big128_$arm.err || { tail -20 gpurun_out/c5_big128_$arm.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/c5_big128_$arm.json')); k=d.get('kernels_one_step',{})
print('$arm', d['value'], d['ms_per_step'], d['config']['token_crc32'], {n: k[n]['ms'] for n in ('dec_gemm','cross_attn','self_attn') if n in k})" | tee -a gpurun_out/ab_r06_c5_big128.txt
done
