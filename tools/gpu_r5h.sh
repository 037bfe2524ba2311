set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
C5="python3 bench.py --beam 5 --word-timestamps --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for lib in abtmp/lib_r4.so abtmp/lib_prefold.so vlog_amd/libwhisper_mi355.so; do
  VLOG_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 600 $C5 > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -20 gpurun_out/c5ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c5ab.json')); k=d['kernels_one_step']
print('$lib', d['value'], d['ms_per_step'], d['config']['token_crc32'], {n: k[n]['ms'] for n in ('dec_gemm','self_attn','cross_attn')})" | tee -a gpurun_out/c5_libs_ab.txt
done
