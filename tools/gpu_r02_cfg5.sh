# Config 5 (beam 5 + batched word timestamps, 150 windows = 750 decoder rows) on the current defaults vs the
# pre-round-2-session-2 decoder plan (fc1 all-rows ring / fc2 skinny), alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-cfg5}
i=0
for kv in BASE=1 VLOG_AMD_DEC_GEMM=fc1=0,fc2=-1:VLOG_AMD_DEC_COLS=fc1=32,fc2=32 BASE=1 VLOG_AMD_DEC_GEMM=fc1=0,fc2=-1:VLOG_AMD_DEC_COLS=fc1=32,fc2=32; do
  i=$((i+1))
  env ${kv//:/ } timeout -k 10 400 python bench.py --beam 5 --word-timestamps --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
