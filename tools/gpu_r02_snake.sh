# Infinity Cache reuse probe for the factored cross-attention: microbenchmark (alternating launches in opposite
# item orders vs one order), then bench.py A/B of the layer-alternating order and the load policy, then the
# hipBLASLt ceiling on the encoder GEMM shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-snake}
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ring_columns or forms" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -12 gpurun_out/${TAG}_t.log; [ $rc -ne 0 ] && exit $rc
for s in 0 1 0 1; do XB_SNAKE=$s XB_ABL=0 XB_F8=0 timeout -k 10 60 ./tools/xattn_bench 150 3 2 >> gpurun_out/${TAG}_micro.txt 2>&1 || exit 1; done
cat gpurun_out/${TAG}_micro.txt
for g in 0 4 8 0 4 8; do echo "GROUP=$g"; VLOG_AMD_GEMM_GROUP=$g timeout -k 10 120 ./tools/gemm_bench 10 2>&1 | head -5; done > gpurun_out/${TAG}_gemm.txt || exit 1; cat gpurun_out/${TAG}_gemm.txt
GEMM_ABL=1 timeout -k 10 120 ./tools/gemm_bench 10 > gpurun_out/${TAG}_gemm_abl.txt 2>&1 || exit 1; grep abl= gpurun_out/${TAG}_gemm_abl.txt
timeout -k 10 150 ./tools/dec_gemm_bench 200 150 > gpurun_out/${TAG}_dec.txt 2>&1 || exit 1; grep -E "RING|launch_gemm" gpurun_out/${TAG}_dec.txt
i=0
for kv in "BASE=1" "VLOG_AMD_XSNAKE=1" "VLOG_AMD_DEC_COLS=fc1=64:VLOG_AMD_DEC_GEMM=fc1=64" "VLOG_AMD_GEMM_GROUP=4" "VLOG_AMD_GEMM_GROUP=8" "VLOG_AMD_XSNAKE=1:VLOG_AMD_XABL=8" "BASE=1" "VLOG_AMD_XSNAKE=1" "VLOG_AMD_DEC_COLS=fc1=64:VLOG_AMD_DEC_GEMM=fc1=64" "VLOG_AMD_GEMM_GROUP=4"; do
  i=$((i+1))
  env ${kv//:/ } timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_one_step']; print(sys.argv[2], d['value'], d['config']['token_crc32'], {n: round(k[n]['ms'],1) for n in k})" gpurun_out/${TAG}_$i.json "$kv"
done
timeout -k 10 200 python tools/blas_probe.py > gpurun_out/${TAG}_blas.txt 2>&1; cat gpurun_out/${TAG}_blas.txt
