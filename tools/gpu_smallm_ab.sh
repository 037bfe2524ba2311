# small-M decoder GEMM routing A/B on the sequential worker call (beam 5 = 5 rows), engine event profiler
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ALLSK="decode_gemm.qkv=-1,decode_gemm.out=-1,decode_gemm.cq=-1,decode_gemm.cout=-1,decode_gemm.fc1=-1,decode_gemm.fc2=-1"
ALLOS="decode_gemm.qkv=-2,decode_gemm.out=-2,decode_gemm.cq=-2,decode_gemm.cout=-2,decode_gemm.fc1=-2,decode_gemm.fc2=-2"
for cfg in "" "decode_gemm_plan=0" "$ALLSK" "$ALLOS" ""; do
  timeout -k 10 300 python tools/prof_worker_seq.py large-v3 "$cfg" >> gpurun_out/smallm.jsonl 2>> gpurun_out/smallm.err || { tail -20 gpurun_out/smallm.err; exit 1; }
  tail -1 gpurun_out/smallm.jsonl | head -c 700; echo
done
