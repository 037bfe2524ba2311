# PMC passes on the encoder GEMM (gemm_8p_kernel, tools/gemm_bench shapes): L2 hit rate and the SQ wait /
# issue split (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES), one pass each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/gpmc
i=0
for C in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex gemm_8p_kernel --output-format csv -d $R/gpurun_out/gpmc/p$i -o run -- $R/tools/gemm_bench 3 > $R/gpurun_out/gpmc/p$i.log 2>&1 || { tail -20 $R/gpurun_out/gpmc/p$i.log; exit 1; }
done
ls -R $R/gpurun_out/gpmc | head -20
