# HBM traffic of the bench's dominant kernel (default: the factored cross-attention xattn_kernel) from PMC
# counters, two separate passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass), each under its own
# time limit.  Run via gpurun.  KREGEX selects the kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
KREGEX=${KREGEX:-xattn_kernel}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex $KREGEX --output-format csv \
    -d $R/gpurun_out/pmc/$C -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-profile --no-cpu-baseline --no-parity $BENCH_ARGS \
    > $R/gpurun_out/pmc/$C.log 2>&1 || { tail -20 $R/gpurun_out/pmc/$C.log; exit 1; }
done
python3 $R/tools/traffic_summary.py $R/gpurun_out/pmc > $R/gpurun_out/pmc/traffic.json && cat $R/gpurun_out/pmc/traffic.json
