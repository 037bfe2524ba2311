# L2-side counters of the decoder chain and the cross-attention (one rocprofv3 --pmc pass, every counter within
# one block's limits: TCP 1, TCC 2): TCP_TCC_READ_REQ_sum = read requests from the CUs' L1s to L2 (the L2 -> CU
# traffic the activation re-reads cost), TCC_HIT_sum / TCC_MISS_sum = the L2 hit rate.  Calibration: the factored
# cross-attention (xattn_kernel) reads each byte of its encoder output once (PMC FETCH_SIZE ≈ algorithmic), so its
# requests per algorithmic byte give the request size for this access width.  Run via gpurun.
set -o pipefail
R=$GRAFT_REPO_ROOT
KREGEX=${KREGEX:-"dec_ring_kernel|xq_kernel|xcomb_vo_kernel|resid_ln_reduce_kernel|self_attn_wave_kernel|xattn_kernel"}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_l2
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KREGEX" \
  --output-format csv -d $R/gpurun_out/pmc_l2/run -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-profile \
  --no-cpu-baseline --no-parity --no-variable > $R/gpurun_out/pmc_l2/run.log 2>&1 || { tail -20 $R/gpurun_out/pmc_l2/run.log; exit 1; }
python3 - "$R/gpurun_out/pmc_l2" <<'PY'
import csv, glob, json, os, sys
from collections import defaultdict
root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
out = {}
for k, c in sorted(acc.items()):
    d = max(len(n[k]), 1)
    hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    out[k] = {"dispatches": d, "tcp_tcc_read_req": round(c.get("TCP_TCC_READ_REQ_sum", 0.0) / d),
              "l2_hit_rate": round(hit / max(hit + miss, 1.0), 4)}
print(json.dumps(out))
PY
