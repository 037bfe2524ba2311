"""Per-launch HBM traffic from rocprofv3 --pmc CSVs (tools/pmc_traffic.sh): FETCH_SIZE / WRITE_SIZE are KiB per
dispatch; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md
§HBM), so read bytes = 2 x FETCH_SIZE x 1024.  Prints {"cross_attn": bytes_per_launch, ...} as JSON."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = {}
for cname in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(root, cname, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(float)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != cname:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals[cname] = (sum(per.values()) / max(len(per), 1), len(per))
fetch, n = vals["FETCH_SIZE"]
write, _ = vals["WRITE_SIZE"]
out = {"cross_attn": round((2.0 * fetch + write) * 1024.0), "cross_attn_detail": {
    "dispatches": n, "fetch_size_kib": round(fetch, 1), "write_size_kib": round(write, 1),
    "read_bytes": round(2.0 * fetch * 1024.0), "write_bytes": round(write * 1024.0),
    "correction": "read = 2 x FETCH_SIZE (gfx950 half-count on 16-B/lane streaming reads)"}}
print(json.dumps(out))

# per kernel (when the regex selected several): mean bytes per dispatch, dispatch count, and the mean counter-reported
# dispatch duration, keyed by the kernel name without its argument list
per_k = defaultdict(lambda: {"n": 0, "fetch": 0.0, "write": 0.0})
for cname in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(root, cname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != cname:
                continue
            k = r["Kernel_Name"].split("(")[0]
            if cname == "FETCH_SIZE":
                per_k[k]["n"] += 1
                per_k[k]["fetch"] += float(r["Counter_Value"])
            else:
                per_k[k]["write"] += float(r["Counter_Value"])
if len(per_k) > 1:
    out["per_kernel"] = {k: {"dispatches": v["n"], "read_bytes": round(2.0 * v["fetch"] / max(v["n"], 1) * 1024.0),
                             "write_bytes": round(v["write"] / max(v["n"], 1) * 1024.0)} for k, v in sorted(per_k.items())}
    print(json.dumps(out))
