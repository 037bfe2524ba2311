#!/usr/bin/env python3
"""Compact view of a rocprofv3 kernel_stats.csv: total ms, calls, average us per kernel (name shortened)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in rows[:n]:
    name = r["Name"].split("(")[0].replace("void ", "")[:60]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):7d} x {float(r['AverageNs'])/1e3:8.2f} us  "
          f"{100*float(r['TotalDurationNs'])/tot:5.1f}%  {name}")
print(f"total {tot/1e6:.1f} ms")
