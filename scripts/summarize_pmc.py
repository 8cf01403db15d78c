#!/usr/bin/env python3
"""Aggregate a scripts/gpu_pmc.sh directory: per kernel, every counter summed over dispatches and dimensions."""
import collections
import csv
import glob
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
ndisp = collections.defaultdict(set)
for f in sorted(glob.glob(src + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ndisp[k].add((f, r.get("Dispatch_Id", "")))
for k, v in agg.items():
    print(f"## {k[:100]}")
    for c, x in sorted(v.items()):
        print(f"  {c:32s} {x:.4g}")
