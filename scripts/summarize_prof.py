#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh output directory into profiles/<tag>.md (+ copies of the CSVs).

HBM traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KB units x 1024): the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of wide coalesced reads;
calibrated here against the known state bytes of lpc_rwm: see DESIGN.md §7)."""
import csv
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)


def counters(kind):
    p = os.path.join(src, kind, "run_counter_collection.csv")
    agg = defaultdict(lambda: [0.0, 0])
    if not os.path.exists(p):
        return agg
    for r in csv.DictReader(open(p)):
        a = agg[r["Kernel_Name"]]
        a[0] += float(r["Counter_Value"])
        a[1] += 1
    return agg


stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
fetch, write = counters("fetch"), counters("write")
lines = [f"# rocprofv3 summary: {tag}", "", f"command: see {tag}.cmd", "",
         "| kernel | calls | avg us | total ms | % | HBM read GB/dispatch (2x FETCH_SIZE) | HBM write GB/dispatch | "
         "achieved GB/s (traffic / avg) |", "|---|---|---|---|---|---|---|---|"]
for r in stats:
    name = r["Name"]
    calls = int(r["Calls"])
    avg = float(r["AverageNs"])
    f = fetch.get(name)
    w = write.get(name)
    rd = 2 * f[0] * 1024 / f[1] / 1e9 if f else float("nan")
    wr = w[0] * 1024 / w[1] / 1e9 if w else float("nan")
    bw = (rd + wr) / (avg * 1e-9) if f and w else float("nan")
    lines.append(f"| `{name[:90]}` | {calls} | {avg / 1e3:.1f} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                 f"{float(r['Percentage']):.2f} | {rd:.4f} | {wr:.4f} | {bw:.1f} |")
open(os.path.join(dst, f"{tag}.md"), "w").write("\n".join(lines) + "\n")
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
for kind in ("fetch", "write"):
    p = os.path.join(src, kind, "run_counter_collection.csv")
    if os.path.exists(p):
        rows = [r for r in csv.DictReader(open(p)) if "mcmc::" in r["Kernel_Name"]]
        with open(os.path.join(dst, f"{tag}_{kind}.csv"), "w", newline="") as fh:
            wr_ = csv.writer(fh)
            wr_.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "VGPR_Count", "SGPR_Count"])
            for r in rows:
                wr_.writerow([r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"],
                              r["VGPR_Count"], r["SGPR_Count"]])
print("\n".join(lines))
