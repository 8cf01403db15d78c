#!/usr/bin/env python3
"""Dev: PMC counters of one kernel's dispatches in a rocprofv3 --pmc run directory (run_counter_collection.csv +
run_kernel_trace.csv), with the derived clock, VALU busy and wait fractions.
usage: pmc_kernel.py <dir> <kernel substring> [dispatch index, default last]"""
import collections
import csv
import sys

d, pat = sys.argv[1], sys.argv[2]
idx = int(sys.argv[3]) if len(sys.argv) > 3 else -1
agg = collections.defaultdict(float)
for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
    if pat in r["Kernel_Name"]:
        agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
ds = sorted(set(k[0] for k in agg))
di = ds[idx]
v = {c: x for (dd, c), x in agg.items() if dd == di}
dur = None
for r in csv.DictReader(open(d + "/run_kernel_trace.csv")):
    if int(r["Dispatch_Id"]) == di:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        print(r["Kernel_Name"][:80], "dispatch", di, "of", len(ds), "dur_ms %.4f" % (dur * 1e3), "vgpr", r["VGPR_Count"],
              "agpr", r.get("Accum_VGPR_Count"), "lds", r["LDS_Block_Size"])
for c, x in sorted(v.items()):
    print("  %-28s %.5g" % (c, x))
if "GRBM_GUI_ACTIVE" in v and dur:
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print("  clock_GHz %.3f" % (cyc / dur / 1e9))
    if "SQ_ACTIVE_INST_VALU" in v:
        print("  valu_busy (4 x ACTIVE_INST_VALU / (1024 SIMDs x cycles)) %.3f" % (4 * v["SQ_ACTIVE_INST_VALU"] / (1024 * cyc)))
if "SQ_WAVES" in v:
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_INSTS_VMEM_RD"):
        if c in v:
            print("  %s per wave %.1f" % (c, v[c] / v["SQ_WAVES"]))
if "SQ_WAVE_CYCLES" in v:
    for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in v:
            print("  %s / SQ_WAVE_CYCLES %.3f" % (c, v[c] / v["SQ_WAVE_CYCLES"]))
