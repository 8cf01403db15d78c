#!/usr/bin/env python3
"""fp64-datapath roofline of a regression step kernel from a scripts/gpu_pmc.sh directory (dev tool).

On a CDNA4 SIMD the fp64 MFMAs and the fp64 VALU instructions share one datapath (a partner
wave's fp64 FMAs slow 3-4x while MFMAs run), so the bound of the logistic / linear kernels is their combined fp64
work against the one fp64 rate, not the MFMA flops alone.  For the kernel's timed dispatch (the last dispatch
of the kernel; profile with --no-ess) it reads every pass and derives, per log-target+gradient evaluation (the
bench line in the pass's log gives the evaluations of the timed launch):
  - mfma_flop   = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (MOPS count 512-flop units, MI355X_MICROARCH.md),
                  checked against 4 n d (the algorithmic count);
  - valu_flop   = 64 x SQ_INSTS_VALU_FLOPS_FP64 (+ _TRANS): the counter is per wave instruction (FMA = 2, MUL /
                  ADD = 1: it equals 2 FMA_F64 + MUL_F64 + ADD_F64 + TRANS_F64), so x 64 lanes;
  - combined    = (mfma_flop + valu_flop) / duration against the 78.6 TF fp64 spec.
Writes profiles/<tag>.md and records the per-evaluation figures in profiles/fp64.json (keyed by kernel name and
workload key) for bench.py.
usage: summarize_fp64.py <gpurun_out/pmc_tag> <tag> <kernel substring>"""
import csv
import glob
import json
import os
import sys

src, tag, pat = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F64_PEAK = 78.6

vals, kname, dur, evals, wkey = {}, None, None, None, None
for pdir in sorted(glob.glob(os.path.join(src, "p*/"))):
    rows = []
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    if not rows:
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) != last:
            continue
        kname = r["Kernel_Name"]
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    log = pdir.rstrip("/") + ".log"
    if os.path.exists(log) and evals is None:
        for ln in open(log):
            if ln.startswith("{") and '"roofline"' in ln:
                d = json.loads(ln)
                evals = d["roofline"]["evals_per_launch"]
                dur = d["roofline"]["avg_launch_ms"] * 1e-3
                flop_per_eval = d["roofline"]["flop_per_eval"]
                wkey = d["config"]["key"]
assert kname and evals, "no dispatch / bench line found"
mfma = vals.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
valu = 64.0 * (vals.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0) + vals.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0))
clock = vals.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / dur / 1e9
comb = (mfma + valu) / dur / 1e12
sys.path.insert(0, root)
from bench import glm_src_hash  # noqa: E402

out = {
    "kernel": kname, "workload_key": wkey, "source": f"profiles/{tag}.md", "src_hash": glm_src_hash(),
    "evals_per_launch": evals, "duration_s": dur, "clock_ghz": clock,
    "mfma_flop_per_eval": mfma / evals, "algorithmic_flop_per_eval": flop_per_eval,
    "valu_fp64_flop_per_eval": valu / evals,
    "fp64_insts_per_eval": {k: vals.get(k, 0.0) / evals for k in
                            ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                             "SQ_INSTS_VALU_TRANS_F64")},
    "combined_tfs": comb, "combined_frac": comb / F64_PEAK,
    "mfma_only_frac": mfma / dur / 1e12 / F64_PEAK,
    # SQ_VALU_MFMA_BUSY_CYCLES sums the CU's four SIMDs (64 cycles per f64 MFMA), SQ_BUSY_CU_CYCLES counts CU cycles
    "mfma_busy": vals.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, 4.0 * vals.get("SQ_BUSY_CU_CYCLES", 1.0)),
}
lines = [f"# fp64 datapath roofline: {tag}", "", f"kernel: `{kname}`", f"workload: `{wkey}`", "",
         f"timed dispatch {dur * 1e3:.3f} ms at {clock:.2f} GHz; {evals:.4g} log-target+gradient evaluations",
         "",
         f"- MFMA flop per evaluation {out['mfma_flop_per_eval']:.4g} (algorithmic 4 n d = {flop_per_eval:.4g})",
         f"- VALU fp64 flop per evaluation {out['valu_fp64_flop_per_eval']:.4g} "
         f"({out['valu_fp64_flop_per_eval'] / max(1.0, out['mfma_flop_per_eval']):.2f} of the MFMA flops)",
         f"- MFMA alone {out['mfma_only_frac']:.3f} of 78.6 TF; **MFMA + VALU fp64 {comb:.1f} TF = "
         f"{out['combined_frac']:.3f} of the shared fp64 rate**",
         f"- MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES) = {out['mfma_busy']:.3f}", "",
         "| counter | timed dispatch | per evaluation |", "|---|---|---|"]
for k in sorted(vals):
    lines.append(f"| {k} | {vals[k]:.6g} | {vals[k] / evals:.4g} |")
open(os.path.join(root, "profiles", tag + ".md"), "w").write("\n".join(lines) + "\n")
jp = os.path.join(root, "profiles", "fp64.json")
db = json.load(open(jp)) if os.path.exists(jp) else {}
db[f"{kname}|{wkey}"] = out
json.dump(db, open(jp, "w"), indent=1, sort_keys=True)
print("\n".join(lines[:12]))
