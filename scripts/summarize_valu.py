#!/usr/bin/env python3
"""VALU roofline of a step kernel from a scripts/gpu_pmc.sh directory (one rocprofv3 --pmc pass per p<i>/).

For the step kernel's timed dispatch (the last dispatch of that kernel: bench.py runs its warmup launch
first; profile with --no-ess so no later launch of the same kernel follows) it reads every counter of every
pass and derives:
  - valu_busy = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES: the fraction of CU-busy time the CU's four VALUs
    were issuing.  SQ_ACTIVE_INST_VALU counts quad-cycles per wave (MI355X_MICROARCH.md: SQ_ACTIVE_INST_*
    count quad-cycles) summed over the CU's waves, i.e. 4 x ACTIVE_INST_VALU VALU-cycles over 4 SIMDs; in
    the profiles SQ_BUSY_CU_CYCLES counts plain cycles summed over CUs (it equals CUs x the dispatch
    duration x the clock that GRBM_GUI_ACTIVE / duration gives), so the ratio needs no further factor.
    This is rocprof's VALUBusy with the dispatch's own busy cycles in place of GRBM_GUI_ACTIVE.
  - the instruction mix per 64 chain-steps (a lane-per-chain wave-step) and the quad-cycles per VALU instruction.
  - clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration.
Writes profiles/<tag>.md and records the per-chain-step figures in profiles/valu.json for bench.py
(keyed by kernel name: the per-chain-step VALU quad-cycles do not depend on the step count).
usage: summarize_valu.py <gpurun_out/pmc_tag> <tag> <kernel substring>"""
import csv
import glob
import json
import os
import sys

src, tag, pat = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
seen, kname, dur, bl = {}, None, None, None      # counter -> its value in every pass that collected it
for d in sorted(glob.glob(os.path.join(src, "p*/"))):
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))) if pat in r["Kernel_Name"]]
    if not rows:
        continue
    # the timed launches are the kernel's full-grid dispatches (a few-chain reference run of the same instance may
    # follow them): the last dispatch of the largest grid
    gmax = max(int(r["Grid_Size"]) for r in rows)
    rows = [r for r in rows if int(r["Grid_Size"]) == gmax]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            seen.setdefault(r["Counter_Name"], {}).setdefault(d, 0.0)
            seen[r["Counter_Name"]][d] += float(r["Counter_Value"])
            kname = r["Kernel_Name"]
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    logp = d.rstrip("/") + ".log"
    if bl is None and os.path.exists(logp):
        for ln in open(logp):
            if ln.startswith("{"):
                bl = json.loads(ln)
vals = {c: sum(pv.values()) / len(pv) for c, pv in seen.items()}   # a counter in several passes: their mean
if kname is None:
    sys.exit(f"no dispatch of a kernel matching {pat!r} in {src}")
units = bl["roofline"]["units_per_launch"]                  # chain-steps of one launch
waves = bl["config"]["chains_per_gpu"] / 64.0
steps = units / bl["config"]["chains_per_gpu"]
v = vals
busy = v["SQ_ACTIVE_INST_VALU"] / v["SQ_BUSY_CU_CYCLES"]
clock = v["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9
cu_cycles = v["SQ_BUSY_CU_CYCLES"] / 256
entry = {
    "kernel": kname, "source": f"profiles/{tag}.md", "workload_key": bl["config"]["key"],
    "duration_s": dur, "clock_ghz": clock,
    "valu_busy": busy,
    "valu_quadcycles_per_chain_step": v["SQ_ACTIVE_INST_VALU"] / units,
    "valu_insts_per_wave_step": v["SQ_INSTS_VALU"] / waves / steps,
    "quadcycles_per_valu_inst": v["SQ_ACTIVE_INST_VALU"] / v["SQ_INSTS_VALU"],
    "dual_issue_frac": v.get("SQ_ACTIVE_INST_VALU2", 0.0) / v["SQ_ACTIVE_INST_VALU"],
    "busy_cycles_per_cu": cu_cycles,
}
L = [f"# VALU roofline: {tag}", "", f"kernel: `{kname}`", f"workload: `{bl['config']['key']}`", "",
     f"timed dispatch: {dur * 1e3:.3f} ms; clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) {clock:.2f} GHz; "
     f"CU busy {cu_cycles:.4g} cycles per CU ({cu_cycles / (dur * clock * 1e9):.3f} of the dispatch)", "",
     f"- **VALU busy = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES = {busy:.3f}**",
     f"- VALU instructions per 64 chain-steps (one wave-step of a lane-per-chain kernel): {entry['valu_insts_per_wave_step']:.1f}; "
     f"quad-cycles per VALU instruction: {entry['quadcycles_per_valu_inst']:.3f}; "
     f"dual-issue quad-cycles (SQ_ACTIVE_INST_VALU2) / SQ_ACTIVE_INST_VALU: {entry['dual_issue_frac']:.4f}", "",
     "| counter | timed dispatch | per 64 chain-steps |", "|---|---|---|"]
for c in sorted(v):
    L.append(f"| {c} | {v[c]:.6g} | {v[c] / waves / steps:.2f} |")
open(os.path.join(root, "profiles", f"{tag}.md"), "w").write("\n".join(L) + "\n")
sys.path.insert(0, root)
from bench import kernel_src_hash  # noqa: E402
entry["src_hash"] = kernel_src_hash(entry.get("kernel", ""))   # the sources it measured (bench.py ignores others)
p = os.path.join(root, "profiles", "valu.json")
tj = json.load(open(p)) if os.path.exists(p) else {}
tj[f"{kname}|{entry['workload_key']}"] = entry        # one entry per kernel and workload
json.dump(tj, open(p, "w"), indent=1, sort_keys=True)
print("\n".join(L))
