#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh output directory into profiles/<tag>.md (+ copies of the CSVs) and
record the step kernel's per-dispatch HBM traffic in profiles/traffic.json for bench.py.

HBM traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KB units x 1024): the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of wide coalesced reads).

The rocprofv3 --stats average mixes the bench's warmup launch and its timed launch (the same kernel with
fewer steps), so the summary also lists every dispatch of the step kernel from the kernel trace; the
timed launch is the last one, and its duration is what bench.py's HIP events measure (avg_launch_ms).
usage: summarize_prof.py <gpurun_out/prof_tag> <tag>"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
STEP_KERNELS = ("mcmc::lpc_", "mcmc::lpp_", "mcmc::wpc_", "mcmc::glm_rwm", "mcmc::glm_mala", "mcmc::glm_hmc", "mcmc::glm_ram")


def rows(kind, name):
    p = os.path.join(src, kind, name)
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


def counters(kind):
    agg = defaultdict(lambda: [0.0, 0])
    per = defaultdict(list)                     # kernel -> per-dispatch values in dispatch order
    for r in sorted(rows(kind, "run_counter_collection.csv"), key=lambda r: int(r["Dispatch_Id"])):
        a = agg[r["Kernel_Name"]]
        a[0] += float(r["Counter_Value"])
        a[1] += 1
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024)
    return agg, per


def bench_line(kind):
    p = os.path.join(src, f"{kind}.log")
    if not os.path.exists(p):
        return None
    for ln in reversed(open(p).read().splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
(fetch, fetch_per), (write, write_per) = counters("fetch"), counters("write")
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

# per-dispatch view of the step kernel (kernel trace + the two PMC passes, matched by dispatch order)
trace = sorted(rows("trace", "run_kernel_trace.csv"), key=lambda r: int(r["Dispatch_Id"]))
step = [r for r in trace if any(k in r["Kernel_Name"] for k in STEP_KERNELS) and "_eval" not in r["Kernel_Name"]]
bl = bench_line("trace")
entry = None
if step:
    kname = step[-1]["Kernel_Name"]
    disp = [r for r in step if r["Kernel_Name"] == kname]
    fp, wp = fetch_per.get(kname, []), write_per.get(kname, [])
    lines += ["", f"## step kernel dispatches: `{kname}`", "",
              "| # | dispatch | duration us | HBM read GB (2x FETCH_SIZE) | HBM write GB | traffic GB/s |",
              "|---|---|---|---|---|---|"]
    per = []
    for i, r in enumerate(disp):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        rd = 2 * fp[i] if i < len(fp) else None
        wr = wp[i] if i < len(wp) else None
        bw = (rd + wr) / (dur * 1e-6) / 1e9 if rd is not None and wr is not None else float("nan")
        per.append({"duration_us": dur, "read_bytes": rd, "write_bytes": wr})
        lines.append(f"| {i} | {r['Dispatch_Id']} | {dur:.1f} | {rd / 1e9 if rd is not None else float('nan'):.4f} | "
                     f"{wr / 1e9 if wr is not None else float('nan'):.4f} | {bw:.1f} |")
    # the timed launches are the last `launches` dispatches (the ones before them are the bench's warmup);
    # traffic and duration are their per-launch means
    nt = max(1, int((bl or {}).get("roofline", {}).get("launches", 1)))
    tl = per[-nt:]
    mean = lambda k: (sum(t[k] for t in tl) / len(tl)) if all(t[k] is not None for t in tl) else None
    timed = {k: mean(k) for k in ("duration_us", "read_bytes", "write_bytes")}
    lines += ["", f"The timed launches are the last {nt} dispatch(es) (the ones before are the bench's warmup); "
                  "the figures below are their per-launch means."]
    if bl is not None:
        roof = bl.get("roofline", {})
        lines.append(f"bench.py in the traced run: avg_launch_ms = {roof.get('avg_launch_ms', float('nan')):.3f} "
                     f"(HIP events) vs {timed['duration_us'] / 1e3:.3f} ms per timed dispatch in the trace; "
                     f"value = {bl['value']:.4g} {bl['unit']}.")
        key = bl.get("config", {}).get("key")
        if key and timed["read_bytes"] is not None and timed["write_bytes"] is not None:
            entry = {"kernel": kname, "source": f"profiles/{tag}.md", "launches_timed": roof.get("launches", 1),
                     "duration_us": timed["duration_us"], "read_bytes": timed["read_bytes"],
                     "write_bytes": timed["write_bytes"],
                     "traffic_bytes": timed["read_bytes"] + timed["write_bytes"]}
open(os.path.join(dst, f"{tag}.md"), "w").write("\n".join(lines) + "\n")
if entry is not None:
    tp = os.path.join(dst, "traffic.json")
    tj = json.load(open(tp)) if os.path.exists(tp) else {}
    tj[bl["config"]["key"]] = entry
    json.dump(tj, open(tp, "w"), indent=1, sort_keys=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
if trace:
    with open(os.path.join(dst, f"{tag}_kernel_trace.csv"), "w", newline="") as fh:
        wr_ = csv.writer(fh)
        wr_.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Duration_us"])
        for r in trace:
            if "mcmc::" in r["Kernel_Name"]:
                wr_.writerow([r["Dispatch_Id"], r["Kernel_Name"], r["Start_Timestamp"], r["End_Timestamp"],
                              f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3:.1f}"])
for kind in ("fetch", "write"):
    p = os.path.join(src, kind, "run_counter_collection.csv")
    if os.path.exists(p):
        rs = [r for r in csv.DictReader(open(p)) if "mcmc::" in r["Kernel_Name"]]
        with open(os.path.join(dst, f"{tag}_{kind}.csv"), "w", newline="") as fh:
            wr_ = csv.writer(fh)
            wr_.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "VGPR_Count", "SGPR_Count"])
            for r in rs:
                wr_.writerow([r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"],
                              r["VGPR_Count"], r["SGPR_Count"]])
print("\n".join(lines))
