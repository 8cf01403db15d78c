#!/usr/bin/env python3
"""Dev probe (GPU): the ESS kernel at the metric shape.  Samples the metric workload (2^20 chains, d=32, RWM(0.1),
SerialMC(1000, 100, 10)) into device buffers, times mcmc_stats_ess over them with HIP events (REPS times), and
prints the Geyer stopping-pair distribution of a host subset (how many lag pairs a series needs; the max over
groups of 16 and 64 series is what a wave that shares rounds pays)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mcmc.jl_amd"))
import mcmchip as mc  # noqa: E402
from mcmchip import _lib  # noqa: E402
import ctypes as ct  # noqa: E402

C = int(os.environ.get("CHAINS", 1 << 20))
d = 32
reps = int(os.environ.get("REPS", "5"))
m = mc.model(mc.IsoNormalDot(), init=np.ones(d))
r = mc.SerialMC(steps=1000, burnin=100, thinning=10)
task = mc.MCMCTask(m, mc.RWM(0.1), r, nchains=C, seed=2, device=0)
h = task.handle()
lib = _lib.load()
nk = len(r.r)
dev = torch.device("cuda", 0)
samples = torch.empty((nk, d, C), dtype=torch.float64, device=dev)
out = _lib.Outputs()
out.samples = samples.data_ptr()
out.on_device = 1
_lib.check(lib.mcmc_chains_reserve_outputs(h, nk, 1))
cfg = r.cfg()
_lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(out)))
torch.cuda.synchronize()
print("sampled", nk, "kept", flush=True)
ess = mc.stats.ess_device(samples, "imse")
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ess = mc.stats.ess_device(samples, "imse")
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
gb = samples.numel() * 8 / 1e9
print(f"ess_ms {min(ts):.3f} (all {['%.3f' % t for t in ts]}) GB {gb:.2f} -> {gb / min(ts):.2f} TB/s", flush=True)
# stopping pairs of a host subset
sub = samples[:, :, :4096].cpu().numpy()          # [n, d, 4096]
x = np.transpose(sub, (2, 0, 1))                   # [C, n, d]
n = x.shape[1]
acv = mc.stats.autocov(x, n - 1)
k = (n - 2) // 2
g = acv[:, 0:2 * k + 2:2] + acv[:, 1:2 * k + 2:2]
nonpos = g <= 0
mstop = np.where(nonpos.any(axis=1), nonpos.argmax(axis=1), k + 1)   # [C, d]
flat = mstop.T.reshape(-1)                          # series in (param, chain) order, as the kernel tiles them
print("stop pair: mean %.2f pcts(50,90,99,max) %s" % (flat.mean(), np.percentile(flat, [50, 90, 99, 100])))
for gsz in (16, 32, 64):
    gm = flat[: len(flat) // gsz * gsz].reshape(-1, gsz).max(axis=1)
    print(f"  max over groups of {gsz}: mean {gm.mean():.2f}  (lag FMAs per series vs need: {gm.mean() / flat.mean():.2f}x)")
print("ess mean", float(torch.nan_to_num(ess).mean()), flush=True)
