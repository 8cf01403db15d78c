#!/usr/bin/env python3
"""Phase timing of the d-sliced regression tile loop (dev tool; a GLM_STAMP build, glm.hip GLM_STAMPT).

Build:  make -C mcmc.jl_amd OBJDIR=build_stamp OUT=mcmchip/libmcmc_hip_stamp.so \
            FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -DGLM_STAMP"
Run:    MCMCHIP_LIB=mcmc.jl_amd/mcmchip/libmcmc_hip_stamp.so python3 scripts/glm_stamps.py [d] [n] [chains]
Prints, per phase of a 16-observation tile, the median shader cycles over workgroups 0..3, waves and tiles 8..23
of the last evaluation: eta (loop top -> partial stored), b1 (barrier 1), elem (-> weights stored), b2, g (G
MFMAs issued), dma (vmcnt(0) on the next tile), b3, and the whole tile."""
import ctypes as ct
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mcmc.jl_amd"))
sys.path.insert(0, ROOT)
import mcmchip as mc  # noqa: E402
from mcmchip import _lib  # noqa: E402
import bench  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 512
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
C = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
X, Y = bench.regression_data("linear", n, d)
m = mc.model(mc.LinearRegression(X, Y), vars=np.zeros(d), gradient=True)
t = (m * mc.HMC(5, 0.001) * mc.SerialMC(steps=2, burnin=0)).batch(C, seed=1)
mc.run(t)
lib = _lib.load()
buf = np.zeros((4, 8, 16, 8), dtype=np.uint32)
fn = lib.mcmc_debug_glm_stamps
fn.argtypes = [ct.c_void_p]
assert fn(buf.ctypes.data) == 0
b64 = buf.astype(np.int64)
ph = np.diff(b64, axis=-1) % (1 << 32)                      # [wg][wave][tile][7]
tile = (b64[:, :, 1:, 0] - b64[:, :, :-1, 0]) % (1 << 32)
names = ["eta", "b1", "elem", "b2", "g", "dma", "b3"]
out = {nm: float(np.median(ph[..., i])) for i, nm in enumerate(names)}
out["tile"] = float(np.median(tile))
out["per_wave_median"] = {nm: [float(np.median(ph[:, w, :, i])) for w in range(8)] for i, nm in enumerate(names)}
out["workload"] = {"d": d, "n": n, "chains": C, "kernel": t.step_kernel}
print(json.dumps(out))
