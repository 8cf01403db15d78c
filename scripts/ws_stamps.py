#!/usr/bin/env python3
"""Phase timing of glm_mala1ws's tile loop (dev tool; a GLM_WS_STAMP build of glm_mala1.hip, glm.hip WS_STAMP).

Build:  hipcc ... -mllvm -amdgpu-mfma-vgpr-form -DGLM_WS_STAMP -c csrc/kernels/glm_mala1.hip -o build_ab/glm_mala1_stamp.o
        and link it with the other objects into mcmchip/ab/libmcmc_hip_wsstamp.so
Run:    MCMCHIP_LIB=mcmc.jl_amd/mcmchip/ab/libmcmc_hip_wsstamp.so python3 scripts/ws_stamps.py
Config 3's workload (logistic n = 1000, d = 128, MALA(0.001), 262 144 chains), two steps; prints, for the M waves
(MFMA) and the V waves (elementwise), the median shader cycles of each phase of a 16-observation tile over
workgroups 0..3, their waves and tiles 8..23 of the last launch:
  M: eta (eta_{t+1} MFMAs + its LDS store), g (G_{t-1} MFMAs issued), bar (barrier wait), tile
  V: stage (tile t+2 to LDS, t+3 loads issued), terms (eta_t read, the logistic terms), rstore, bar, tile"""
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

C = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
X, Y = bench.regression_data("logistic", 1000, 128)
m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(128), gradient=True)
t = (m * mc.MALA(0.001) * mc.SerialMC(steps=2, burnin=0)).batch(C, seed=1)
mc.run(t)
lib = _lib.load()
buf = np.zeros((4, 8, 16, 8), dtype=np.uint32)
fn = lib.mcmc_debug_ws_stamps
fn.argtypes = [ct.c_void_p]
assert fn(buf.ctypes.data) == 0
b64 = buf.astype(np.int64)
ph = np.diff(b64, axis=-1) % (1 << 32)                      # [wg][wave][tile][7]
tile = (b64[:, :, 1:, 0] - b64[:, :, :-1, 0]) % (1 << 32)  # loop top to loop top
M, V = slice(0, 4), slice(4, 8)
out = {"M": {nm: float(np.median(ph[:, M, :, i])) for i, nm in enumerate(["eta", "g", "bar"])},
       "V": {nm: float(np.median(ph[:, V, :, i])) for i, nm in enumerate(["stage", "terms", "rstore", "bar"])}}
out["M"]["tile"] = float(np.median(tile[:, M]))
out["V"]["tile"] = float(np.median(tile[:, V]))
out["M"]["bar_p90"] = float(np.percentile(ph[:, M, :, 2], 90))
out["V"]["bar_p90"] = float(np.percentile(ph[:, V, :, 3], 90))
out["chains"] = C
# the workgroup's phases outside the tile loop (per wave: start, proposal barrier, bx / tile-2 barrier, eta_0 barrier,
# loop end, final barrier, end (M waves only))
if hasattr(lib, "mcmc_debug_ws_wg"):
    wg = np.zeros((4, 8, 8), dtype=np.uint32)
    lib.mcmc_debug_ws_wg.argtypes = [ct.c_void_p]
    assert lib.mcmc_debug_ws_wg(wg.ctypes.data) == 0
    w64 = wg.astype(np.int64)
    dd = np.diff(w64, axis=-1) % (1 << 32)
    names = ["proposal", "bx_tile2", "eta0", "loop", "final_bar", "finish"]
    out["wg_M"] = {nm: float(np.median(dd[:, 0:4, i])) for i, nm in enumerate(names)}
    out["wg_V"] = {nm: float(np.median(dd[:, 4:8, i])) for i, nm in enumerate(names[:5])}
    out["wg_M"]["total"] = float(np.median((w64[:, 0:4, 6] - w64[:, 0:4, 0]) % (1 << 32)))
    w2 = np.zeros((4, 8, 8), dtype=np.uint32)
    lib.mcmc_debug_ws_wg2.argtypes = [ct.c_void_p]
    assert lib.mcmc_debug_ws_wg2(w2.ctypes.data) == 0
    w2 = w2.astype(np.int64)
    st = w64[:, :, 0]
    out["prop_V"] = {"normals": float(np.median((w2[:, 4:8, 0] - st[:, 4:8]) % (1 << 32))), "M_normals": float(np.median((w2[:, 0:4, 0] - st[:, 0:4]) % (1 << 32))),
                     "qf_sum": float(np.median((w2[:, 4:8, 1] - w2[:, 4:8, 0]) % (1 << 32))),
                     "table": float(np.median((w2[:, 4:8, 2] - w2[:, 4:8, 1]) % (1 << 32)))}
    fin0 = w64[:, 0:4, 5]                                     # M: the final barrier passed
    out["finish_M"] = {"llacc": float(np.median((w2[:, 0:4, 3] - fin0) % (1 << 32))),
                       "qb": float(np.median((w2[:, 0:4, 4] - w2[:, 0:4, 3]) % (1 << 32))),
                       "accept": float(np.median((w2[:, 0:4, 5] - w2[:, 0:4, 4]) % (1 << 32))),
                       "stores": float(np.median((w2[:, 0:4, 6] - w2[:, 0:4, 5]) % (1 << 32))),
                       "rest": float(np.median((w64[:, 0:4, 6] - w2[:, 0:4, 6]) % (1 << 32)))}
    out["prop_M"] = {"tile0": float(np.median((w2[:, 0:4, 0] - st[:, 0:4]) % (1 << 32))),
                     "tile1": float(np.median((w2[:, 0:4, 1] - w2[:, 0:4, 0]) % (1 << 32)))}
print(json.dumps(out))
