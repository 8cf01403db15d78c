import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mcmc.jl_amd"), os.path.join(ROOT, "tests")]
import mcmchip as mc
import oracle_ref as orc
from test_gpu_parity import _glm_model, GLM_SAMPLERS
for rep in range(2):
    for kind in ("logistic", "linear"):
        m = _glm_model(kind, 3)
        r = mc.SerialMC(steps=2)
        ch = mc.run((m * GLM_SAMPLERS["rwm"]() * r).batch(40, seed=7))
        oc = orc.OracleChains(m, GLM_SAMPLERS["rwm"](), nchains=40, seed=7)
        s, g, a = oc.run(r)
        print("REP", rep, kind, "bits differ", int(np.count_nonzero(ch.diagnostics["accept"].T != a.astype(bool))),
              "orc x0", s[:, :, 0], flush=True)
