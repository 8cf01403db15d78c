"""Dev: repeated GLM RWM/MALA runs on GPU vs oracle; prints mismatch counts per case."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mcmc.jl_amd"), os.path.join(ROOT, "tests")]
import mcmchip as mc
import oracle_ref as orc
from test_gpu_parity import _glm_model, GLM_SAMPLERS
print("lib", mc._lib.LIB_PATH, flush=True)
ref = {}
for rep in range(int(os.environ.get("REPS", "4"))):
    line = []
    for sname in ("rwm", "mala", "hmc"):
        for kind in ("logistic", "linear"):
            for d in (3, 16, 37):
                m = _glm_model(kind, d)
                r = mc.SerialMC(steps=6)
                ch = mc.run((m * GLM_SAMPLERS[sname]() * r).batch(40, seed=7))
                key = (sname, kind, d)
                if key not in ref:
                    oc = orc.OracleChains(m, GLM_SAMPLERS[sname](), nchains=40, seed=7)
                    ref[key] = oc.run(r)
                s, g, a = ref[key]
                nb = int(np.count_nonzero(ch.diagnostics["accept"].T != a.astype(bool)))
                ns = int(np.count_nonzero(ch._samples != s))
                line.append(f"{sname[0]}{kind[1]}{d}:{nb}/{ns}")
    print(rep, " ".join(line), flush=True)
