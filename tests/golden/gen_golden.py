#!/usr/bin/env python3
"""Generate the committed golden chain fixtures tests/golden/chains_*.npz (test infrastructure).

Each fixture is one small SerialMC run -- model inputs, sampler, runner, seed, chain count -- and what the
oracle (oracle/oracle.c, the C restatement of RWM.jl / MALA.jl / HMC.jl / HMCDA.jl / RAM.jl and
SerialMC.jl:37-85) produced for it: kept samples [nkept][d][C], kept gradients, accept flags and the
per-chain evaluation counts.  The reference itself cannot run here (Julia 0.2, no toolchain),
so these vectors are the build's own: they pin the oracle against regressions (tests/test_golden.py,
CPU) and let the GPU tests check the HIP path against data that does not need the oracle at run time.

The cases are defined in CASES below (tests/test_golden.py reads the same table).  Regenerate with
    python tests/golden/gen_golden.py
after an intentional change of the arithmetic contract, and say so in the commit.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "mcmc.jl_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import mcmchip as mc  # noqa: E402


def _glm_data(kind, d, n):
    """Deterministic small regression data (no RNG: a fixed trigonometric design)."""
    i = np.arange(n)[:, None]
    j = np.arange(1, d)[None, :]
    X = np.hstack([np.ones((n, 1)), np.sin(0.7 * i * j + 0.3 * j)])
    beta0 = 0.4 * np.cos(np.arange(d))
    eta = X @ beta0
    if kind == "logistic":
        Y = (np.cos(1.3 * np.arange(n)) * 0.5 + 0.5 < 1 / (1 + np.exp(-eta))).astype(float)
    else:
        Y = eta + 0.5 * np.sin(2.1 * np.arange(n))
    return X, Y


def make_model(spec):
    kind, d = spec["model"], spec["d"]
    if kind == "readme":             # README.md:60 mymodel1 = model(v-> -dot(v,v), init=ones(3)); no model scale,
        return mc.model(mc.IsoNormalDot(), init=np.ones(d))    # so RWM runs its uniform-scale kernel instance
    if kind == "iso":
        return mc.model(mc.IsoNormalDot(), init=np.linspace(0.5, 1.5, d), grad=True,
                        scale=np.linspace(0.8, 1.2, d))
    if kind == "normal":
        return mc.model(mc.NormalDSL(0.3, 1.7), v=np.linspace(-1, 1, d), gradient=True)
    if kind == "abs":
        return mc.model(mc.AbsNormalDSL(1.0, 0.7), x=np.linspace(-1, 1, d), gradient=True)
    if kind == "gamma":
        return mc.model(mc.DistDSL("Gamma", 2.0, 1.5), v=np.linspace(0.5, 2.0, d), gradient=True)
    X, Y = _glm_data(kind, d, spec["n"])
    if kind == "logistic":
        return mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)
    return mc.model(mc.LinearRegression(X, Y, prior_sigma=1.0, noise_sigma=1.0), vars=np.zeros(d), gradient=True)


SAMPLERS = {
    "rwm": lambda glm: mc.RWM(0.05 if glm else 0.6),
    "rwm01": lambda glm: mc.RWM(0.1),                     # README.md:85 and every BASELINE RWM config
    "mala": lambda glm: mc.MALA(0.002 if glm else 0.4),
    "mala_tuned": lambda glm: mc.MALA(0.01 if glm else 2.0, mc.EmpMCTuner(0.6, adaptStep=3 if glm else 7)),
    "hmc": lambda glm: mc.HMC(3, 0.02) if glm else mc.HMC(4, 0.3),
    "hmc_tuned": lambda glm: (mc.HMC(2, 0.05, mc.EmpMCTuner(0.7, adaptStep=3, maxStep=6)) if glm
                              else mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9))),
    "hmcda": lambda glm: mc.HMCDA(len=0.1 if glm else 0.8),
    "ram": lambda glm: mc.RAM(1.0, 0.3 if glm else 0.234),
    "ram_wide": lambda glm: mc.RAM(0.15, 0.234),            # 33 <= d <= 256: two chains per wave
}

# (name, model spec, sampler, runner (steps, burnin, thinning), chains, seed)
CASES = []
for _s in ("rwm", "mala", "mala_tuned", "hmc", "hmc_tuned", "hmcda", "ram"):
    CASES.append((f"iso3_{_s}", dict(model="iso", d=3), _s, (40, 5, 3), 8, 101))
    CASES.append((f"normal3_{_s}", dict(model="normal", d=3), _s, (40, 5, 3), 8, 102))
    CASES.append((f"logistic5_{_s}", dict(model="logistic", d=5, n=20), _s, (30, 3, 3), 8, 103))
    CASES.append((f"linear5_{_s}", dict(model="linear", d=5, n=20), _s, (30, 3, 3), 8, 104))
for _s in ("rwm", "mala", "hmc", "hmcda"):
    CASES.append((f"iso40_{_s}", dict(model="iso", d=40), _s, (30, 3, 3), 4, 105))     # wave-per-chain
    CASES.append((f"abs2_{_s}", dict(model="abs", d=2), _s, (40, 5, 3), 8, 106))
    CASES.append((f"gamma3_{_s}", dict(model="gamma", d=3), _s, (40, 5, 3), 8, 107))
# HMCDA adapts its step only while i < burnin (HMCDA.jl:133): give it a burnin to adapt over
CASES = [(n, sp, s, (r[0], 15, r[2]) if s == "hmcda" else r, C, sd) for n, sp, s, r, C, sd in CASES]
CASES.append(("iso32_rwm", dict(model="iso", d=32), "rwm", (40, 5, 3), 64, 108))          # metric shape, small
CASES.append(("iso40_ram", dict(model="iso", d=40), "ram_wide", (30, 3, 3), 5, 109))   # two chains per wave, a dead half
CASES.append(("gamma200_ram", dict(model="gamma", d=200), "ram_wide", (12, 2, 2), 3, 110))   # two slot groups per lane
# the exact configurations the benchmarks run (uniform scale: the kernel instances bench.py dispatches),
# at small chain counts that are not multiples of 64
CASES.append(("readme_rwm", dict(model="readme", d=3), "rwm01", (1000, 100, 1), 1, 1))   # config 1: README.md:60,85
CASES.append(("readme3_c2_rwm", dict(model="readme", d=3), "rwm01", (100, 10, 10), 200, 1))    # config 2's kernel
CASES.append(("metric32_rwm", dict(model="readme", d=32), "rwm01", (100, 10, 10), 200, 1))     # the metric's kernel
CASES.append(("readme_c37_rwm", dict(model="readme", d=3), "rwm01", (300, 30, 7), 37, 3))      # look-ahead kernel


def case_sampler(spec, sname):
    return SAMPLERS[sname](spec["model"] in ("logistic", "linear"))


def order_for(spec):
    """None: the library's own summation order for the model / sampler (oracle_ref.kernel_order): lane per chain
    for d <= 16, two lanes per chain for 16 < d <= 32 (RAM: lane per chain), wave per chain beyond; regression
    kernels have their own fixed order (the oracle picks it from the model)."""
    return None


def fixture_path(name):
    return os.path.join(HERE, f"chains_{name}.npz")


def oracle_run(spec, sname, runner, C, seed):
    import oracle_ref as orc
    m = make_model(spec)
    oc = orc.OracleChains(m, case_sampler(spec, sname), nchains=C, seed=seed, order=order_for(spec))
    r = mc.SerialMC(steps=runner[0], burnin=runner[1], thinning=runner[2])
    s, g, acc = oc.run(r, nthreads=1)
    return s, g, acc.astype(np.uint8), oc.n_evals.copy()


def main():
    import oracle_ref as orc
    orc.build()
    for name, spec, sname, runner, C, seed in CASES:
        s, g, acc, ev = oracle_run(spec, sname, runner, C, seed)
        out = dict(samples=s, accept=acc, evals=ev)
        if g is not None:
            out["gradients"] = g
        np.savez_compressed(fixture_path(name), **out)
        print(f"{name}: samples {s.shape}, accept rate {acc.mean():.3f}")


if __name__ == "__main__":
    main()
