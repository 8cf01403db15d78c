#!/usr/bin/env python3
"""Throughput benchmark of the many-chain MCMC inner loop (BASELINE.json metric).

Default workload (BASELINE.json "metric"): d = 32 iso-Normal target -dot(v,v),
RWM(0.1), init ones(32), SerialMC(steps=1000, burnin=100, thinning=10), 2^20
chains per GPU, seed 1, fp64.  A "step" is one MCMC step of every chain (one
pass of the hot path over the chain batch).  The timed region is one
run_serialmc call of `--steps` steps with kept samples, gradients and accept
bits written to device-resident outputs; chain state and model data are in
HBM before the clock starts.

Other BASELINE.json configs (--config): readme (config 1), d3 (config 2),
logistic128 (config 3), hmc1024 (config 4, per-GPU shard), linear512
(config 5, per-GPU shard); binomial is the reference's own published benchmark
unit (benchmarks/benchunits/binomial.jl: logistic n=1000, d=10, RWM(0.1), 100
steps), printed beside its benchlog.csv numbers.

  python bench.py [--config metric] [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU; weak scaling:
                                                      every rank runs the per-GPU chain count)
Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mcmc.jl_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F64_MFMA_PEAK_TFS = 78.6       # MI355X spec, dense fp64 matrix (not in the guide; measured in DESIGN.md §7)
VALU_PEAK_TCYC = 1024 * 2.4e9 / 1e12   # VALU issue: 256 CUs x 4 SIMDs, one instruction-cycle each, at 2.4 GHz

# BASELINE.json configs.  chains are per GPU; steps/warmup are the defaults when not given.
CONFIGS = {
    "metric": dict(model="iso", d=32, chains=1 << 20, sampler="rwm", steps=1000, warmup=100, thinning=10,
                   desc="d=32 iso-Normal, RWM(0.1), 2^20 chains/GPU (BASELINE metric)"),
    "readme": dict(model="iso", d=3, chains=1, sampler="rwm", steps=1000, warmup=100, thinning=1,
                   desc="config 1: d=3 iso-Normal, RWM(0.1), SerialMC(1000,100), 1 chain"),
    "d3": dict(model="iso", d=3, chains=1 << 20, sampler="rwm", steps=1000, warmup=100, thinning=10,
               desc="config 2: d=3 iso-Normal, RWM(0.1), 1,048,576 chains"),
    "logistic128": dict(model="logistic", d=128, n=1000, chains=262144, sampler="mala", steps=200, warmup=10,
                        thinning=10, desc="config 3: logistic regression n=1000 d=128, MALA(0.001), "
                                          "262,144 chains"),
    "hmc1024": dict(model="iso", d=1024, chains=524288 // 8, sampler="hmc", steps=1000, warmup=100,
                    thinning=20, desc="config 4: d=1024 iso-Normal, HMC(10, 0.1), 524,288 chains over 8 GPUs "
                                       "(65,536/GPU)"),
    "linear512": dict(model="linear", d=512, n=4096, chains=65536 // 8, sampler="hmcda", steps=20, warmup=100,
                      thinning=1, adapt=True,
                      desc="config 5: linear regression n=4096 d=512, HMCDA(), 65,536 chains over 8 GPUs (8,192/GPU); "
                           "the configured burnin (100 steps of dual averaging, HMCDA.jl:133-138) runs untimed as the "
                           "warmup, then the timed steps run at each chain's adapted dualLeapStep: a step is "
                           "round(len/eps) leapfrogs of that chain (HMCDA.jl:104)"),
    # round 5: the widened regression sizes (not BASELINE configs)
    "linear1024": dict(model="linear", d=1024, n=4096, chains=65536 // 8, sampler="hmcda", steps=4, warmup=30,
                       thinning=1, adapt=True,
                       desc="linear regression n=4096 d=1024 (config 5 at twice its width: eight 128-coordinate "
                            "slices a chain tile), HMCDA(), 8,192 chains; 30 untimed dual-averaging steps, then the "
                            "timed steps at each chain's adapted step"),
    "ramlinear128": dict(model="linear", d=128, n=1000, chains=1 << 15, sampler="ram", steps=40, warmup=10,
                         thinning=10, desc="RAM(1., 0.3) on linear regression n=1000 d=128, 32,768 chains (the "
                                           "split step: regression eval kernel + wave-per-chain factor update)"),
    # the reference's own published benchmark unit (benchmarks/benchunits/binomial.jl:1-25, benchlog.csv:350-352)
    "binomial": dict(model="logistic", d=10, n=1000, chains=1 << 18, sampler="rwm", steps=100, warmup=10,
                     thinning=1, desc="benchmarks/benchunits/binomial.jl: logistic regression n=1000 d=10, "
                                      "RWM(0.1), 100 steps (the reference's published unit, run batched)"),
    # the reference's second published benchmark unit (benchmarks/benchunits/bare_distribs.jl:7-27,
    # benchlog.csv:298-300): y = x * v; y ~ Normal(1, 1) over v = ones(1000), scalar x from the mean, RWM(0.1)
    "bare_normal": dict(model="distobs", dist=("Normal", 1.0, 1.0), d=1, chains=1 << 20, sampler="rwm", steps=100,
                        warmup=10, thinning=1, desc="benchmarks/benchunits/bare_distribs.jl: y = x * v; "
                                                    "y ~ Normal(1, 1), v = ones(1000), RWM(0.1), 100 steps (the "
                                                    "reference's published unit, run batched)"),
    # the adaptive RAM sampler (not a BASELINE config)
    "ram32": dict(model="iso", d=32, chains=1 << 18, sampler="ram", steps=200, warmup=20, thinning=10,
                  desc="RAM(1., 0.234) on d=32 iso-Normal, 262,144 chains (a 32x32 jump factor per chain)"),
    "ram256": dict(model="iso", d=256, chains=1 << 16, sampler="ram", steps=100, warmup=10, thinning=10,
                   desc="RAM(1., 0.234) on d=256 iso-Normal, 65,536 chains (wave per chain, a 256x256 jump factor "
                        "per chain)"),
    "ramlinear": dict(model="linear", d=10, n=1000, chains=1 << 16, sampler="ram", steps=200, warmup=20,
                      thinning=10, desc="examples/linear_regression.jl:28: RAM(1., 0.3), n=1000 d=10, "
                                        "65,536 chains"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="metric", choices=list(CONFIGS))
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--d", type=int, default=None)
    p.add_argument("--chains", type=int, default=None, help="chains per GPU")
    p.add_argument("--sampler", default=None, choices=["rwm", "mala", "hmc", "hmcda", "ram"])
    p.add_argument("--thinning", type=int, default=None)
    p.add_argument("--spl", type=int, default=-1, help="steps per launch (0: whole run in one launch; "
                                                       "-1: default of the library)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-ess", action="store_true", help="skip the ESS/sec leg")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--strong", action="store_true", help="fixed total chains (--chains) split over ranks")
    p.add_argument("--pcie", action="store_true", help="also time one run with host output buffers (kept samples "
                                                       "cross PCIe after the loop); reported apart, never `value`")
    return p.parse_args()


def regression_data(kind, n, d, key=0x5EED):
    """X = [1 | N(0,1)], beta0 ~ N(0,1); Y Bernoulli(logistic(X beta0)) or
    X beta0 + N(0,1).  Drawn from numpy's Philox4x32-10 on its own key (not the chains' stream)."""
    g = np.random.Generator(np.random.Philox(key=key))
    X = np.hstack([np.ones((n, 1)), g.standard_normal((n, d - 1))])
    beta0 = g.standard_normal(d)
    eta = X @ beta0
    if kind == "logistic":
        Y = (g.random(n) < 1.0 / (1.0 + np.exp(-eta))).astype(np.float64)
    else:
        Y = eta + g.standard_normal(n)
    return X, Y


def build_model(mc, cfg, d):
    if cfg["model"] == "distobs":                    # bare_distribs.jl:8-16: start at the distribution's mean
        name, p1, p2 = cfg["dist"]
        return mc.model(mc.DistObsDSL(name, p1, p2, v=np.ones(1000)), x=p1, gradient=True)
    if cfg["model"] == "iso":
        return mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    X, Y = regression_data(cfg["model"], cfg["n"], d)
    if cfg["model"] == "logistic":
        return mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)
    return mc.model(mc.LinearRegression(X, Y), vars=np.zeros(d), gradient=True)


def build_sampler(mc, cfg, name):
    if cfg["model"] == "logistic" and name == "mala":
        return mc.MALA(0.001)                        # test/test_syntax.jl:28
    if name == "ram":
        return mc.RAM(1.0, 0.3) if cfg["model"] == "linear" else mc.RAM(1.0, 0.234)
    return {"rwm": lambda: mc.RWM(0.1), "mala": lambda: mc.MALA(0.1), "hmc": lambda: mc.HMC(10, 0.1),
            "hmcda": lambda: mc.HMCDA()}[name]()


def hbm_bytes_per_unit(d, sampler):
    """SURVEY.md §8(d) algorithmic bytes per chain-step (state round trip + 1 accept bit) and per kept
    chain-step (sample, + gradient for gradient samplers)."""
    per_step = (32 * d if sampler == "mala" else 16 * d) + 16 + 1 / 8
    if sampler == "ram":                 # + the jump factor S read and written back (d(d+1)/2 doubles)
        per_step += 8 * d * (d + 1)
    per_kept = 8 * d * (1 if sampler in ("rwm", "ram") else 2)
    return per_step, per_kept


def _norm_kernel(name):
    """'void mcmc::lpc_rwm<8, true, mcmc::IsoDot, true>(mcmc::KernelArgs)' -> 'lpc_rwm<8,true,IsoDot,true>'."""
    n = name.split("(")[0].replace("void ", "").replace("mcmc::", "").replace(" ", "")
    return n


def measured_traffic(wkey, kname):
    """HBM bytes per launch of the step kernel for this workload: 2 x FETCH_SIZE + WRITE_SIZE of the timed
    dispatch(es) in a committed rocprofv3 run of the same bench command (MI355X_MICROARCH.md §HBM correction),
    or None when no profile of this exact workload and this kernel instance is committed (a profile of another
    kernel for the same workload is stale and is not used)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    e = json.load(open(p)).get(wkey)
    if e is None or _norm_kernel(e["kernel"]) != _norm_kernel(kname):
        return None
    return {"bytes_per_launch": e["traffic_bytes"], "read_bytes": e["read_bytes"], "write_bytes": e["write_bytes"],
            "source": e["source"], "unit": "B"}


def step_kernel_src_hash():
    """sha256 over the sources the lane- and wave-per-chain step kernels are compiled from (csrc/*.hpp, the
    Box-Muller tables, kernels/lpc*, kernels/wpc*): a VALU profile recorded under another hash measured other code.
    ram.hpp / ram_wave.hpp (the RAM jump-factor templates and the wave-per-chain RAM body) and glm_layout.hpp (the
    regression X image) are left out: no RWM / MALA / HMC step kernel instantiates them."""
    import glob
    import hashlib
    base = os.path.join(ROOT, "mcmc.jl_amd", "csrc")
    skip = {"ram.hpp", "ram_wave.hpp", "glm_layout.hpp"}
    files = sorted([f for f in glob.glob(os.path.join(base, "*.hpp")) if os.path.basename(f) not in skip]
                   + glob.glob(os.path.join(base, "*.inc"))
                   + glob.glob(os.path.join(base, "kernels", "lpc*")) + glob.glob(os.path.join(base, "kernels", "wpc*"))
                   + [os.path.join(base, "kernels", "layout_api.hpp")])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, base).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def kernel_src_hash(kname):
    """The source hash a profile of this kernel instance is keyed by: the regression kernels (glm*) are built from
    glm_src_hash's sources, every other step kernel from step_kernel_src_hash's."""
    return glm_src_hash() if _norm_kernel(kname).startswith("glm") else step_kernel_src_hash()


def measured_valu(kname, wkey):
    """VALU issue cost of the step kernel per chain-step (SQ_ACTIVE_INST_VALU quad-cycles / chain-steps of the
    timed dispatch) and its measured VALU-busy fraction, from a committed rocprofv3 PMC run of this kernel
    instance, built from these sources, on this same workload (profiles/valu.json, written by
    scripts/summarize_valu.py), or None.  The workload must match: per-launch work (table staging, state load
    and store) is spread over the launch's steps, so a 20-step profile does not price a 1000-step run."""
    p = os.path.join(ROOT, "profiles", "valu.json")
    if not os.path.exists(p):
        return None
    h = kernel_src_hash(kname)
    for k, e in json.load(open(p)).items():
        if (_norm_kernel(e.get("kernel", k)) == _norm_kernel(kname) and e.get("src_hash") == h
                and e.get("workload_key") == wkey):
            return e
    return None


# The metric kernel's VALU floor ("VALU floor"): the lane-operations RWM(0.1) on the d = 32
# iso-Normal needs per chain-step, one instruction each, no moves, address or select overhead --
# Philox4x32-10: 8.5 blocks (32 normals + half an accept block) x 10 rounds x (2 v_mad_u64_u32 + 2 v_xor3) = 340;
# Box-Muller radius: 16 x (7 FMAs + conversion, residual, 3 index ops) = 192; angle: 16 x (conversion, index, 4 + 3
# polynomial FMAs, 2 products with the radius) = 176; proposal x + z*scale, two roundings (RWM.jl:59): 64;
# log-target -dot(v, v): 32 FMAs + pair combine + negate = 35; accept: 52-bit uniform, screened log, decision and
# the 16 64-bit moves of an accepted state = 40 -> 847 lane-operations = 13.23 wave instructions per chain-step.
VALU_FLOOR_METRIC = {"lane_ops_per_chain_step": {"philox": 340, "radius": 192, "angle": 176, "proposal": 64,
                                                 "log_target": 35, "accept": 40}}
VALU_FLOOR_METRIC["insts_per_chain_step"] = sum(VALU_FLOOR_METRIC["lane_ops_per_chain_step"].values()) / 64.0


def valu_floor(args, vm):
    """valu_floor / floor_frac of the metric workload (d = 32 iso-Normal RWM): the floor above against the measured
    VALU instructions per chain-step of the committed PMC profile (quad-cycles per chain-step / quad-cycles per
    instruction); None for other workloads."""
    if args.config != "metric" or args.sampler != "rwm" or args.d != 32:
        return None
    meas = vm["valu_quadcycles_per_chain_step"] / vm["quadcycles_per_valu_inst"]
    fl = VALU_FLOOR_METRIC["insts_per_chain_step"]
    return {"floor_insts_per_chain_step": fl, "measured_insts_per_chain_step": meas, "floor_frac": fl / meas,
            "lane_ops_per_chain_step": VALU_FLOOR_METRIC["lane_ops_per_chain_step"],
            "note": "floor = the arithmetic the RWM step needs at one lane-operation each (DESIGN.md §5.1b), / 64 "
                    "lanes; measured from the committed SQ_INSTS / SQ_ACTIVE_INST_VALU profile of this kernel"}


def glm_src_hash():
    """sha256 over the sources the regression step kernels are compiled from (csrc/*.hpp, the tables,
    kernels/glm*.hip): an fp64 profile recorded under another hash measured other code."""
    import glob
    import hashlib
    base = os.path.join(ROOT, "mcmc.jl_amd", "csrc")
    files = sorted(glob.glob(os.path.join(base, "*.hpp")) + glob.glob(os.path.join(base, "*.inc"))
                   + glob.glob(os.path.join(base, "kernels", "glm*.hip")))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, base).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def measured_fp64(kname, wkey):
    """The regression kernel's fp64 work per evaluation (MFMA flops and VALU fp64 flops) from a committed
    rocprofv3 PMC run of this kernel instance, these sources and this workload (profiles/fp64.json, written by
    scripts/summarize_fp64.py), or None.  fp64 MFMA and fp64 VALU share one datapath on CDNA4,
    so the combined rate is the bound the line reports beside the MFMA-only fraction."""
    p = os.path.join(ROOT, "profiles", "fp64.json")
    if not os.path.exists(p):
        return None
    h = glm_src_hash()

    def shape(key):                      # per-evaluation work does not depend on the step count or thinning
        return "|".join(f for f in (key or "").split("|") if not f.startswith(("steps=", "thinning=")))
    def kern(name):                      # the profile's glm_hmc<NM, NW, DA, REC> is the run's glm_hmc<NM, NW, DA>
        n = _norm_kernel(name)
        return n[:-len(",false>")] + ">" if n.startswith("glm_hmc<") and n.count(",") == 3 and n.endswith(",false>") else n
    for k, e in json.load(open(p)).items():
        if (kern(e.get("kernel", k)) == kern(kname) and e.get("src_hash") == h
                and shape(e.get("workload_key")) == shape(wkey)):
            return e
    return None


def host_cpus():
    """The host cores this process may use: its CPU affinity set, capped by the cgroup's CPU quota when one is
    set (a GPU box shows every CPU of the machine in nproc / os.cpu_count() but grants a share of them), plus
    the CPU model (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"usable": usable, "nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota, "model": model}


def cpu_baseline(model, sampler, seconds, C=4096, leaps_per_step=None):
    """The oracle (scalar C port of SerialMC + sampler, OpenMP over chains) on a bounded sample, on every host
    core this process may use (host_cpus); a one-chain workload (config 1) is timed as one chain on one core.
    leaps_per_step: an adaptive-trajectory sampler (HMCDA) whose cost per step depends on the adapted step size:
    the sample then runs without adaptation (burnin 0) and is converted from leapfrogs/s at the GPU run's
    measured leapfrogs per chain-step -- adapting on the host first would take minutes (config 5: ~300 leapfrogs
    of 8.4 Mflop per chain-step once adapted)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as orc
    import mcmchip as mc
    host = host_cpus()
    threads = max(1, min(host["usable"], C))
    # double the sample until one run takes about `seconds` / 2 (state set-up excluded); that last run is the
    # sample -- same runner shape (burnin = steps/10, thinning 10) at every size, so an adaptive sampler's
    # cost per step is measured as configured, and the wall time stays bounded (< ~2 x seconds in total)
    steps, dt = 1, 0.0
    while True:
        oc = orc.OracleChains(model, sampler, nchains=C, seed=1)
        burnin = 0 if leaps_per_step else steps // 10
        t0 = time.perf_counter()
        oc.run(mc.SerialMC(steps=steps, burnin=burnin, thinning=10 if steps >= 20 else 1), nthreads=threads)
        dt = time.perf_counter() - t0
        print(f"bench: cpu_baseline sample {C} chains x {steps} steps: {dt:.2f} s", file=sys.stderr, flush=True)
        if dt >= seconds / 2 or steps >= 1 << 25:
            break
        steps *= 2 if dt > seconds / 16 else 4
    if leaps_per_step:
        leaps = float(np.sum(oc.n_evals))
        return {"value": leaps / dt / leaps_per_step, "unit": "chain-steps/s", "cores": threads, "kind": "port",
                "host": host, "leapfrogs_per_s": leaps / dt, "leapfrogs_per_chain_step": leaps_per_step,
                "sample": f"{C} chains x {steps} steps on the host without adaptation ({leaps:.0f} leapfrogs, "
                          f"{dt:.1f} s), oracle/oracle.c OpenMP over {threads} threads; chain-steps/s = leapfrogs/s "
                          f"/ the GPU run's {leaps_per_step:.1f} leapfrogs per adapted chain-step"}
    return {"value": C * steps / dt, "unit": "chain-steps/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": f"{C} chains x {steps} steps of the same workload on the host ({dt:.1f} s), "
                      f"oracle/oracle.c OpenMP over {threads} threads (every usable core; chains are independent, "
                      f"so the rate is per chain-step)"}


BENCHLOG_REFERENCE = {
    "binomial": {"source": "benchmarks/benchlog.csv:350-352 (binomial 10x1000, CodeHash 276db306bb, Windows, "
                           "2 CPU cores, 2013-08-29)", "eval_ms": 0.25765, "evalallg_ms": 0.74805, "rwm100_ms": 25.690},
    "bare_normal": {"source": "benchmarks/benchlog.csv:298-300 (:(Normal(1,1)) on vector of 1000, CodeHash "
                              "276db306bb, Windows, 2 CPU cores, 2013-08-29)",
                    "eval_ms": 0.60083, "evalallg_ms": 0.64702, "rwm100_ms": 61.634},
}


def binomial_units(mc, model, C, local, config="binomial"):
    """The reference's benchmark unit benchmarks/benchunits/binomial.jl:21-27 on this build, for context beside
    benchlog.csv:350-352 (0.258 ms loglik eval, 0.748 ms loglik + gradient, 25.69 ms per 100 RWM steps of one
    chain; 2-core Windows CPU, 2013): the host API's batched model.eval / model.evalallg (mcmc_model_eval: host
    arrays in and out, PCIe included) over C parameter vectors and over one, and `run(m * RWM(0.1), steps=100)`
    of one chain (SerialMC(steps=100), every sample kept, returned to the host)."""
    import ctypes as ct
    from mcmchip import _lib
    lib = _lib.load()
    d = model.size
    mh = model._handle(local)
    out = {}
    for n in (1, C):
        x = np.ascontiguousarray(np.repeat(model.init[:, None], n, axis=1))
        lp = np.empty(n)
        g = np.empty((d, n))
        for name, gp in (("eval", None), ("evalallg", g)):
            gptr = gp.ctypes.data_as(ct.POINTER(ct.c_double)) if gp is not None else None
            args = (mh, n, x.ctypes.data_as(ct.POINTER(ct.c_double)), lp.ctypes.data_as(ct.POINTER(ct.c_double)), gptr)
            _lib.check(lib.mcmc_model_eval(*args))
            reps = 20 if n == 1 else 5
            t0 = time.perf_counter()
            for _ in range(reps):
                _lib.check(lib.mcmc_model_eval(*args))
            dt = (time.perf_counter() - t0) / reps
            out[f"{name}_{'1' if n == 1 else 'batch'}"] = {"points": n, "call_ms": dt * 1e3,
                                                            "us_per_point": dt * 1e6 / n}
    r = mc.SerialMC(steps=100)
    t1 = mc.MCMCTask(model, mc.RWM(0.1), r, nchains=1, seed=1, device=local)
    mc.run(t1)
    times = []
    for _ in range(10):                                   # benchmark(f3, "100 RWM steps", name, 10)
        t1.reset()
        t0 = time.perf_counter()
        mc.run(t1)
        times.append(time.perf_counter() - t0)
    out["rwm100_1chain_ms"] = {"avg": 1e3 * sum(times) / len(times), "min": 1e3 * min(times)}
    out["reference"] = dict(BENCHLOG_REFERENCE[config], note="context, not the target: one 2013 CPU core pair, "
                                                             "one chain")
    return out


class _heartbeat:
    """A progress line on stderr every 30 s while a long library call runs (ctypes releases the GIL), so a minutes-long
    warmup (config 5 at d = 1024) is not mistaken for a hang."""

    def __init__(self, what: str, every: float = 30.0):
        import threading
        self.what, self.every, self.stop = what, every, threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self.stop.wait(self.every):
            print(f"bench: {self.what} running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        return False


def spawn_workers(args, argv):
    """`--gpus N` (N > 1) started as a plain process (no torchrun, WORLD_SIZE unset): re-launch this same command
    under torch.distributed.run with N processes, one per GPU, and return its exit code.  Runs before anything
    touches the GPU, and starts the workers as a child process (never an exec)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_workers(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one process per GPU is required")
    # the contract is ONE JSON line on stdout: libraries that print to fd 1 (RCCL's version banner at
    # init_process_group, gloo's connection lines) are sent to stderr; the line goes to the saved stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch            # first: libmcmc_hip.so then binds to the HIP runtime torch already loaded
    # MCMC_BENCH_BACKEND=gloo: rehearse the multi-rank path on a 1-GPU box (ranks share cuda:0, host-side
    # reductions); the driver's N-GPU runs use the default, RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("MCMC_BENCH_BACKEND", "nccl")
    if world > 1 or "MASTER_ADDR" in os.environ:        # under torchrun: the process group even for N = 1
        import torch.distributed as dist
        if backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    red_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    import mcmchip as mc
    from mcmchip import _lib

    cfg0 = CONFIGS[args.config]
    for k in ("d", "chains", "sampler", "thinning", "steps", "warmup"):
        if getattr(args, k) is None:
            setattr(args, k, cfg0[k])
    d = args.d
    C = max(1, args.chains // world) if args.strong else args.chains
    model = build_model(mc, cfg0, d)
    sampler = build_sampler(mc, cfg0, args.sampler)
    K, W = args.steps, args.warmup
    burnin = K // 10
    runner = mc.SerialMC(steps=K, burnin=burnin, thinning=args.thinning)
    # HMCDA adapts its leapStep per chain during the burn-in (HMCDA.jl:133): config 5, and any --sampler hmcda run,
    # warm up through that adaptation, so the timed steps run at the adapted trajectory lengths
    adaptive = bool(cfg0.get("adapt")) or args.sampler == "hmcda"
    if adaptive and K // 10 >= W + 2:
        sys.exit("bench.py: the timed run's burnin would reach past the adaptation warmup")
    task = mc.MCMCTask(model, sampler, runner, nchains=C, seed=1, device=local, chain_offset=rank * C,
                       steps_per_launch=max(args.spl, 0))
    h = task.handle()
    lib = _lib.load()

    # device-resident outputs (caller-owned, as the C ABI's on_device mode)
    dev = torch.device("cuda", local)
    nkept = len(runner.r)
    samples = torch.empty((nkept, d, C), dtype=torch.float64, device=dev)
    grad_sampler = args.sampler not in ("rwm", "ram")
    grads = torch.empty((nkept, d, C), dtype=torch.float64, device=dev) if grad_sampler else None
    bits = torch.empty((nkept, (C + 63) // 64), dtype=torch.int64, device=dev)
    out = _lib.Outputs()
    out.samples = samples.data_ptr()
    out.gradients = grads.data_ptr() if grads is not None else None
    out.accept_bits = bits.data_ptr()
    out.on_device = 1

    # library-owned output staging sized before the clock starts (the timed run allocates nothing)
    _lib.check(lib.mcmc_chains_reserve_outputs(h, nkept, 0 if args.pcie else 1))
    adapt = None
    if W > 0:
        # adaptive configs (config 5, HMCDA): the warmup is the configured burnin, W steps of dual averaging
        # (HMCDA.jl:133: adapts while i < burnin); the timed run continues the same chains (runners.jl:14) past
        # it, so every timed step runs at the chain's dualLeapStep (HMCDA.jl:140)
        wr = (mc.SerialMC(steps=W + 1, burnin=W, thinning=1) if adaptive
              else mc.SerialMC(steps=W, burnin=0, thinning=1))
        wout = _lib.Outputs()
        cfg = wr.cfg()
        ta = time.perf_counter()
        print(f"bench: warmup {W} steps", file=sys.stderr, flush=True)   # progress on stderr (stdout: the line)
        with _heartbeat("warmup"):
            _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(wout)))
            torch.cuda.synchronize(dev)
        print(f"bench: warmup done in {time.perf_counter() - ta:.1f} s", file=sys.stderr, flush=True)
        if adaptive:
            eps = task.tuner_state()["step_bar"]
            adapt = {"warmup": f"SerialMC(steps={W + 1}, burnin={W}): {W - 1} dual-averaging updates, untimed",
                     "warmup_s": time.perf_counter() - ta, "warmup_evals": task.evals,
                     "eps_bar": {"median": float(np.median(eps)), "min": float(eps.min()), "max": float(eps.max())},
                     "leapfrogs_per_step_at_eps_bar": {"median": float(np.median(np.maximum(1, np.round(2.0 / eps)))),
                                                       "max": float(np.max(np.maximum(1, np.round(2.0 / eps))))}}
    torch.cuda.synchronize(dev)
    ev0 = task.evals
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    cfg = runner.cfg()
    hb = _heartbeat("timed run").__enter__()            # started before the clock: it only sleeps in between
    t0 = time.perf_counter()
    _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(out)))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    T = time.perf_counter() - t0
    hb.__exit__(None, None, None)
    print(f"bench: timed {K} steps in {T:.3f} s", file=sys.stderr, flush=True)
    kernel_ms = out.kernel_ms
    evals = task.evals - ev0
    if dist is not None:
        t = torch.tensor([T, kernel_ms], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        T, kernel_ms = float(t[0]), float(t[1])
    total_chains = C * world
    value = total_chains * K / T

    # ESS/sec: sum over chains of min over parameters of the IMSE ESS of the kept
    # samples, per second of sampling; computed on the device after the timed region, timed apart.  When the
    # timed run keeps fewer than 20 samples per chain (the IMSE/IPSE estimators need a usable number of lags;
    # e.g. --steps 20 keeps 2), a separate run of the configuration's own SerialMC (BASELINE: 1000 steps,
    # burnin 100, thinning 10) on fresh chains of the same workload is sampled and timed for it.
    ess_line = None
    if not args.no_ess:
        leg = "timed run"
        e_samples, e_T, e_nkept = samples, T, nkept
        es, eb, et = cfg0["steps"], cfg0["steps"] // 10, cfg0["thinning"]
        if nkept < 20 and len(mc.SerialMC(steps=es, burnin=eb, thinning=et).r) < 20:
            leg = f"none: neither the timed run ({nkept}) nor the configuration's SerialMC keeps 20 samples per chain"
            e_nkept = nkept
        elif nkept < 20:
            er = mc.SerialMC(steps=es, burnin=eb, thinning=et)
            e_nkept = len(er.r)
            etask = mc.MCMCTask(model, sampler, er, nchains=C, seed=2, device=local, chain_offset=rank * C,
                                steps_per_launch=max(args.spl, 0))
            e_samples = torch.empty((e_nkept, d, C), dtype=torch.float64, device=dev)
            e_grads = torch.empty((e_nkept, d, C), dtype=torch.float64, device=dev) if grad_sampler else None
            eout = _lib.Outputs()
            eout.samples = e_samples.data_ptr()
            eout.gradients = e_grads.data_ptr() if e_grads is not None else None
            eout.on_device = 1
            eh = etask.handle()
            _lib.check(lib.mcmc_chains_reserve_outputs(eh, e_nkept, 1))
            ecfg = er.cfg()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            _lib.check(lib.mcmc_run_serialmc(eh, ct.byref(ecfg), ct.byref(eout)))
            torch.cuda.synchronize(dev)
            e_T = time.perf_counter() - t0
            del e_grads
            leg = (f"separate run: SerialMC(steps={es}, burnin={eb}, thinning={et}) of the same workload, seed 2 "
                   f"(the timed run keeps {nkept} < 20 samples per chain)")
        if e_nkept >= 20:
            torch.cuda.synchronize(dev)
            te = time.perf_counter()
            ess = mc.stats.ess_device(e_samples, "imse")
            # a chain that never moved has a 0/0 ESS (var.jl gives NaN), and an antithetic series whose first
            # Geyer pair is <= 0 gets a negative IMSE variance (var.jl:53-57, m = 0): both count as 0 samples
            ess_min_sum = torch.nan_to_num(ess, nan=0.0).clamp(min=0.0).min(dim=0).values.sum()
            torch.cuda.synchronize(dev)
            ess_s = time.perf_counter() - te
            if dist is not None:
                esum = ess_min_sum.double().reshape(1).to(red_dev)
                tmax = torch.tensor([e_T], dtype=torch.float64, device=red_dev)
                dist.all_reduce(esum, op=dist.ReduceOp.SUM)
                dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
                ess_min_sum, e_T = esum[0], float(tmax[0])
            ess_line = {"ess_per_sec": float(ess_min_sum) / e_T, "vtype": "imse", "kept_per_chain": e_nkept,
                        "sum_min_ess": float(ess_min_sum), "sampling_s": e_T, "ess_compute_s": ess_s, "leg": leg,
                        "note": "sum_c min_j ESS_cj (ess.jl:6-10, Geyer IMSE; NaN or negative estimates count as "
                                "0) / sampling seconds of that run; ESS on the GPU (kernels/stats.hip), outside "
                                "the timed region"}
        if e_samples is not samples:
            del e_samples

    pcie = None
    if args.pcie:
        # the same run with caller-owned host buffers (C ABI on_device = 0): the kept samples, gradients and
        # accept bits are copied to host memory after the step loop; pinned if the allocation succeeds
        try:
            hs = torch.empty((nkept, d, C), dtype=torch.float64, pin_memory=True)
            hg = torch.empty((nkept, d, C), dtype=torch.float64, pin_memory=True) if grad_sampler else None
            hb = torch.empty((nkept, (C + 63) // 64), dtype=torch.int64, pin_memory=True)
            kind = "pinned"
        except RuntimeError:
            hs = torch.empty((nkept, d, C), dtype=torch.float64)
            hg = torch.empty((nkept, d, C), dtype=torch.float64) if grad_sampler else None
            hb = torch.empty((nkept, (C + 63) // 64), dtype=torch.int64)
            kind = "pageable"
        hout = _lib.Outputs()
        hout.samples = hs.data_ptr()
        hout.gradients = hg.data_ptr() if hg is not None else None
        hout.accept_bits = hb.data_ptr()
        hout.on_device = 0
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(hout)))
        Tp = time.perf_counter() - t0
        pcie = {"value": C * world * K / Tp, "unit": "chain-steps/s", "ms_per_step": Tp * 1e3 / K,
                "host_buffers": kind, "bytes_to_host": int(hs.numel() * 8 + (hg.numel() * 8 if hg is not None else 0)
                                                          + hb.numel() * 8),
                "note": "the same workload with host output buffers: the step loop plus the device-to-host copy "
                        "of the kept outputs after it"}
        del hs, hg, hb
    gather = None
    if dist is not None and world > 1:
        # the end-of-run gather, after and apart from the timed region: the timed run's kept
        # samples (+ gradients), accept bits chunked point to point into rank 0's host memory (sharded.py
        # gather_shards); capped at GATHER_CAP_BYTES of global samples so a 1000-step 8-GPU metric run does not
        # fill the host (the kept rows gathered are then the first `rows` of each rank)
        from mcmchip.sharded import gather_shards
        GATHER_CAP_BYTES = 32 << 30
        row_bytes = d * C * 8 * world * (2 if grads is not None else 1)
        rows = max(1, min(nkept, GATHER_CAP_BYTES // max(1, row_bytes)))
        gparts = {"samples": samples[:rows], "accept_bits": bits[:rows]}
        if grads is not None:
            gparts["gradients"] = grads[:rows]
        if backend != "nccl":
            gparts = {k: v.cpu() for k, v in gparts.items()}
        gstats = {}
        torch.cuda.synchronize(dev)
        dist.barrier()
        tg = time.perf_counter()
        g_out = gather_shards(gparts, C, C, C * world, dst=0, stats=gstats)
        gmax = torch.tensor([time.perf_counter() - tg], dtype=torch.float64, device=red_dev)
        dist.all_reduce(gmax, op=dist.ReduceOp.MAX)
        gbytes = sum(v.numel() * v.element_size() for v in gparts.values()) * world
        gather = {"gather_s": float(gmax[0]), "bytes": int(gbytes), "GB_per_s": gbytes / float(gmax[0]) / 1e9,
                  "kept_rows": rows, "of_kept_rows": nkept, "max_recv_buffer_bytes": gstats.get("max_recv_buffer_bytes"),
                  "max_buffer_bytes_per_source": gstats.get("max_buffer_bytes_per_source"),
                  "max_sources_in_flight": gstats.get("max_sources_in_flight"), "slots": gstats.get("slots"),
                  "note": "chunked point-to-point gather of the timed run's outputs into rank 0's host memory, "
                          "receives from every source rank in flight together (two buffers per source), each "
                          "landed chunk copied to page-locked host memory on a side stream while the next arrives; "
                          "timed apart (max over ranks); never inside the step loop"}
        del g_out, gparts
    spl = args.spl if args.spl >= 0 else 0
    nl = ct.c_int64(0)
    _lib.check(lib.mcmc_chains_launches(h, K, ct.byref(nl)))
    launches = nl.value                                  # the library's plan (some kernels fuse one step)
    # per-GPU workload key: the PMC traffic of a committed rocprofv3 run of this same workload
    # (profiles/traffic.json, written by scripts/summarize_prof.py) fills roofline.traffic
    wkey = f"{args.config}|d={d}|chains={C}|{args.sampler}|steps={K}|thinning={args.thinning}|spl={spl}"
    kname = task.step_kernel                            # the instance the timed run launched (C ABI)
    tdet = measured_traffic(wkey, kname)
    traffic = tdet["bytes_per_launch"] if tdet else None
    avg_launch_s = kernel_ms * 1e-3 / launches          # HIP events around the launches, on their stream
    units = C * K / launches                            # chain-steps per launch
    if cfg0["model"] in ("iso", "distobs"):
        # HBM: the fused kernel reads and writes the chain state once per launch (x [d][C], lp [C]) and
        # streams the kept samples (+ gradients) and accept bits; SURVEY.md §8(d)'s per-step state round trip
        # (16 d + 16 + 1/8 B per chain-step) is what an unfused step would move, kept as `survey_bytes`
        per_step, per_kept = hbm_bytes_per_unit(d, args.sampler)
        state_b = 2 * C * (8 * d + 8)                  # x [d][C] and lp [C], read and written
        fused = launches * state_b + C * nkept * (per_kept + 1 / 8)
        if args.sampler == "ram":
            # the jump factor S (d(d+1)/2 doubles per chain) does not fit on chip: read and written every step
            fused += C * K * 8 * d * (d + 1)
        hbm_ach = fused / launches / avg_launch_s / 1e9
        survey = C * K * per_step + C * nkept * per_kept
        hbm = {"achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_ach / HBM_PEAK_GBS,
               "algorithmic_bytes_per_launch": fused / launches, "traffic": traffic, "traffic_detail": tdet,
               "note": "fused design: chain state in and out once per launch + kept samples/gradients + accept bits"
                       + (" + the RAM jump factor read and written every step" if args.sampler == "ram" else "")}
        survey_bytes = {"bytes_per_unit": {"chain_step": per_step, "kept_chain_step": per_kept},
                        "equivalent_GBps": survey / launches / avg_launch_s / 1e9,
                        "note": "SURVEY.md §8(d) bytes of an unfused step (state round trip every step); the "
                                "fused kernel never moves them, so this rate can exceed HBM peak: it is the north "
                                "star's '% of HBM roofline' yardstick, not a roofline"}
        vm = measured_valu(kname, wkey)
        if vm is not None and args.sampler != "ram":
            # the binding resource: VALU issue.  SQ_ACTIVE_INST_VALU quad-cycles x 4 = SIMD-cycles of VALU issue
            # per chain-step (measured, committed profile of this kernel instance); achieved = that x chain-steps
            # per launch / the live launch time; peak = 1024 SIMDs x 2.4 GHz (the spec engine clock)
            cyc = 4.0 * vm["valu_quadcycles_per_chain_step"]
            ach = cyc * units / avg_launch_s / 1e12
            roof = {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_TCYC, "unit": "T VALU-issue-cycles/s",
                    "frac": ach / VALU_PEAK_TCYC, "traffic": traffic, "kernel": kname, "launches": launches,
                    "avg_launch_ms": avg_launch_s * 1e3, "units_per_launch": units,
                    "valu_cycles_per_unit": cyc, "valu_busy_measured": vm["valu_busy"],
                    "clock_ghz_measured": vm["clock_ghz"], "valu_source": vm["source"],
                    "hbm": hbm, "survey_bytes": survey_bytes,
                    "valu_floor": valu_floor(args, vm),
                    "note": "units = chain-steps; VALU cycles per unit from rocprofv3 PMC (SQ_ACTIVE_INST_VALU); "
                            "valu_busy_measured = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES of that profile (at "
                            "the measured clock); HBM moves only the per-launch state and the kept outputs "
                            "(hbm.frac)"}
        else:
            roof = {"bound": "hbm", "achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_detail": tdet, "kernel": kname,
                    "launches": launches, "avg_launch_ms": avg_launch_s * 1e3,
                    "algorithmic_bytes_per_launch": fused / launches, "units_per_launch": units,
                    "survey_bytes": survey_bytes,
                    "note": ("RAM: the jump factor S (d(d+1)/2 doubles a chain) is read and written every step, "
                             "so HBM binds (the factor update and matvec are 2 flops per 8-byte element)"
                             if args.sampler == "ram" else
                             "no committed VALU profile of this kernel instance built from these sources "
                             "(profiles/valu.json src_hash): HBM roofline of the fused design")}
        if args.sampler == "ram" and vm is not None:
            # RAM binds on HBM (the factor); the profile's VALU issue rides along
            cyc = 4.0 * vm["valu_quadcycles_per_chain_step"]
            roof["valu"] = {"achieved": cyc * units / avg_launch_s / 1e12, "peak": VALU_PEAK_TCYC,
                            "unit": "T VALU-issue-cycles/s", "frac": cyc * units / avg_launch_s / 1e12 / VALU_PEAK_TCYC,
                            "valu_busy_measured": vm["valu_busy"], "source": vm["source"]}
        if C <= 64:
            roof["binding"] = ("latency: a few-chain kernel runs each chain's steps as one dependent chain of "
                               "operations (C <= 64: lpc_rwm_spec / lpc_rwm_la), so neither the VALU nor the HBM "
                               "fraction is the bound; ms_per_step is the step's dependent-path latency")
    else:
        flop_per_eval = 4.0 * cfg0["n"] * d                           # eta = X beta, then X^T r
        flops = flop_per_eval * evals
        achieved = flops / launches / avg_launch_s / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": achieved / F64_MFMA_PEAK_TFS, "traffic": traffic, "traffic_detail": tdet, "kernel": kname,
                "launches": launches, "avg_launch_ms": avg_launch_s * 1e3, "flop_per_eval": flop_per_eval,
                "evals_per_launch": evals / launches, "units_per_launch": C * K / launches,
                "note": "units = log-target+gradient evaluations (leapfrogs for HMC/HMCDA, counted on the "
                        "device); 4 n d fp64 flop each (SURVEY.md §8(d))"}
        if args.sampler == "ram":
            # RAM on a regression target: the jump factor S (d(d+1)/2 doubles a chain) is read and written every
            # step (glm_ram, glm_ram_wave.hip), beside the state's round trip; HBM against the MFMA eval, the
            # larger fraction names the bound
            ram_b = C * K * (8.0 * d * (d + 1) + 16.0 * d + 16.0) + C * nkept * (8.0 * d + 1 / 8)
            hbm_ach = ram_b / launches / avg_launch_s / 1e9
            hbm = {"achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_ach / HBM_PEAK_GBS,
                   "algorithmic_bytes_per_launch": ram_b / launches, "traffic": traffic,
                   "bytes_per_unit": {"chain_step": 8.0 * d * (d + 1) + 16.0 * d + 16.0, "kept_chain_step": 8.0 * d},
                   "note": "the RAM jump factor read and written every step + the state round trip + kept rows"}
            if hbm["frac"] >= roof["frac"]:
                mf = dict(roof)
                for k in ("kernel", "launches", "avg_launch_ms", "traffic", "traffic_detail"):
                    mf.pop(k, None)
                roof = {"bound": "hbm", "achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": hbm["frac"], "traffic": traffic, "kernel": kname, "launches": launches,
                        "avg_launch_ms": avg_launch_s * 1e3, "algorithmic_bytes_per_launch": ram_b / launches,
                        "bytes_per_unit": hbm["bytes_per_unit"], "mfma": mf, "note": hbm["note"]}
            else:
                roof["hbm"] = hbm
        vm = measured_valu(kname, wkey)
        if vm is not None:
            # the small regression targets (d <= 16: one MFMA covers a 16-chain tile's contraction): the per-step
            # RNG and elementwise work issue on the VALU, which the fp64 MFMAs also occupy; the
            # VALU issue fraction of a committed PMC profile names the bound when it is the larger
            cyc = 4.0 * vm["valu_quadcycles_per_chain_step"]
            ach = cyc * C * K / launches / avg_launch_s / 1e12
            vroof = {"achieved": ach, "peak": VALU_PEAK_TCYC, "unit": "T VALU-issue-cycles/s",
                     "frac": ach / VALU_PEAK_TCYC, "valu_cycles_per_unit": cyc, "valu_busy_measured": vm["valu_busy"],
                     "clock_ghz_measured": vm["clock_ghz"], "valu_source": vm["source"],
                     "note": "units = chain-steps; SQ_ACTIVE_INST_VALU of a committed PMC profile (fp64 MFMAs "
                             "included: they issue on the VALU)"}
            if vroof["frac"] > roof["frac"]:
                mf = dict(roof)
                for k in ("kernel", "launches", "avg_launch_ms", "traffic", "traffic_detail"):
                    mf.pop(k, None)
                roof = dict(vroof, bound="valu", traffic=traffic, kernel=kname, launches=launches,
                            avg_launch_ms=avg_launch_s * 1e3, units_per_launch=C * K / launches, mfma=mf)
            else:
                roof["valu"] = vroof
        fm = measured_fp64(kname, wkey)
        if fm is not None:                                            # MFMA + VALU fp64 on the shared datapath
            per_eval = fm["mfma_flop_per_eval"] + fm["valu_fp64_flop_per_eval"]
            comb = per_eval * evals / launches / avg_launch_s / 1e12
            roof["fp64_combined"] = {
                "achieved": comb, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": comb / F64_MFMA_PEAK_TFS,
                "mfma_flop_per_eval": fm["mfma_flop_per_eval"], "valu_fp64_flop_per_eval": fm["valu_fp64_flop_per_eval"],
                "source": fm["source"],
                "note": "fp64 MFMA and fp64 VALU instructions share the SIMD's fp64 datapath: (measured MFMA flops + "
                        "64 x SQ_INSTS_VALU_FLOPS_FP64 per evaluation of a committed PMC profile) x the live "
                        "launch's evaluations / its time"}
    # acceptance over the timed run's kept steps (accept bits, SerialMC.jl:55-63)
    pop8 = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.float64, device=dev)
    acceptance = float(pop8[bits.view(torch.uint8).long()].sum()) / max(1, nkept * C)
    if cfg0["model"] not in ("iso", "distobs"):
        roof["leapfrogs_per_chain_step" if args.sampler in ("hmc", "hmcda") else "evals_per_chain_step"] = \
            evals / (C * K)
        roof["chain_evals_per_s"] = evals * world / T
    line = {
        "metric": "MCMC steps*chains/sec (1M chains, d=32)" if args.config == "metric"
        else f"MCMC steps*chains/sec ({cfg0['desc'].split(':')[0]})",
        "value": value,
        "unit": "chain-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": T * 1e3 / K,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (chains start at model.init; Philox4x32-10 streams, seed 1"
                + ("; regression data from numpy Philox, key 0x5EED)" if cfg0["model"] not in ("iso", "distobs")
                   else ")"),
        "config": {
            "workload": f"{args.config}: {cfg0['desc']}; SerialMC(steps={K}, burnin={burnin}, "
                        f"thinning={args.thinning}), {C} chains/GPU, {type(sampler).__name__}",
            "d": d, "chains_per_gpu": C, "global_chains": total_chains, "sampler": args.sampler,
            "burnin": burnin, "thinning": args.thinning, "kept_per_chain": nkept,
            "steps_per_launch": spl, "evals": evals, "key": wkey,
            "parallelism": f"chains sharded over {world} GPU(s), no collective in the step loop",
            "process_group": (("nccl (RCCL)" if backend == "nccl" else backend) if dist is not None else None),
        },
        "roofline": roof,
        "acceptance": acceptance,
        "ess": ess_line,
    }
    if adapt is not None:
        line["adaptation"] = adapt
    if args.config in ("binomial", "bare_normal") and rank == 0:
        line["reference_units"] = binomial_units(mc, model, C, local, args.config)
    if pcie is not None:
        line["pcie_inclusive"] = pcie
    if gather is not None:
        line["gather"] = gather
    if rank == 0 and not args.no_cpu_baseline:          # after the timed region, also on N > 1 lines
        lps = evals / (C * K) if args.sampler == "hmcda" else None
        line["cpu_baseline"] = cpu_baseline(model, sampler, args.cpu_seconds,
                                            C=min(C, 4096 if cfg0["model"] == "iso" else 64), leaps_per_step=lps)
    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()                                  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
