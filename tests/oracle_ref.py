"""ctypes harness for oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker.  It maps the product's configuration objects (mcmchip
models, samplers, runners) onto the oracle's C structs and runs the CPU
restatement (oracle/oracle.c) on the same seeds.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

D = ct.POINTER(ct.c_double)


class OModel(ct.Structure):
    _fields_ = [("kind", ct.c_int32), ("d", ct.c_int32), ("mu", ct.c_double), ("sigma", ct.c_double),
                ("prior_sigma", ct.c_double), ("noise_sigma", ct.c_double), ("link_sign", ct.c_double),
                ("n", ct.c_int64), ("X", D), ("Y", D), ("scale", D), ("dist", ct.c_int32)]


class OSampler(ct.Structure):
    _fields_ = [("kind", ct.c_int32), ("tuner", ct.c_int32), ("scale", ct.c_double), ("drift_step", ct.c_double),
                ("n_leaps", ct.c_int64), ("leap_step", ct.c_double), ("rate", ct.c_double), ("len", ct.c_double),
                ("shrinkage", ct.c_double), ("t0", ct.c_double), ("step", ct.c_double), ("adapt_step", ct.c_int64),
                ("max_step", ct.c_int64), ("target_path", ct.c_double), ("target_rate", ct.c_double),
                ("max_leaps", ct.c_int64)]


class OState(ct.Structure):
    _fields_ = [("x", D), ("lp", D), ("t_step", D), ("t_bar", D), ("t_h", D),
                ("t_leaps", ct.POINTER(ct.c_int32)), ("t_acc", ct.POINTER(ct.c_int32)),
                ("t_prop", ct.POINTER(ct.c_int32)), ("n_evals", ct.POINTER(ct.c_int64)), ("ram_L", D)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        L = ct.CDLL(ORACLE_LIB)
        L.orc_init.restype = ct.c_int64
        L.orc_init.argtypes = [ct.POINTER(OModel), ct.POINTER(OSampler), ct.c_int64, ct.POINTER(OState), ct.c_int]
        L.orc_run.restype = None
        L.orc_run.argtypes = [ct.POINTER(OModel), ct.POINTER(OSampler), ct.c_uint64, ct.c_int64, ct.c_int64,
                              ct.c_int64, ct.c_int64, ct.c_int64, ct.c_int64, ct.c_int64, ct.c_int64,
                              ct.POINTER(OState), D, D, ct.POINTER(ct.c_uint8), ct.c_int, ct.c_int]
        L.orc_eval_batch.restype = None
        L.orc_eval_batch.argtypes = [ct.POINTER(OModel), ct.c_int64, D, D, D, ct.c_int]
        L.orc_detmath.restype = None
        L.orc_detmath.argtypes = [ct.c_int, ct.c_int64, D, D, D]
        L.orc_philox.restype = None
        L.orc_philox.argtypes = [ct.c_int64, ct.POINTER(ct.c_uint32), ct.POINTER(ct.c_uint32),
                                 ct.POINTER(ct.c_uint32)]
        _lib = L
    return _lib


def _d(a):
    return None if a is None else a.ctypes.data_as(D)


def _i(a):
    return None if a is None else a.ctypes.data_as(ct.POINTER(ct.c_int32))


class OracleModel:
    """Keeps the numpy buffers alive for the C struct."""

    def __init__(self, m):
        t = m.target
        self.scale = np.ascontiguousarray(m.scale, dtype=np.float64)
        self.init = np.ascontiguousarray(m.init, dtype=np.float64)
        self.X = getattr(t, "X", None)
        self.Y = getattr(t, "Y", None)
        s = OModel()
        s.kind = t.kind
        s.d = m.size
        s.mu = getattr(t, "mu", 0.0)
        s.sigma = getattr(t, "sigma", 1.0)
        s.prior_sigma = getattr(t, "prior_sigma", 1.0)
        s.noise_sigma = getattr(t, "noise_sigma", 1.0)
        s.link_sign = getattr(t, "link_sign", 1.0)
        s.dist = getattr(t, "dist", 0)
        if self.X is not None:
            s.n = self.X.shape[0]
            s.X = _d(self.X)
            s.Y = _d(self.Y)
        elif getattr(t, "series", None) is not None:       # the OU model's series (MODEL_OU)
            self.Y = t.series
            s.n = self.Y.shape[0]
            s.Y = _d(self.Y)
        s.scale = _d(self.scale)
        self.s = s
        self.size = m.size


def oracle_sampler(sp) -> OSampler:
    c = sp.cfg()
    o = OSampler()
    for f, _ in OSampler._fields_:
        setattr(o, f, getattr(c, f))
    return o


ORDER_PAIR = -2          # oracle.c ORC_ORDER_PAIR: two lanes per chain (16 < d <= 32)
ORDER_HALF = -3          # oracle.c ORC_ORDER_HALF: two chains per wave (RAM steps on separable targets, 32 < d <= 256)
RAM_HALF_MAX_D = 256     # samplers.hpp HalfWaveChain: the widest d the two-chains-per-wave RAM kernel runs


def kernel_order(m, sampler_kind=None):
    """The summation order of the kernel family the library runs for this model / sampler:
    regression targets have their own fixed order (the oracle picks it from the model: 0 here); separable targets:
    lane per chain for d <= 16 (0), two lanes per chain for 16 < d <= 32 (ORDER_PAIR; RAM runs lane per chain there
    but sums its log-target in that order, its |z|^2 left to right), wave per chain up to 2048 (1), block per chain
    of 4 / 8 waves up to 8192 / 16384.  RAM for 32 < d <= 256 runs two chains per wave (ORDER_HALF; the chains'
    initial log-targets still come from the eval kernel's order 1, oracle.c orc_eval_order)."""
    d = m.size
    if getattr(m.target, "X", None) is not None:         # logistic / linear regression
        return 0
    if sampler_kind == 5 and 32 < d <= RAM_HALF_MAX_D:
        return ORDER_HALF
    return 0 if d <= 16 else ORDER_PAIR if d <= 32 else 1 if d <= 2048 else 4 if d <= 8192 else 8


class OracleChains:
    """The oracle's twin of an MCMCTask: per-chain state kept between runs.  order None: the library's own
    (kernel_order)."""

    def __init__(self, m, sampler, nchains, seed=1, chain_offset=0, init_x=None, order=None):
        self.om = OracleModel(m)
        self.os = oracle_sampler(sampler)
        self.kind = sampler.kind
        self.C = int(nchains)
        self.seed = int(seed)
        self.chain0 = int(chain_offset)
        self.order = int(kernel_order(m, sampler.kind) if order is None else order)
        d, C = m.size, self.C
        if init_x is None:
            self.x = np.ascontiguousarray(np.repeat(self.om.init[:, None], C, axis=1))
        else:
            self.x = np.ascontiguousarray(np.asarray(init_x, dtype=np.float64).reshape(d, C))
        self.lp = np.zeros(C)
        self.t_step = np.zeros(C)
        self.t_bar = np.zeros(C)
        self.t_h = np.zeros(C)
        self.t_leaps = np.zeros(C, dtype=np.int32)
        self.t_acc = np.zeros(C, dtype=np.int32)
        self.t_prop = np.zeros(C, dtype=np.int32)
        self.n_evals = np.zeros(C, dtype=np.int64)
        # RAM jump factor, packed lower rows [d(d+1)/2][C]
        self.ram_L = np.zeros((d * (d + 1) // 2 if sampler.kind == 5 else 1, C))
        self.st = OState(_d(self.x), _d(self.lp), _d(self.t_step), _d(self.t_bar), _d(self.t_h),
                         _i(self.t_leaps), _i(self.t_acc), _i(self.t_prop),
                         self.n_evals.ctypes.data_as(ct.POINTER(ct.c_int64)), _d(self.ram_L))
        bad = lib().orc_init(ct.byref(self.om.s), ct.byref(self.os), C, ct.byref(self.st), self.order)
        if bad:
            raise AssertionError("Initial values out of model support, try other values")
        self.steps_done = 0

    def run_leaps(self, runner, cap):
        """run() with the storeLeaps record (mcmc_chains_store_leaps layout); returns (samples, grads, accept,
        leaps dict with pars / grad / m [nkept][cap+1][d][C], logTarget / H [nkept][cap+1][C], nleaps [nkept][C])"""
        d, C = self.om.size, self.C
        nk = len(runner.r)
        samples = np.full((nk, d, C), np.nan)
        grads = np.full((nk, d, C), np.nan)
        acc = np.zeros((nk, C), dtype=np.uint8)
        lv = {"pars": np.full((nk, cap + 1, d, C), np.nan), "grad": np.full((nk, cap + 1, d, C), np.nan),
              "m": np.full((nk, cap + 1, d, C), np.nan), "logTarget": np.full((nk, cap + 1, C), np.nan),
              "H": np.full((nk, cap + 1, C), np.nan), "nleaps": np.zeros((nk, C), dtype=np.int32)}
        L = lib()
        L.orc_run_leaps.restype = None
        L.orc_run_leaps(ct.byref(self.om.s), ct.byref(self.os), ct.c_uint64(self.seed), ct.c_int64(self.chain0),
                        ct.c_int64(C), ct.c_int64(self.steps_done), ct.c_int64(runner.burnin),
                        ct.c_int64(runner.thinning), ct.c_int64(runner.len), ct.byref(self.st), _d(samples), _d(grads),
                        acc.ctypes.data_as(ct.POINTER(ct.c_uint8)), ct.c_int(self.order), ct.c_int64(cap),
                        _d(lv["pars"]), _d(lv["grad"]), _d(lv["m"]), _d(lv["logTarget"]), _d(lv["H"]),
                        lv["nleaps"].ctypes.data_as(ct.POINTER(ct.c_int32)))
        self.steps_done += runner.len
        return samples, grads, acc, lv

    def run(self, runner, nthreads=None, c_begin=0, c_end=None, want_grads=True):
        d, C = self.om.size, self.C
        nk = len(runner.r)
        samples = np.full((nk, d, C), np.nan)
        grads = np.full((nk, d, C), np.nan) if (want_grads and self.kind not in (1, 5)) else None
        acc = np.zeros((nk, C), dtype=np.uint8)
        if nthreads is None:
            nthreads = min(8, os.cpu_count() or 1)
        c_end = C if c_end is None else c_end
        lib().orc_run(ct.byref(self.om.s), ct.byref(self.os), ct.c_uint64(self.seed), self.chain0, C, c_begin, c_end,
                      self.steps_done, runner.burnin, runner.thinning, runner.len, ct.byref(self.st),
                      _d(samples), _d(grads), acc.ctypes.data_as(ct.POINTER(ct.c_uint8)), self.order, nthreads)
        self.steps_done += runner.len
        return samples, grads, acc


def seqmc(targets, particles, steps, burnin, trigger, seed, target_seeds, order=None):
    """orc_seqmc: run_seqmc (SeqMC.jl:43-122) over [(model, sampler), ...] with particles [npart, d].
    Returns samples [steps-burnin][d][npart], weights [steps-burnin][npart], resampled flags [steps][nt]."""
    P = np.asarray(particles, dtype=np.float64)
    npart, d = P.shape
    chains = [OracleChains(m, s, nchains=npart, seed=ts, order=order) for (m, s), ts in zip(targets, target_seeds)]
    nt = len(chains)
    if order is None:
        order = chains[0].order
        if any(c.order != order for c in chains):   # orc_seqmc takes one order for every target
            raise NotImplementedError("oracle seqmc: targets whose kernels sum in different orders")
    models = (ct.POINTER(OModel) * nt)(*[ct.pointer(c.om.s) for c in chains])
    samplers = (ct.POINTER(OSampler) * nt)(*[ct.pointer(c.os) for c in chains])
    states = (ct.POINTER(OState) * nt)(*[ct.pointer(c.st) for c in chains])
    seeds = (ct.c_uint64 * nt)(*[c.seed for c in chains])
    done = (ct.c_int64 * nt)(*([0] * nt))
    nst = steps - burnin
    samples = np.empty((nst, d, npart))
    weights = np.empty((nst, npart))
    flags = np.zeros((steps, nt), dtype=np.int32)
    part = np.ascontiguousarray(P.T)
    L = lib()
    L.orc_seqmc.restype = None
    L.orc_seqmc.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int64, D,
                            ct.c_int64, ct.c_int64, ct.c_double, ct.c_uint64, ct.c_int, D, D,
                            ct.POINTER(ct.c_int32)]
    L.orc_seqmc(models, samplers, seeds, states, done, nt, npart, _d(part), steps, burnin, trigger,
                ct.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), order, _d(samples), _d(weights),
                flags.ctypes.data_as(ct.POINTER(ct.c_int32)))
    return samples, weights, flags


def eval_batch(m, xs, order=None):
    """model.eval / evalallg of every column; order None: the library's eval kernel's order (kernel_order)"""
    if order is None:
        order = kernel_order(m)
    om = OracleModel(m)
    xs = np.ascontiguousarray(np.asarray(xs, dtype=np.float64).reshape(m.size, -1))
    C = xs.shape[1]
    lp = np.empty(C)
    g = np.empty((m.size, C))
    lib().orc_eval_batch(ct.byref(om.s), C, _d(xs), _d(lp), _d(g), order)
    return lp, g


def detmath(op, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), dtype=np.float64)
    out = np.empty(4 * len(x) if op == 6 else len(x))
    lib().orc_detmath(op, len(x), _d(x), _d(y), _d(out))
    return out


def ess(samples, vtype=1, maxlag=0, batchlen=100):
    """orc_ess: samples [nkept][d][C] -> (ess [d][C], var [d][C]); vtype 1 imse, 2 ipse, 3 bm."""
    s = np.ascontiguousarray(samples, dtype=np.float64)
    n, d, C = s.shape
    e = np.empty((d, C))
    v = np.empty((d, C))
    L = lib()
    L.orc_ess.restype = None
    L.orc_ess.argtypes = [D, ct.c_int64, ct.c_int64, ct.c_int64, ct.c_int, ct.c_int64, ct.c_int64, D, D]
    L.orc_ess(_d(s), n, d, C, vtype, maxlag, batchlen, _d(e), _d(v))
    return e, v


def philox(ctr, key):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    key = np.ascontiguousarray(key, dtype=np.uint32).reshape(-1, 2)
    out = np.empty_like(ctr)
    P = ct.POINTER(ct.c_uint32)
    lib().orc_philox(len(ctr), ctr.ctypes.data_as(P), key.ctypes.data_as(P), out.ctypes.data_as(P))
    return out
