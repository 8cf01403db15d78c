"""Host-side mirror of MCMC.jl's model x sampler x runner API, driving the C ABI.

Names, argument meaning and error behaviour follow the reference:

  model(f; init, scale, grad)    src/modellers/mcmcmodels.jl:27-33, likmodel.jl:100-143
  RWM, MALA, HMC, HMCDA, RAM     src/samplers/{RWM,MALA,HMC,HMCDA,RAM}.jl (constructors + @asserts)
  EmpMCTuner                     src/samplers/samplers.jl:32-50
  SerialMC(steps, burnin, thinning) / SerialMC(range)   src/runners/SerialMC.jl:12-35
  m * s * r -> MCMCTask          src/MCMC.jl:87-98
  run(task) / run(chain)         src/runners/runners.jl:7-14,45 ; SerialMC.jl:37-85
  resume(chain; steps)           src/runners/runners.jl:48-68 ; SerialMC.jl:93-97
  MCMCChain                      src/MCMC.jl:58-84

What is new: one MCMCTask is a *batch* of `nchains` independent Markov chains
of the same (model, sampler, runner) -- the reference's `run(Array{MCMCTask})`
(runners.jl:17-26) for the homogeneous case -- each chain with its own random
stream keyed by (seed, global chain id, step).  Julia closures cannot cross a
C ABI, so `model()` takes an entry of the model catalogue (IsoNormalDot,
NormalDSL, LogisticRegression, LinearRegression) in place of a function.
"""
from __future__ import annotations

import ctypes as ct
import math
from typing import Optional, Sequence, Union

import numpy as np

from . import _lib
from ._lib import check, dptr

__all__ = [
    "IsoNormalDot", "NormalDSL", "AbsNormalDSL", "DistDSL", "DistObsDSL", "LogisticRegression", "LinearRegression", "ProbitRegression", "vaso_data",
    "OrnsteinUhlenbeck", "ou_series", "MCMCLikelihoodModel", "model",
    "RWM", "MALA", "HMC", "HMCDA", "RAM", "EmpMCTuner", "EmpiricalMCMCTuner", "SerialMC", "MCMCTask", "MCMCChain",
    "run", "resume", "device_count",
]

# ------------------------------------------------------------------ device contexts
_CTX: dict = {}


def device_count() -> int:
    n = ct.c_int(0)
    check(_lib.load().mcmc_device_count(ct.byref(n)))
    return n.value


def _ctx(device: int) -> ct.c_void_p:
    if device not in _CTX:
        h = ct.c_void_p()
        check(_lib.load().mcmc_ctx_create(int(device), ct.byref(h)))
        _CTX[device] = h
    return _CTX[device]


def _f64(a, n: Optional[int] = None) -> np.ndarray:
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if n is not None and arr.shape != (n,):
        raise ValueError(f"expected a vector of length {n}, got shape {arr.shape}")
    return arr


# ------------------------------------------------------------------ model catalogue
class IsoNormalDot:
    """The README target `v -> -dot(v,v)`; its gradient `v -> -2v` is `IsoNormalDot.grad` (README.md:60,63)."""
    kind = _lib.MODEL_ISO_NORMAL_DOT
    grad = "v -> -2v"


class NormalDSL:
    """The DSL model `v ~ Normal(mu, sigma)` with gradient=true (README.md:67-72)."""
    kind = _lib.MODEL_NORMAL_DSL

    def __init__(self, mu: float = 0.0, sigma: float = 1.0):
        self.mu, self.sigma = float(mu), float(sigma)


class AbsNormalDSL:
    """The DSL model `y = abs(x); y ~ Normal(mu, sigma)` (README.md:246-251, the SeqMC example)."""
    kind = _lib.MODEL_ABS_NORMAL_DSL

    def __init__(self, mu: float = 0.0, sigma: float = 1.0):
        self.mu, self.sigma = float(mu), float(sigma)


class DistDSL:
    """The DSL statement `v ~ Dist(p1, p2)` over the parameter vector (elementwise, summed), for the DSL's
    continuous distributions with x-derivative rules (MCMCDerivRules.jl:56-104): Normal, Uniform,
    Weibull, Beta, TDist, Exponential, Gamma, Cauchy, LogNormal, Laplace (Distributions.jl parameters and
    defaults)."""
    kind = _lib.MODEL_DIST_DSL
    _DEFAULTS = {"Normal": (0.0, 1.0), "Uniform": (0.0, 1.0), "Weibull": (1.0, 1.0), "Beta": (1.0, 1.0),
                 "TDist": (1.0, 0.0), "Exponential": (1.0, 0.0), "Gamma": (1.0, 1.0), "Cauchy": (0.0, 1.0),
                 "LogNormal": (0.0, 1.0), "Laplace": (0.0, 1.0)}

    def __init__(self, dist: str, *params: float):
        if dist not in _lib.DISTS:
            raise ValueError(f"unsupported distribution {dist!r}; one of {sorted(_lib.DISTS)}")
        p = list(self._DEFAULTS[dist])
        if len(params) > 2:
            raise ValueError("at most two parameters")
        for i, v in enumerate(params):
            p[i] = float(v)
        self.name, self.dist = dist, _lib.DISTS[dist]
        self.mu, self.sigma = p                         # p1, p2 in the C ABI's mu / sigma slots


class DistObsDSL(DistDSL):
    """The DSL block `y = x * v; y ~ Dist(p1, p2)` of the reference's bare_distribs benchmark unit
    (benchmarks/benchunits/bare_distribs.jl:13, v = ones(1000) there): a scalar parameter x scaling the data vector v,
    log-target sum_i logpdf(Dist, x v_i).  v rides in the C ABI's data slots (X = v as one column, Y = v)."""
    kind = _lib.MODEL_DIST_OBS

    def __init__(self, dist: str, *params: float, v=None):
        super().__init__(dist, *params)
        v = np.ones(1000) if v is None else v
        self.Y = np.ascontiguousarray(np.asarray(v, dtype=np.float64).reshape(-1))
        self.X = self.Y.reshape(-1, 1)


class LogisticRegression:
    """examples/logistic_regression.jl:16-22: vars ~ Normal(0, prior); prob = 1/(1+exp(-X*vars)); Y ~ Bernoulli(prob).
    link_sign=-1 gives test/test_syntax.jl:13's exp(+X*vars) variant."""
    kind = _lib.MODEL_LOGISTIC

    def __init__(self, X, Y, prior_sigma: float = 1.0, link_sign: float = 1.0):
        self.X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        self.Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
        self.prior_sigma, self.link_sign = float(prior_sigma), float(link_sign)


class LinearRegression:
    """examples/linear_regression.jl:14-20: vars ~ Normal(0, prior); resid = Y - X*vars; resid ~ Normal(0, noise)."""
    kind = _lib.MODEL_LINEAR

    def __init__(self, X, Y, prior_sigma: float = 1.0, noise_sigma: float = 1.0):
        self.X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        self.Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
        self.prior_sigma, self.noise_sigma = float(prior_sigma), float(noise_sigma)


class ProbitRegression:
    """examples/probit_regression.jl:18-40: log-prior MvNormal(zeros(d), prior_sigma^2 I) (priorstd = 10 in the
    example) + dot(logcdf(Normal(), X*pars), Y) + dot(logcdf(Normal(), -X*pars), 1 - Y), Y in {0, 1}; gradient
    X'*(Y.*exp(A - logcdf(X*pars)) - (1 - Y).*exp(A - logcdf(-X*pars))) - pars/prior_sigma^2, A = -((X*pars).^2 +
    log(2pi))/2.  vaso_data() builds the example's design matrix."""
    kind = _lib.MODEL_PROBIT

    def __init__(self, X, Y, prior_sigma: float = 10.0):
        self.X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        self.Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
        self.prior_sigma = float(prior_sigma)


class OrnsteinUhlenbeck:
    """examples/ornstein.jl:19-30: parameters (tau, sigma, mu) with tau ~ Uniform(0, 100), sigma ~ Uniform(0, 2),
    mu ~ Uniform(0, 20); fac = exp(-1/tau); resid = x[2:end] - x[1:end-1]*fac - mu*(1-fac); resid ~ Normal(0, sigma),
    over the series x.  The example: model(OrnsteinUhlenbeck(x), tau=0.05, sigma=1., mu=1., gradient=True) with
    m.scale = [1000., 1., 10.] (ornstein.jl:29-30), run under RAM() and HMC(5, 0.002)."""
    kind = _lib.MODEL_OU

    def __init__(self, x):
        self.series = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
        if self.series.shape[0] < 2:
            raise ValueError("the Ornstein-Uhlenbeck model needs a series of at least 2 values")


def ou_series(duration: int = 1000, mu0: float = 10.0, tau0: float = 20.0, sigma0: float = 0.1, seed: int = 1):
    """The example's simulated series (examples/ornstein.jl:6-17): x[1] = 1, x[i] = x[i-1] exp(-1/tau0) +
    mu0 (1 - exp(-1/tau0)) + sigma0 randn().  numpy's normal stream stands in for Julia's srand(1) randn, so the
    values are the example's process, not its exact draws."""
    rng = np.random.default_rng(seed)
    x = np.empty(duration)
    x[0] = 1.0
    e = np.exp(-1.0 / tau0)
    for i in range(1, duration):
        x[i] = x[i - 1] * e + mu0 * (1.0 - e) + sigma0 * rng.standard_normal()
    return x


def vaso_data(path):
    """The probit example's design matrix (examples/probit_regression.jl:7-16): vaso.txt's covariates standardised
    (mean / sample std per column), polynomial order 1, a leading column of ones; the last column is y."""
    vaso = np.loadtxt(path)
    cov, y = vaso[:, :-1], vaso[:, -1]
    cov = (cov - cov.mean(axis=0)) / cov.std(axis=0, ddof=1)
    X = np.hstack([np.ones((cov.shape[0], 1)), cov])
    return X, y


class MCMCLikelihoodModel:
    """MCMCLikelihoodModel (likmodel.jl:20-57): target + init + scale + pmap, uploaded once per GPU."""

    def __init__(self, target, init, scale=1.0, gradient: bool = False, pmap: Optional[dict] = None):
        self.target = target
        init = [float(init)] if np.isscalar(init) else init                   # likmodel.jl:112
        self.init = _f64(init).reshape(-1)
        self.size = int(self.init.shape[0])
        if np.isscalar(scale):
            self.scale = float(scale) * np.ones(self.size)                     # likmodel.jl:115
        else:
            self.scale = _f64(scale).reshape(-1)
        if self.scale.shape[0] != self.size:                                   # likmodel.jl:44
            raise AssertionError(f"scale parameter size ({self.scale.shape[0]}) different from initial values "
                                 f"({self.size})")
        self.has_gradient = bool(gradient)         # hasgradient(m) = m.evalg != nothing (mcmcmodels.jl:19)
        self.pmap = pmap if pmap is not None else {"pars": (1, (self.size,))}  # likmodel.jl:118
        if hasattr(target, "X"):
            if target.X.ndim != 2 or target.X.shape[1] != self.size:
                raise ValueError(f"X must be [n, {self.size}]")
            if target.Y.shape != (target.X.shape[0],):
                raise ValueError("Y must have one entry per row of X")
        self._dev: dict = {}

    # device handle, created on first use per GPU
    def _handle(self, device: int) -> ct.c_void_p:
        if device in self._dev:
            return self._dev[device]
        desc = self._desc()
        h = ct.c_void_p()
        check(_lib.load().mcmc_model_create(_ctx(device), ct.byref(desc), ct.byref(h)))
        self._dev[device] = h
        return h

    def _desc(self) -> _lib.ModelDesc:
        """The C ABI model descriptor (its pointers borrow this model's arrays)."""
        t = self.target
        desc = _lib.ModelDesc()
        desc.kind = t.kind
        desc.has_gradient = 1 if self.has_gradient else 0
        desc.d = self.size
        desc.init = dptr(self.init)
        desc.scale = dptr(self.scale)
        desc.mu = getattr(t, "mu", 0.0)
        desc.sigma = getattr(t, "sigma", 1.0)
        desc.prior_sigma = getattr(t, "prior_sigma", 1.0)
        desc.noise_sigma = getattr(t, "noise_sigma", 1.0)
        desc.link_sign = getattr(t, "link_sign", 1.0)
        desc.dist = getattr(t, "dist", 0)
        if hasattr(t, "X"):
            desc.n = t.X.shape[0]
            desc.X = dptr(t.X)
            desc.Y = dptr(t.Y)
        elif hasattr(t, "series"):
            desc.n = t.series.shape[0]
            desc.Y = dptr(t.series)
        return desc

    def eval(self, x, device: int = 0):
        """model.eval on a batch: x [d] or [d, nchains] -> lp (likmodel.jl:21)."""
        return self.evalallg(x, device=device, _grad=False)[0]

    def evalallg(self, x, device: int = 0, _grad: bool = True):
        """model.evalallg on a batch: x [d] or [d, nchains] -> (lp, grad) (likmodel.jl:25)."""
        xa = np.asarray(x, dtype=np.float64)
        single = xa.ndim == 1
        xa = np.ascontiguousarray(xa.reshape(self.size, -1))
        C = xa.shape[1]
        lp = np.empty(C)
        g = np.empty((self.size, C)) if _grad else None
        check(_lib.load().mcmc_model_eval(self._handle(device), C, dptr(xa), dptr(lp), dptr(g)))
        if single:
            return lp[0], (g[:, 0] if g is not None else None)
        return lp, g

    def __mul__(self, sampler):
        return _ModelSampler(self, sampler)

    def __del__(self):
        try:
            lib = _lib.load()
            for h in self._dev.values():
                lib.mcmc_model_destroy(h)
        except Exception:
            pass


def model(f, mtype: str = "likelihood", init=None, scale=1.0, gradient: bool = False,
          grad=None, **dsl_init) -> MCMCLikelihoodModel:
    """model() entry point (mcmcmodels.jl:27-33).

    Function style (likmodel.jl:100-143): model(IsoNormalDot(), init=ones(3)) has no gradient, like
    `model(v-> -dot(v,v), init=ones(3))`; pass grad=IsoNormalDot.grad (or grad=True) for mymodel2's
    `grad=v->-2v` (README.md:60-63).  DSL style (likmodel.jl:72-96): model(NormalDSL(0, 1), v=ones(3),
    gradient=True), model(LogisticRegression(X, Y), vars=zeros(10), gradient=True)."""
    if mtype != "likelihood":
        raise ValueError(f"unknown model type {mtype!r}")
    if dsl_init:
        if init is not None:
            raise AssertionError("'init' kwargs not allowed for model as expression\n")   # likmodel.jl:80
        # modelVars (expr_funcs.jl:76-90): parameters packed column-major, concatenated in keyword order
        init = np.concatenate([np.asarray(v, dtype=np.float64).reshape(-1, order="F") for v in dsl_init.values()])
    if init is None:
        init = [1.0]                                                                       # likmodel.jl:107
    if grad is not None and grad is not False:
        gradient = True
    return MCMCLikelihoodModel(f, init, scale=scale, gradient=gradient)


# ------------------------------------------------------------------ samplers
class EmpiricalMCMCTuner:
    """EmpiricalMCMCTuner (samplers.jl:32-50)."""

    def __init__(self, targetRate: float, adaptStep: int = 100, maxStep: int = 200, targetPath: float = 1.0,
                 verbose: bool = False):
        if not adaptStep > 0:
            raise AssertionError(f"Adaptation step size ({adaptStep}) should be > 0")
        if not maxStep > 0:
            raise AssertionError(f"Adaptation step size ({maxStep}) should be > 0")
        if not 0 < targetRate < 1:
            raise AssertionError(f"Target acceptance rate ({targetRate}) should be between 0 and 1")
        self.targetRate, self.adaptStep, self.maxStep = float(targetRate), int(adaptStep), int(maxStep)
        self.targetPath, self.verbose = float(targetPath), bool(verbose)


EmpMCTuner = EmpiricalMCMCTuner


class _Sampler:
    kind = 0
    tuner = None
    uses_gradient = True       # MALA, HMC, HMCDA need model.evalg; RWM and RAM do not

    def cfg(self) -> _lib.SamplerCfg:
        c = _lib.SamplerCfg()
        c.kind = self.kind
        t = self.tuner
        if t is not None:
            c.tuner = 1
            c.adapt_step, c.max_step = t.adaptStep, t.maxStep
            c.target_path, c.target_rate = t.targetPath, t.targetRate
        return c

    def __mul__(self, runner):                     # sampler * runner (for model * (sampler * runner) chains)
        return _SamplerRunner(self, runner)


class RWM(_Sampler):
    """Random-walk Metropolis (RWM.jl:24-36)."""
    kind = _lib.SAMPLER_RWM
    uses_gradient = False

    def __init__(self, scale: float = 1.0, tuner=None):
        if not scale > 0:
            raise AssertionError("scale should be > 0")                       # RWM.jl:29
        if tuner is not None:
            raise NotImplementedError("RWMTuner is abstract in the reference (RWM.jl:18)")
        self.scale = float(scale)

    def cfg(self):
        c = super().cfg()
        c.scale = self.scale
        return c


class MALA(_Sampler):
    """Metropolis-adjusted Langevin (MALA.jl:50-62)."""
    kind = _lib.SAMPLER_MALA

    def __init__(self, driftStep: Union[float, EmpiricalMCMCTuner] = 1.0, tuner=None, scale: Optional[float] = None):
        if isinstance(driftStep, EmpiricalMCMCTuner):          # MALA(s::MCMCTuner) = MALA(1.0, t)
            driftStep, tuner = 1.0, driftStep
        if scale is not None:                                  # MALA(;scale, tuner) keyword form
            driftStep = scale
        if not driftStep > 0:
            raise AssertionError("MALA drift step should be > 0")              # MALA.jl:55
        self.driftStep, self.tuner = float(driftStep), tuner

    def cfg(self):
        c = super().cfg()
        c.drift_step = self.driftStep
        return c


class HMC(_Sampler):
    """Hamiltonian Monte Carlo (HMC.jl:53-74); positional forms as the reference's constructors:
    HMC(), HMC(nLeaps), HMC(nLeaps, leapStep), HMC(leapStep::Float64), HMC(tuner)."""
    kind = _lib.SAMPLER_HMC

    def __init__(self, *args, nLeaps: Optional[int] = None, leapStep: Optional[float] = None, tuner=None,
                 storeLeaps: bool = False):
        n, e = 10, 0.1
        a = list(args)
        if a and isinstance(a[-1], EmpiricalMCMCTuner):
            tuner = a.pop()
        if len(a) == 1:
            if isinstance(a[0], float):
                e = a[0]                                        # HMC(leapStep::Float64) = HMC(10, leapStep)
            else:
                n = int(a[0])                                   # HMC(nLeaps::Int) = HMC(nLeaps, 0.1)
        elif len(a) == 2:
            n, e = int(a[0]), float(a[1])
        elif len(a) > 2:
            raise TypeError("HMC(nLeaps, leapStep[, tuner])")
        if nLeaps is not None:
            n = int(nLeaps)
        if leapStep is not None:
            e = float(leapStep)
        if not n > 0:
            raise AssertionError("inner steps should be > 0")                  # HMC.jl:60
        if not e > 0:
            raise AssertionError("inner steps scaling should be > 0")          # HMC.jl:61
        self.nLeaps, self.leapStep, self.tuner = n, e, tuner
        self.storeLeaps = bool(storeLeaps)

    def leaps_cap(self) -> int:
        """leapfrog states stored per kept step (storeLeaps): nLeaps, or the tuner's maxStep bound"""
        return max(self.nLeaps, self.tuner.maxStep) if self.tuner is not None else self.nLeaps

    def cfg(self):
        c = super().cfg()
        c.n_leaps, c.leap_step = self.nLeaps, self.leapStep
        return c


class HMCDA(_Sampler):
    """HMC with dual-averaging step size (HMCDA.jl:24-43)."""
    kind = _lib.SAMPLER_HMCDA

    def __init__(self, rate: float = 0.65, len: float = 2.0, shrinkage: float = 0.05, t0: float = 10.0,
                 step: float = 0.75, storeLeaps: bool = False, max_leaps: int = 0):
        if not 0.0 < rate < 1.0:
            raise AssertionError(f"Target acceptance rate ({rate}) should be between 0 and 1")
        if not len > 0:
            raise AssertionError(f"len parameter of HMCDA sampler ({len}) must be non-negative")
        if not shrinkage > 0.0:
            raise AssertionError(f"shrinkage parameter of HMCDA sampler ({shrinkage}) must be positive")
        if not t0 >= 0:
            raise AssertionError(f"t0 parameter of HMCDA sampler ({t0}) must be non-negative")
        self.rate, self.len, self.shrinkage, self.t0, self.step = rate, len, shrinkage, t0, step
        self.max_leaps = int(max_leaps)
        self.storeLeaps = bool(storeLeaps)

    def leaps_cap(self) -> int:
        """leapfrog states stored per kept step (storeLeaps): max_leaps when set, else 256 (the trajectory
        length round(len / leapStep) adapts; diagnostics["leaps"]["nleaps"] always holds the full count)"""
        return self.max_leaps if self.max_leaps > 0 else 256

    def cfg(self):
        c = super().cfg()
        c.rate, c.len, c.shrinkage, c.t0, c.step = self.rate, self.len, self.shrinkage, self.t0, self.step
        c.max_leaps = self.max_leaps
        return c


class RAM(_Sampler):
    """Robust adaptive Metropolis (RAM.jl:22-34): RAM(), RAM(scale), RAM(scale, rate),
    RAM(scale=..., rate=...).  Each chain adapts its own d x d jump factor (kept on the device)."""
    kind = _lib.SAMPLER_RAM
    uses_gradient = False

    def __init__(self, scale: float = 1.0, rate: float = 0.234):
        if not scale > 0:
            raise AssertionError("scale should be > 0")                                           # RAM.jl:27
        if not (rate > 0.0 and rate < 1.0):
            raise AssertionError(f"target acceptance rate ({rate}) should be between 0 and 1")   # RAM.jl:28
        self.scale, self.rate = float(scale), float(rate)

    def cfg(self):
        c = super().cfg()
        c.scale, c.rate = self.scale, self.rate
        return c


# ------------------------------------------------------------------ runner
class SerialMC:
    """SerialMC runner (SerialMC.jl:12-35): keeps samples i in r = (burnin+1):thinning:steps."""

    def __init__(self, steps: Union[int, range] = 100, burnin: int = 0, thinning: int = 1):
        if isinstance(steps, range):                           # SerialMC(steps::Range)
            r = steps
            burnin = r.start - 1
            thinning = r.step
            length = r[-1] if len(r) else r.start - 1
        else:
            length = int(steps)
        if not burnin >= 0:
            raise AssertionError(f"Burnin rounds ({burnin}) should be >= 0")
        if not length > burnin:
            raise AssertionError(f"Total MCMC length ({length}) should be > to burnin ({burnin})")
        if not thinning >= 1:
            raise AssertionError(f"Thinning ({thinning}) should be >= 1")
        self.burnin, self.thinning, self.len = int(burnin), int(thinning), int(length)
        self.r = range(self.burnin + 1, self.len + 1, self.thinning)

    def cfg(self) -> _lib.RunnerCfg:
        c = _lib.RunnerCfg()
        c.burnin, c.thinning, c.len = self.burnin, self.thinning, self.len
        return c


# ------------------------------------------------------------------ task / chain
class _ModelSampler:
    def __init__(self, m, s):
        self.m, self.s = m, s

    def __mul__(self, r):
        return _spin(self.m, self.s, r)


class _SamplerRunner:
    def __init__(self, s, r):
        self.s, self.r = s, r

    def __rmul__(self, m):
        return _spin(m, self.s, self.r)


# ------------------------------------------------------------------ the global random stream
class _GlobalStream:
    """The reference's tasks draw their random numbers from Julia's one global RNG as they run, so every spun task
    -- each element of m * [s1, s2] * r, a second run(m * s * r), the fresh task of resume -- samples a chain of its
    own (MCMC.jl:87-98, SerialMC.jl:93-97).  Here a chain's stream is the Philox key (seed) and its global chain id
    (DESIGN.md §3), so the mirror of that global RNG is a seed plus a cursor over chain ids: a task spun by `*` (or
    resume) takes the next ids when it first runs, exactly as a Julia task first consumes the global RNG when it
    runs.  srand(seed) restarts the cursor (Julia's srand).

    The Philox key of a drawn stream is drawn_key(seed): the seed with the top bit set.  Explicit seeds (MCMCTask's
    default seed=1, run(..., seed=s), SeqMC's target keys) live below 2^63, so a drawn chain never replays a chain a
    task with an explicit seed and offset samples, whatever the two cursors are."""
    seed = 1
    next_chain = 0


DRAWN_KEY_BIT = 1 << 63


def drawn_key(seed: int) -> int:
    """The Philox key of the global stream's chains under srand(seed): a key space of its own (top bit set)."""
    return (int(seed) & (DRAWN_KEY_BIT - 1)) | DRAWN_KEY_BIT


def srand(seed: int) -> None:
    """srand(seed) for GPU tasks: later spun tasks draw global chain ids 0, 1, ... under Philox key `seed`."""
    _GlobalStream.seed = int(seed)
    _GlobalStream.next_chain = 0


def _draw_chains(n: int):
    """(seed, first global chain id) of n chains taken from the global stream; ids are 32-bit (the Philox counter's
    chain word), so a cursor that would pass 2^32 moves on to the next key."""
    n = int(n)
    if _GlobalStream.next_chain + n > 1 << 32:
        _GlobalStream.seed += 1
        _GlobalStream.next_chain = 0
    first = _GlobalStream.next_chain
    _GlobalStream.next_chain += n
    return drawn_key(_GlobalStream.seed), first


def _spin(m, s, r):
    """m * s * r with the reference's array broadcasting (MCMC.jl:87-98).  Every task draws its own chains from
    the global stream when it first runs (seed / chain_offset None until then)."""
    ms = m if isinstance(m, (list, tuple)) else None
    ss = s if isinstance(s, (list, tuple)) else None
    rs = r if isinstance(r, (list, tuple)) else None
    if ms is None and ss is None and rs is None:
        return MCMCTask(m, s, r, seed=None, chain_offset=None)
    n = max(len(x) for x in (ms, ss, rs) if x is not None)
    pick = lambda v, i: v[i] if isinstance(v, (list, tuple)) else v  # noqa: E731
    return [MCMCTask(pick(m, i), pick(s, i), pick(r, i), seed=None, chain_offset=None) for i in range(n)]


class MCMCTask:
    """A batch of `nchains` independent chains of (model, sampler, runner) on one GPU (MCMC.jl:33-39).

    seed / chain_offset name the chains' random streams (Philox key, first global chain id).  None (tasks spun by
    `*`): drawn from the global stream when the task first runs (_GlobalStream)."""

    def __init__(self, model: MCMCLikelihoodModel, sampler: _Sampler, runner: SerialMC, nchains: int = 1,
                 seed: Optional[int] = 1, device: int = 0, chain_offset: Optional[int] = 0, init_x=None,
                 steps_per_launch: int = 0, devices: Optional[Sequence[int]] = None):
        self._h = None
        self._group = None
        self._fork = None            # (batch task, first chain): chains of a batched run(Array), forked on first use
        self._stopped = False        # prun's tasks (run_serialmc_exit: stop!, SerialMC.jl:87-91)
        if not isinstance(runner, SerialMC) and type(runner).__name__ != "SeqMC":
            raise NotImplementedError("runners: SerialMC (one batch) or SeqMC (lists of targets, run_seqmc)")
        if sampler.uses_gradient and not model.has_gradient:
            name = type(sampler).__name__
            raise AssertionError(f"{name} sampler requires model with gradient function")
        self.model, self.sampler, self.runner = model, sampler, runner
        self.nchains, self.device = int(nchains), int(device)
        self.seed = None if seed is None else int(seed)
        self.chain_offset = None if chain_offset is None else int(chain_offset)
        if self.seed is not None and self.chain_offset is None:
            self.chain_offset = 0
        if self.seed is None and self.chain_offset is not None:
            raise ValueError("a task with an explicit chain_offset needs an explicit seed")
        self.init_x = None if init_x is None else np.ascontiguousarray(
            np.asarray(init_x, dtype=np.float64).reshape(model.size, self.nchains))
        self.steps_per_launch = int(steps_per_launch)
        # devices: run the batch as one mcmc_group over these GPUs (contiguous 64-chain-aligned blocks, one
        # per listed device; a device may repeat); None: one context on `device`
        self.devices = None if devices is None else tuple(int(x) for x in devices)
        if self.devices is not None and len(self.devices) == 0:
            raise ValueError("devices must list at least one GPU")

    def batch(self, nchains: int, seed: Optional[int] = None, **kw) -> "MCMCTask":
        """Same (model, sampler, runner) over `nchains` chains.  An explicit seed names the stream outright
        (chain_offset defaults to 0); without one the new task keeps this task's stream (drawn when it runs, for a
        spun task)."""
        off = kw.get("chain_offset", self.chain_offset)
        if seed is not None and off is None:
            off = 0
        if seed is None:
            seed = self.seed
            if seed is None and off is not None:
                seed = drawn_key(_GlobalStream.seed)
        return MCMCTask(self.model, self.sampler, self.runner, nchains=nchains, seed=seed,
                        device=kw.get("device", self.device), chain_offset=off, init_x=kw.get("init_x"),
                        steps_per_launch=kw.get("steps_per_launch", self.steps_per_launch),
                        devices=kw.get("devices", self.devices))

    def _draw(self) -> None:
        if self.seed is None:
            self.seed, self.chain_offset = _draw_chains(self.nchains)

    def handle(self) -> ct.c_void_p:
        """The mcmc_chains (one context) or, with `devices`, the mcmc_group_chains of this task."""
        if self._stopped:
            raise AssertionError("the task was stopped by prun (run_serialmc_exit, SerialMC.jl:87-91)")
        if self._h is None and self._fork is not None:             # chains k.. of a batched run: a copy of them
            src, first = self._fork
            h = ct.c_void_p()
            check(_lib.load().mcmc_chains_fork(src.handle(), first, self.nchains, ct.byref(h)))
            self._h, self._fork = h, None
        self._draw()
        if self._h is None and self.devices is not None:
            lib = _lib.load()
            g = ct.c_void_p()
            devs = (ct.c_int32 * len(self.devices))(*self.devices)
            check(lib.mcmc_group_create(devs, len(self.devices), ct.byref(g)))
            self._group = g
            h = ct.c_void_p()
            desc = self.model._desc()
            cfg = self.sampler.cfg()
            check(lib.mcmc_group_chains_create(g, ct.byref(desc), ct.byref(cfg), self.nchains, self.chain_offset,
                                               ct.c_uint64(self.seed & 0xFFFFFFFFFFFFFFFF), dptr(self.init_x),
                                               ct.byref(h)))
            if self.steps_per_launch:
                check(lib.mcmc_group_chains_set_steps_per_launch(h, self.steps_per_launch))
            self._h = h
        if self._h is None:
            mh = self.model._handle(self.device)
            h = ct.c_void_p()
            cfg = self.sampler.cfg()
            check(_lib.load().mcmc_chains_create(mh, ct.byref(cfg), self.nchains, self.chain_offset,
                                                 ct.c_uint64(self.seed & 0xFFFFFFFFFFFFFFFF),
                                                 dptr(self.init_x), ct.byref(h)))
            if self.steps_per_launch:
                check(_lib.load().mcmc_chains_set_steps_per_launch(h, self.steps_per_launch))
            self._h = h
        return self._h

    def blocks(self):
        """[(mcmc_chains handle or None, first chain, chain count)] per listed device (group tasks), or the
        single batch as one block."""
        h = self.handle()
        if self.devices is None:
            return [(h, 0, self.nchains)]
        out = []
        for b in range(len(self.devices)):
            c, f, n = ct.c_void_p(), ct.c_int64(), ct.c_int64()
            check(_lib.load().mcmc_group_chains_block(h, b, ct.byref(c), ct.byref(f), ct.byref(n)))
            out.append((c if c.value else None, f.value, n.value))
        return out

    @property
    def steps_done(self) -> int:
        if self._h is None:
            return self._fork[0].steps_done if self._fork is not None else 0
        v = ct.c_int64(0)
        if self.devices is not None:
            check(_lib.load().mcmc_group_chains_steps_done(self._h, ct.byref(v)))
        else:
            check(_lib.load().mcmc_chains_steps_done(self._h, ct.byref(v)))
        return v.value

    @property
    def evals(self) -> int:
        """Log-target evaluations over all chains since the chains were created/reset."""
        if self._h is None:
            return 0
        tot = 0
        for c, _, _ in self.blocks():
            if c is not None:
                v = ct.c_int64(0)
                check(_lib.load().mcmc_chains_evals(c, ct.byref(v)))
                tot += v.value
        return tot

    def tuner_state(self):
        """Per-chain adaptive state after the last run (mcmc_chains_tuner_state): a dict of [nchains] arrays
        "step" (MALA driftStep / HMC leapStep under the empirical tuners; HMCDA leapStep), "step_bar" (HMCDA's
        dualLeapStep, HMCDA.jl:138) and "nleaps" (tuned HMC); NaN / 0 where the sampler does not adapt it."""
        C = self.nchains
        step = np.empty(C)
        bar = np.empty(C)
        nl = np.empty(C, dtype=np.int32)
        for c, f, n in self.blocks():
            if c is None:
                continue
            a, b, k = np.empty(n), np.empty(n), np.empty(n, dtype=np.int32)
            check(_lib.load().mcmc_chains_tuner_state(c, a.ctypes.data, b.ctypes.data, k.ctypes.data))
            step[f:f + n], bar[f:f + n], nl[f:f + n] = a, b, k
        return {"step": step, "step_bar": bar, "nleaps": nl}

    @property
    def step_kernel(self) -> str:
        """The step kernel instance the last run launched (mcmc_chains_step_kernel), e.g.
        "lpc_rwm<8, true, IsoDot, true>"; "" before the first run (group tasks: block 0's)."""
        buf = ct.create_string_buffer(160)
        check(_lib.load().mcmc_chains_step_kernel(self.blocks()[0][0], buf, len(buf)))
        return buf.value.decode()

    def ram_factor(self) -> np.ndarray:
        """RAM: the current jump factor S of every chain as [nchains][d][d] lower-triangular matrices."""
        if self._h is None:
            raise AssertionError("the task has not run")
        d, C = self.model.size, self.nchains
        packed = np.empty((d * (d + 1) // 2, C))
        for c, f, n in self.blocks():
            if c is not None:
                part = np.empty((d * (d + 1) // 2, n))
                check(_lib.load().mcmc_chains_ram_factor(c, part.ctypes.data))
                packed[:, f:f + n] = part
        return unpack_ram_factor(packed, d)

    def reset(self) -> None:
        if self._h is not None:
            if self.devices is not None:
                check(_lib.load().mcmc_group_chains_reset(self._h))
            else:
                check(_lib.load().mcmc_chains_reset(self._h))

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None:
                if self.devices is not None:
                    _lib.load().mcmc_group_chains_destroy(self._h)
                else:
                    _lib.load().mcmc_chains_destroy(self._h)
            if getattr(self, "_group", None) is not None:
                _lib.load().mcmc_group_destroy(self._group)
        except Exception:
            pass


class MCMCChain:
    """Result of a run (MCMC.jl:58-80), batched over chains.

    samples[c] is chain c's [nkept x d] sample matrix (the reference's DataFrame);
    gradients likewise (all NaN for RWM, SerialMC.jl:42); diagnostics["accept"][c]
    is the per-kept-step accept flag and diagnostics["step"] = collect(r)."""

    def __init__(self, r: range, samples, gradients, diagnostics: dict, task: MCMCTask, runTime: float,
                 kernel_ms: float = float("nan"), final_x=None, final_lp=None):
        self.range = r
        self._samples = samples                 # [nkept, d, nchains] (C ABI layout)
        self._gradients = gradients
        self.diagnostics = diagnostics
        self.task = task
        self.runTime = runTime
        self.kernel_ms = kernel_ms
        self.final_x, self.final_lp = final_x, final_lp

    def _chains(self, first: int, count: int, task: "MCMCTask") -> "MCMCChain":
        """Chains [first, first + count) of this result as the result of `task`."""
        sl = slice(first, first + count)
        diags = dict(self.diagnostics)
        diags["accept"] = self.diagnostics["accept"][sl]
        if "leaps" in diags:
            diags["leaps"] = {k: v[..., sl] for k, v in self.diagnostics["leaps"].items()}
        g = None if self._gradients is None else self._gradients[:, :, sl]
        fx = None if self.final_x is None else self.final_x[:, sl]
        flp = None if self.final_lp is None else self.final_lp[sl]
        return MCMCChain(self.range, self._samples[:, :, sl], g, diags, task, self.runTime, self.kernel_ms, fx, flp)

    @property
    def samples(self) -> np.ndarray:
        return np.transpose(self._samples, (2, 0, 1))

    @property
    def gradients(self) -> np.ndarray:
        if self._gradients is None:
            nk, d, C = self._samples.shape
            return np.full((C, nk, d), np.nan)
        return np.transpose(self._gradients, (2, 0, 1))

    @property
    def nchains(self) -> int:
        return self._samples.shape[2]

    def __repr__(self) -> str:                                                 # MCMC.jl:82-84
        nk, d, C = self._samples.shape
        return f"{d} parameters, {nk} samples (per parameter), {C} chain(s), {round(self.runTime, 1)} sec."


def unpack_ram_factor(packed: np.ndarray, d: int) -> np.ndarray:
    """[d(d+1)/2][C] packed lower rows -> [C][d][d]."""
    C = packed.shape[1]
    S = np.zeros((C, d, d))
    r, c = np.tril_indices(d)                                  # row-major order of the packed rows
    S[:, r, c] = packed.T
    return S


def _unpack_bits(bits: np.ndarray, C: int) -> np.ndarray:
    """[nkept][ceil(C/64)] u64 -> bool [C, nkept]; bit c%64 of word c//64 is chain c."""
    nk = bits.shape[0]
    b = np.unpackbits(bits.view(np.uint8).reshape(nk, -1), axis=1, bitorder="little")[:, :C]
    return b.astype(bool).T.copy()


def _run_task(t: MCMCTask) -> MCMCChain:
    lib = _lib.load()
    h = t.handle()
    r = t.runner
    d, C = t.model.size, t.nchains
    nk = len(r.r)
    nw = (C + 63) // 64
    samples = np.empty((nk, d, C))
    grads = np.empty((nk, d, C)) if t.sampler.uses_gradient else None
    bits = np.zeros((nk, nw), dtype=np.uint64)
    fx = np.empty((d, C))
    flp = np.empty(C)
    out = _lib.Outputs()
    out.samples = samples.ctypes.data
    out.gradients = grads.ctypes.data if grads is not None else None
    out.accept_bits = bits.ctypes.data
    out.final_x = fx.ctypes.data
    out.final_lp = flp.ctypes.data
    out.on_device = 0
    leaps = None
    if t.devices is not None and getattr(t.sampler, "storeLeaps", False):
        raise NotImplementedError("storeLeaps on a group task: run the batch on one device")
    if getattr(t.sampler, "storeLeaps", False):              # HMC.jl:145-150 / HMCDA.jl:110-117
        cap = t.sampler.leaps_cap()
        leaps = {"pars": np.empty((nk, cap + 1, d, C)), "grad": np.empty((nk, cap + 1, d, C)),
                 "m": np.empty((nk, cap + 1, d, C)), "logTarget": np.empty((nk, cap + 1, C)),
                 "H": np.empty((nk, cap + 1, C)), "nleaps": np.empty((nk, C), dtype=np.int32)}
        check(lib.mcmc_chains_store_leaps(h, cap, *(leaps[k].ctypes.data for k in
                                                    ("pars", "grad", "m", "logTarget", "H", "nleaps"))))
    cfg = r.cfg()
    gather_s = None
    if t.devices is not None:
        gs = ct.c_double(0.0)
        check(lib.mcmc_group_run_serialmc(h, ct.byref(cfg), ct.byref(out), ct.byref(gs)))
        gather_s = gs.value
    else:
        check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(out)))
    diags = {"step": list(r.r), "accept": _unpack_bits(bits, C)}
    if gather_s is not None:
        diags["gather_s"] = gather_s                         # end gather of the group run, timed apart
    if leaps is not None:
        # per kept step: the trajectory's states, leap 0 = state0 (the reference's leapStates array of
        # HMCSample(pars, grad, m, logTarget, H)), NaN past nleaps
        diags["leaps"] = leaps
    return MCMCChain(r.r, samples, grads, diags, t, out.runtime_s, out.kernel_ms, fx, flp)


def _same_task_kind(t: MCMCTask, t0: MCMCTask) -> bool:
    """t can share one chain batch with t0: the same model object, sampler configuration and runner, a stream
    still to be drawn, one context, every chain at model.init."""
    return (isinstance(t, MCMCTask) and t._h is None and t._fork is None and not t._stopped and t.seed is None
            and t.model is t0.model and type(t.sampler) is type(t0.sampler)
            and bytes(t.sampler.cfg()) == bytes(t0.sampler.cfg())
            and getattr(t.sampler, "storeLeaps", False) == getattr(t0.sampler, "storeLeaps", False)
            and isinstance(t.runner, SerialMC)
            and (t.runner.burnin, t.runner.thinning, t.runner.len) == (t0.runner.burnin, t0.runner.thinning,
                                                                       t0.runner.len)
            and t.init_x is None and t.devices is None and t0.devices is None and t.device == t0.device
            and t.steps_per_launch == t0.steps_per_launch)


def _run_batched(ts, stop: bool = False, devices=None):
    """One chain batch for an array of like tasks: the tasks' chains are consecutive global ids drawn from the
    stream, one mcmc_run_serialmc (or one group run over `devices`) advances them all, and task k's MCMCChain holds
    its own chains.  Its task then continues them (run(c) = run(c.task), runners.jl:14) from a fork of the batch's
    state, or, with stop (prun), is stopped as run_serialmc_exit leaves it (SerialMC.jl:87-91)."""
    t0 = ts[0]
    n = [t.nchains for t in ts]
    seed, off = _draw_chains(sum(n))
    bt = MCMCTask(t0.model, t0.sampler, t0.runner, nchains=sum(n), seed=seed, device=t0.device, chain_offset=off,
                  steps_per_launch=t0.steps_per_launch, devices=devices)
    ch = _run_task(bt)
    out, f = [], 0
    for t, k in zip(ts, n):
        t.seed, t.chain_offset = seed, off + f
        if stop:
            t._stopped = True
        else:
            t._fork = (bt, f)
        out.append(ch._chains(f, k, t))
        f += k
    return out


def run(t, *args, nchains: Optional[int] = None, seed: Optional[int] = None, **kw):
    """run(task) / run(chain) (continue) / run(m, s, r) / run([tasks])  (runners.jl:7-32,45).

    run([tasks]) of SerialMC tasks spun by `*` from one model, sampler configuration and runner (m * [s, s] * r,
    [m, m] * s * r, ...) runs them as ONE chain batch (one launch sequence for all of them); each returned
    MCMCChain's task continues its own chains.  Other arrays run task by task, as the reference does."""
    if args:                                                 # run(m, s, r)
        return run(_spin(t, args[0], args[1]), nchains=nchains, seed=seed, **kw)
    if isinstance(t, (list, tuple)):
        if not t:
            return []
        kinds = {type(x.runner if isinstance(x, MCMCTask) else x.task.runner) for x in t}
        if len(kinds) != 1:
            raise AssertionError("Runners do not have the same runner type")
        if next(iter(kinds)).__name__ == "SeqMC":                 # run(t::Array{MCMCTask}) -> run_seqmc
            from .seqmc import run_seqmc
            return run_seqmc(t, seed=1 if seed is None else seed, **kw)
        if nchains is None and seed is None and not kw and all(_same_task_kind(x, t[0]) for x in t):
            return _run_batched(list(t))
        return [run(x, nchains=nchains, seed=seed, **kw) for x in t]
    if isinstance(t, MCMCChain):                              # run(c::MCMCChain) = run(c.task)
        return _run_task(t.task)
    if nchains is not None or seed is not None or kw:
        if t._h is not None or t._fork is not None:
            raise ValueError("task already started; build a new task to change nchains/seed")
        t = t.batch(nchains if nchains is not None else t.nchains, seed=seed, **kw)
    return _run_task(t)


def prun(t, devices: Optional[Sequence[int]] = None):
    """prun(tasks) (runners.jl:35-42): pmap(run_serialmc_exit, t) -- every task run to its end, in parallel, then
    stopped.  Here like tasks form one chain batch over `devices` (default: every visible GPU, as one mcmc_group
    when there are several; the results do not depend on the device count) and come back stopped; other arrays run
    task by task."""
    if isinstance(t, MCMCTask):
        t = [t]
    t = list(t)
    if not t:
        return []
    kinds = {type(x.runner) for x in t}
    if len(kinds) != 1:
        raise AssertionError("Runners do not have the same runner type")
    if not isinstance(t[-1].runner, SerialMC):
        return None                                          # the reference's prun only runs SerialMC tasks
    if devices is None and not getattr(t[0].sampler, "storeLeaps", False):   # storeLeaps records: one device
        nd = device_count()
        devices = tuple(range(nd)) if nd > 1 else None
    if all(_same_task_kind(x, t[0]) for x in t):
        return _run_batched(t, stop=True, devices=devices)
    out = [_run_task(x) for x in t]
    for x in t:
        x._stopped = True
    return out


def resume(c, steps: int = 100, seed: Optional[int] = None, chain_offset: Optional[int] = None):
    """resume(chain; steps) (SerialMC.jl:93-97): run(t.model, t.sampler, SerialMC(steps, thinning)) -- a *new*
    task from model.init.  Its chains are drawn from the global stream (the reference's new task samples on from the
    advanced global RNG), so they are not a replay of the original run; seed / chain_offset name them outright."""
    if isinstance(c, (list, tuple)):
        return [resume(x, steps=steps, seed=seed, chain_offset=chain_offset) for x in c]
    t = c.task if isinstance(c, MCMCChain) else c
    if seed is not None and chain_offset is None:
        chain_offset = 0
    if seed is None and chain_offset is not None:
        seed = drawn_key(_GlobalStream.seed)
    nt = MCMCTask(t.model, t.sampler, SerialMC(steps=steps, thinning=t.runner.thinning), nchains=t.nchains,
                  seed=seed, device=t.device, chain_offset=chain_offset, init_x=t.init_x,
                  steps_per_launch=t.steps_per_launch, devices=t.devices)
    return _run_task(nt)


def reset(t, x) -> np.ndarray:
    """MCMC.reset(t::MCMCTask, x) (MCMC.jl:39; the samplers' :reset hooks, RWM.jl:49, MALA.jl:75-80, HMC.jl:114-116,
    HMCDA.jl:82-83, RAM.jl:47): every chain of the task moves to x ([d], or [d][nchains] per chain) and its
    log-target (and gradient) is re-evaluated there; step counter, tuners and RAM factor are kept.  Returns the
    log-targets at x [nchains]."""
    if t.devices is not None:
        raise NotImplementedError("reset of a group task: reset its blocks' tasks on one device")
    h = t.handle()
    d, C = t.model.size, t.nchains
    xs = np.asarray(x, dtype=np.float64)
    xs = np.ascontiguousarray(np.repeat(xs.reshape(d, 1), C, axis=1) if xs.size == d else xs.reshape(d, C))
    lp = np.empty(C)
    check(_lib.load().mcmc_chains_set_state(h, dptr(xs), dptr(lp)))
    return lp
