"""SeqMC population runner (src/runners/SeqMC.jl): targets x particles on the GPU.

Particle n is chain n of every target's chain batch.  Per outer step and target, every particle is
reset into the target and advanced one step of that target's sampler (the same HIP kernels as
SerialMC), then the importance weights are updated and, when var(W) < trigger, the particles are
resampled -- all on the device (kernels/seqmc.hip), with no host round trip inside the loop.
"""
from __future__ import annotations

import ctypes as ct
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .api import MCMCChain, MCMCTask

__all__ = ["SeqMC", "run_seqmc", "resume_seqmc", "SeqMCChain", "target_seed"]


class SeqMC:
    """SeqMC(steps, burnin, trigger) runner (SeqMC.jl:21-35)."""

    def __init__(self, steps: int = 1, burnin: int = 0, trigger: float = 1e-10):
        if not burnin >= 0:
            raise AssertionError(f"Burnin rounds ({burnin}) should be >= 0")
        if not steps > burnin:
            raise AssertionError(f"Steps ({steps}) should be > to burnin ({burnin})")
        self.steps, self.burnin, self.trigger = int(steps), int(burnin), float(trigger)

    def cfg(self) -> "_SeqCfg":
        c = _SeqCfg()
        c.steps, c.burnin, c.trigger = self.steps, self.burnin, self.trigger
        return c


class _SeqCfg(ct.Structure):
    _fields_ = [("steps", ct.c_int64), ("burnin", ct.c_int64), ("trigger", ct.c_double)]


def target_seed(seed: int, t: int) -> int:
    """Philox key of target t's chains: distinct per target, so that particle n does not reuse the
    same normals in every target of an outer step; below 2^63, the explicit-seed key space (api.drawn_key)."""
    return (int(seed) + (t + 1) * 0x9E3779B97F4A7C15) & 0x7FFFFFFFFFFFFFFF


class SeqMCChain(MCMCChain):
    """MCMCChain of a SeqMC run (SeqMC.jl:116-121): rows are (outer step, particle), step-major."""

    @property
    def samples(self) -> np.ndarray:
        nk, d, n = self._samples.shape
        return np.transpose(self._samples, (0, 2, 1)).reshape(nk * n, d)

    @property
    def gradients(self) -> np.ndarray:            # SeqMC stores none (SeqMC.jl:118 TODO)
        return np.empty((0, self._samples.shape[1]))


def _particles(particles, d: Optional[int], seed: int) -> np.ndarray:
    if particles is None:                         # [[randn()] for i in 1:100] (SeqMC.jl:43)
        g = np.random.Generator(np.random.Philox(key=int(seed) & 0xFFFFFFFFFFFFFFFF))
        return g.standard_normal((100, d or 1))
    p = np.asarray(particles, dtype=np.float64)
    return p.reshape(len(p), -1)


def run_seqmc(targets: Sequence[MCMCTask], particles=None, seed: int = 1, device: int = 0) -> SeqMCChain:
    """run(targets; particles) for SeqMC tasks (SeqMC.jl:43-122); the runner of the last target sets
    steps, burnin and trigger."""
    targets = list(targets)
    if not targets:
        raise ValueError("no targets")
    d = targets[-1].model.size
    if not all(t.model.size == d for t in targets):
        raise AssertionError("Models do not have the same parameter vector size")          # SeqMC.jl:49
    runner = targets[-1].runner
    P = _particles(particles, d, seed)
    if P.shape[1] != d:
        raise ValueError(f"particles must have {d} coordinates")
    npart = P.shape[0]
    batches = [MCMCTask(t.model, t.sampler, runner, nchains=npart, seed=target_seed(seed, k), device=device)
               for k, t in enumerate(targets)]
    handles = (ct.c_void_p * len(batches))(*[b.handle() for b in batches])
    nstore = runner.steps - runner.burnin
    samples = np.empty((nstore, d, npart))
    weights = np.empty((nstore, npart))
    flags = np.zeros((runner.steps, len(batches)), dtype=np.int32)
    part = np.ascontiguousarray(P.T)                                                        # [d][npart]
    rt = ct.c_double(0.0)
    cfg = runner.cfg()
    _lib.check(_lib.load().mcmc_run_seqmc(handles, len(batches), npart, part.ctypes.data, ct.byref(cfg),
                                          ct.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), 0, samples.ctypes.data,
                                          weights.ctypes.data, flags.ctypes.data, ct.byref(rt)))
    diags = {"weigths": weights.reshape(-1),                                               # sic (SeqMC.jl:119)
             "particle": np.tile(np.arange(1, npart + 1), nstore),
             "resampled": flags.astype(bool)}
    r = range(runner.burnin + 1, nstore * npart + 1)                                        # SeqMC.jl:116
    ch = SeqMCChain(r, samples, None, diags, batches, rt.value)
    return ch


def resume_seqmc(targets: Sequence[MCMCTask], steps: int = 100, **kw) -> SeqMCChain:
    """resume_seqmc (SeqMC.jl:125-128): the same targets, a new SeqMC(steps, trigger) run."""
    trig = targets[-1].runner.trigger
    new = [MCMCTask(t.model, t.sampler, SeqMC(steps=steps, trigger=trig)) for t in targets]
    return run_seqmc(new, **kw)
