"""Output analysis of a batched MCMCChain (src/stats/*.jl), vectorised over chains.

acceptance   summary.jl:6-15      100 * sum(accept[lags]) / length(lags)
mean         mean.jl:6
mcvar_iid    var.jl:7-8           var(x) / n
mcvar_bm     var.jl:20-27         batch means
mcvar_imse   var.jl:45-75         Geyer's initial monotone sequence estimator
mcvar_ipse   var.jl:95-117        Geyer's initial positive sequence estimator
var          var.jl:137-149       dispatch on vtype
ess, actime  ess.jl:6-20          n * var_iid / var_vtype, var_vtype / var_iid

Autocovariances follow StatsBase.acf(x, lags, correlation=false): the demeaned
sum sum_{t} z_t z_{t+k} / n.  They are computed by FFT over all chains and
parameters at once (the reference loops per column), so values agree with the
reference's direct sums to rounding, not bitwise ("parity unpinned":
StatsBase is not vendored and has no fixture).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

__all__ = ["acceptance", "mean", "mcvar_iid", "mcvar_bm", "mcvar_imse", "mcvar_ipse", "var", "ess", "actime",
           "autocov", "ess_device", "ess_per_sec"]


def _samples(c) -> np.ndarray:
    """[nchains, nkept, d] from an MCMCChain or an array."""
    s = c.samples if hasattr(c, "samples") else np.asarray(c, dtype=np.float64)
    if s.ndim == 1:
        s = s[None, :, None]
    elif s.ndim == 2:
        s = s[None]
    return s


def acceptance(c, lags=None, reject: bool = False) -> np.ndarray:
    """Per-chain acceptance (or rejection) percentage over kept steps `lags` (1-based range)."""
    acc = np.asarray(c.diagnostics["accept"])          # [nchains, nkept] bool
    nk = acc.shape[1]
    if lags is None:
        lags = range(1, nk + 1)
    if not lags[-1] <= nk:
        raise AssertionError("Range of acceptance rate not within post-burnin range of MCMC chain")
    idx = np.asarray(list(lags)) - 1
    rlen = len(idx)
    s = acc[:, idx].sum(axis=1)
    return ((rlen - s) if reject else s) * 100 / rlen


def mean(c) -> np.ndarray:
    return _samples(c).mean(axis=1)


def autocov(x: np.ndarray, maxlag: int) -> np.ndarray:
    """acf(x, 0:maxlag, correlation=false) along axis 1 of x [C, n, d] -> [C, maxlag+1, d]."""
    n = x.shape[1]
    z = x - x.mean(axis=1, keepdims=True)
    nfft = 1
    while nfft < 2 * n:
        nfft *= 2
    f = np.fft.rfft(z, n=nfft, axis=1)
    acv = np.fft.irfft(f * np.conj(f), n=nfft, axis=1)[:, : maxlag + 1] / n
    return acv


def mcvar_iid(c) -> np.ndarray:
    s = _samples(c)
    return s.var(axis=1, ddof=1) / s.shape[1]


def mcvar_bm(c, batchlen: int = 100) -> np.ndarray:
    s = _samples(c)
    nb = s.shape[1] // batchlen
    if not nb > 1:
        raise AssertionError("Choose batch size such that the number of batches is greather than one")
    bm = s[:, : nb * batchlen].reshape(s.shape[0], nb, batchlen, s.shape[2]).mean(axis=2)
    return batchlen * bm.var(axis=1, ddof=1) / (nb * batchlen)


def _geyer(c, maxlag, monotone: bool) -> np.ndarray:
    s = _samples(c)
    n = s.shape[1]
    if maxlag is None:
        maxlag = n - 1
    k = (maxlag - 1) // 2
    acv = autocov(s, maxlag)                                  # [C, maxlag+1, d]
    if 2 * k + 2 > acv.shape[1]:
        acv = np.concatenate([acv, np.zeros((acv.shape[0], 2 * k + 2 - acv.shape[1], acv.shape[2]))], axis=1)
    g = acv[:, 0 : 2 * k + 2 : 2] + acv[:, 1 : 2 * k + 2 : 2]  # g[j] = acv[2j] + acv[2j+1], j = 0..k
    nonpos = g <= 0
    m = np.where(nonpos.any(axis=1), nonpos.argmax(axis=1), k + 1)   # first j with g[j] <= 0, else k+1
    if monotone:
        g = np.minimum.accumulate(g, axis=1)
    j = np.arange(g.shape[1])[None, :, None]
    gs = np.where(j < m[:, None, :], g, 0.0).sum(axis=1)
    return (-acv[:, 0] + 2 * gs) / n


def mcvar_imse(c, maxlag=None) -> np.ndarray:
    return _geyer(c, maxlag, monotone=True)


def mcvar_ipse(c, maxlag=None) -> np.ndarray:
    return _geyer(c, maxlag, monotone=False)


def var(c, vtype: str = "imse", **kw) -> np.ndarray:
    vt = vtype.lstrip(":")
    if vt not in ("bm", "iid", "imse", "ipse"):
        raise AssertionError(f"Unknown variance type {vtype}")
    return {"bm": mcvar_bm, "iid": mcvar_iid, "imse": mcvar_imse, "ipse": mcvar_ipse}[vt](c, **kw)


def ess(c, vtype: str = "imse", **kw) -> np.ndarray:
    """Effective sample size per chain and parameter (ess.jl:6-10)."""
    vt = vtype.lstrip(":")
    if vt not in ("bm", "imse", "ipse"):
        raise AssertionError(f"Unknown ESS type {vtype}")
    n = _samples(c).shape[1]
    return n * var(c, "iid") / var(c, vt, **kw)


def actime(c, vtype: str = "imse", **kw) -> np.ndarray:
    """Integrated autocorrelation time (ess.jl:13-17)."""
    vt = vtype.lstrip(":")
    if vt not in ("bm", "imse", "ipse"):
        raise AssertionError(f"Unknown integrated autocorrelation time type {vtype}")
    return var(c, vt, **kw) / var(c, "iid")


_VT = {"imse": 1, "ipse": 2, "bm": 3}


def ess_device(c, vtype: str = "imse", maxlag: Optional[int] = None, batchlen: int = 100, device: int = 0,
               return_var: bool = False):
    """ESS of every (chain, parameter) series on the GPU (kernels/stats.hip; ess.jl:6-10).

    `c` is an MCMCChain (host samples; returns numpy [nchains, d] like `ess`) or a device tensor
    [nkept, d, nchains] in the C-ABI layout (returns a device tensor [d, nchains], nothing crosses PCIe)."""
    import ctypes as ct
    from . import _lib
    from .api import _ctx
    vt = vtype.lstrip(":")
    if vt not in _VT:
        raise AssertionError(f"Unknown ESS type {vtype}")
    lib = _lib.load()
    ml = 0 if maxlag is None else int(maxlag)
    if hasattr(c, "data_ptr"):                                   # torch device tensor
        import torch
        if c.dim() != 3 or c.dtype != torch.float64 or not c.is_contiguous():
            raise ValueError("expected a contiguous float64 tensor [nkept, d, nchains]")
        n, d, C = c.shape
        e = torch.empty((d, C), dtype=torch.float64, device=c.device)
        v = torch.empty((d, C), dtype=torch.float64, device=c.device) if return_var else None
        _lib.check(lib.mcmc_stats_ess(_ctx(c.device.index or 0), c.data_ptr(), n, d, C, _VT[vt], ml, batchlen, 1,
                                      e.data_ptr(), v.data_ptr() if v is not None else None))
        return (e, v) if return_var else e
    s = np.ascontiguousarray(c._samples if hasattr(c, "_samples") else c, dtype=np.float64)
    n, d, C = s.shape
    e = np.empty((d, C))
    v = np.empty((d, C)) if return_var else None
    _lib.check(lib.mcmc_stats_ess(_ctx(device), s.ctypes.data, n, d, C, _VT[vt], ml, batchlen, 0, e.ctypes.data,
                                  v.ctypes.data if v is not None else None))
    return (e.T.copy(), v.T.copy()) if return_var else e.T.copy()


def ess_per_sec(ess_dc, seconds: float) -> float:
    """sum over chains of min over parameters of ESS, per sampling second."""
    m = ess_dc.min(dim=0).values.sum().item() if hasattr(ess_dc, "min") and hasattr(ess_dc, "dim") \
        else float(np.min(ess_dc, axis=0).sum())
    return m / seconds
