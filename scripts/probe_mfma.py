"""Dev probe: which fp64 accumulation order does v_mfma_f64_16x16x4_f64 implement?"""
import ctypes as ct
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mcmc.jl_amd"))
from mcmchip import _lib  # noqa: E402
from mcmchip.api import _ctx  # noqa: E402


def mfma(A, B, C, nk):
    D = np.empty((16, 16))
    _lib.check(_lib.load().mcmc_debug_mfma_f64(_ctx(0), nk, _lib.dptr(np.ascontiguousarray(A)),
                                              _lib.dptr(np.ascontiguousarray(B)), _lib.dptr(np.ascontiguousarray(C)),
                                              _lib.dptr(D)))
    return D


def fma_chain(A, B, C, order):
    D = C.copy()
    for k in order:
        D = np.array([[float(np.float64(A[i, k]) * B[k, j] + D[i, j]) for j in range(16)] for i in range(16)])
    return D


def fma_exact(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def chain_fma(A, B, C, order):
    D = C.copy()
    for k in order:
        for i in range(16):
            for j in range(16):
                D[i, j] = fma_exact(A[i, k], B[k, j], D[i, j])
    return D


def exact_sum(A, B, C):
    from fractions import Fraction
    D = np.empty_like(C)
    for i in range(16):
        for j in range(16):
            s = Fraction(C[i, j]) + sum(Fraction(A[i, k]) * Fraction(B[k, j]) for k in range(A.shape[1]))
            D[i, j] = float(s)
    return D


rng = np.random.default_rng(0)
res = {}
for trial in range(3):
    nk = 1
    A = rng.normal(size=(16, 4)) * np.exp(rng.uniform(-20, 20, size=(16, 4)))
    B = rng.normal(size=(4, 16)) * np.exp(rng.uniform(-20, 20, size=(4, 16)))
    C = rng.normal(size=(16, 16)) * np.exp(rng.uniform(-20, 20, size=(16, 16)))
    D = mfma(A, B, C, nk)
    cands = {
        "fma k=0..3": chain_fma(A, B, C, [0, 1, 2, 3]),
        "fma k=3..0": chain_fma(A, B, C, [3, 2, 1, 0]),
        "exact sum, one rounding": exact_sum(A, B, C),
        "mul+add k=0..3": fma_chain(A, B, C, [0, 1, 2, 3]),
    }
    for name, v in cands.items():
        res.setdefault(name, []).append(int(np.sum(D.view(np.uint64) == v.view(np.uint64))))
print("matches out of 256 per trial:", res)
# layout sanity: identity-ish
A = np.zeros((16, 4)); A[np.arange(16), np.arange(16) % 4] = 1.0
B = np.arange(64, dtype=float).reshape(4, 16) * 1.5 + 0.25
C = np.zeros((16, 16))
D = mfma(A, B, C, 1)
print("layout ok:", np.array_equal(D, A @ B))
