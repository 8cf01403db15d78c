"""Dev analysis of scripts/probe_mfma4.hip's layout dump: the operand layout of v_mfma_f64_4x4x4_4b_f64 and the
accumulation order of each output (which lane holds A[i][k], B[k][j], D[i][j] of which block; is D an fma chain
over k = 0..3 like v_mfma_f64_16x16x4_f64, scripts/probe_mfma.py).

Run: python3 scripts/probe_mfma4.py gpurun_out/<call>/mfma4_layout.bin"""
import itertools
import sys
from fractions import Fraction

import numpy as np

h = np.fromfile(sys.argv[1], dtype=np.float64).reshape(-1, 4, 64)


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def orders():
    def chain(ks):
        def f(a, b, c):
            acc = c
            for k in ks:
                acc = fma(a[k], b[k], acc)
            return acc
        return f

    def exact(a, b, c):
        return float(Fraction(c) + sum(Fraction(a[k]) * Fraction(b[k]) for k in range(4)))

    def pairwise(a, b, c):                     # (a0 b0 + a1 b1) + (a2 b2 + a3 b3) + c, each product exact
        p = [Fraction(a[k]) * Fraction(b[k]) for k in range(4)]
        return float(Fraction(float(Fraction(float(p[0] + p[1])) + Fraction(float(p[2] + p[3])))) + Fraction(c))
    return {"fma k=0..3": chain([0, 1, 2, 3]), "fma k=3..0": chain([3, 2, 1, 0]), "exact, one rounding": exact,
            "pairwise": pairwise}


blocks = {"block = lane // 16": lambda l: (l // 16, l % 16), "block = lane % 4": lambda l: (l % 4, l // 4)}
ij = {"(x = l16 % 4, y = l16 // 4)": lambda t: (t % 4, t // 4), "(x = l16 // 4, y = l16 % 4)": lambda t: (t // 4, t % 4)}
best = []
for (bn, bf), (an, af), (bbn, bbf), (dn, df) in itertools.product(blocks.items(), ij.items(), ij.items(), ij.items()):
    # A: (i, k) = af(l16); B: (j, k) = bbf(l16); D: (j, i) = df(l16)
    lane = {}
    for l in range(64):
        b, t = bf(l)
        lane[("A", b) + af(t)] = l                   # A[b][i][k]
        lane[("B", b) + bbf(t)] = l                  # B[b][j][k]
        lane[("D", b) + df(t)] = l                   # D[b][j][i]
    for on, of in orders().items():
        hits = 0
        for A, B, C, D in h:
            for b in range(4):
                for i in range(4):
                    for j in range(4):
                        ld = lane[("D", b, j, i)]
                        a = [A[lane[("A", b, i, k)]] for k in range(4)]
                        bb = [B[lane[("B", b, j, k)]] for k in range(4)]
                        hits += of(a, bb, C[ld]) == D[ld]
        best.append((hits, bn, "A (i, k) = " + an, "B (j, k) = " + bbn, "D (j, i) = " + dn, on))
best.sort(reverse=True)
total = len(h) * 64
for r in best[:8]:
    print(f"{r[0]}/{total}", *r[1:], sep=" | ")
