"""CPU tests of the oracle (oracle/oracle.c) -- pins the parity checker.

The reference ships no golden vectors; the oracle is pinned by
  * the Random123 Philox4x32-10 known-answer vectors,
  * a numpy twin of the stream (independent restatement),
  * accuracy of the deterministic fp64 math against numpy/libm,
  * the reference's own distributional test (KS, test/test_dists.jl:7-47),
  * the reference's finite-difference gradient test (test/dsl/helper_diff.jl:8-37),
  * the README's HMC statistics (README.md:110-154),
  * bookkeeping invariants (SerialMC ranges, continuation, sharding).
"""
import json
import math
import os

import numpy as np
import pytest
from scipy import stats

import mcmchip as mc
import oracle_ref as orc

HERE = os.path.dirname(os.path.abspath(__file__))


# ------------------------------------------------------------------ Philox
def _kat():
    with open(os.path.join(HERE, "golden", "philox_kat.json")) as f:
        return json.load(f)["vectors"]


def test_philox_known_answers():
    for v in _kat():
        ctr = np.array([int(x, 16) for x in v["ctr"]], dtype=np.uint32)
        key = np.array([int(x, 16) for x in v["key"]], dtype=np.uint32)
        out = orc.philox(ctr, key)[0]
        assert [format(int(x), "08x") for x in out] == v["out"]


def philox_numpy(ctr, key):
    """Independent numpy restatement of Philox4x32-10 (Salmon et al. 2011)."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = key[:, 0].astype(np.uint64), key[:, 1].astype(np.uint64)
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    mask = np.uint64(0xFFFFFFFF)
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(0x9E3779B9)) & mask
            k1 = (k1 + np.uint64(0xBB67AE85)) & mask
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & mask, p1 & mask, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & mask,
             p0 & mask]
    return np.stack(c, axis=1).astype(np.uint32)


def test_philox_matches_numpy_twin():
    rng = np.random.default_rng(7)
    ctr = rng.integers(0, 2**32, size=(5000, 4), dtype=np.uint64).astype(np.uint32)
    key = rng.integers(0, 2**32, size=(5000, 2), dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(orc.philox(ctr, key), philox_numpy(ctr, key))


# ------------------------------------------------------------------ deterministic math
def _ulps(a, b):
    return np.abs(a - b) / np.spacing(np.maximum(np.abs(b), np.finfo(float).tiny))


def test_det_log_accuracy():
    rng = np.random.default_rng(0)
    for lo, hi in [(1e-300, 1e-200), (0.3, 3.0), (2.0, 1e10), (1e-320, 1e-310)]:
        x = rng.uniform(lo, hi, 100000)
        assert _ulps(orc.detmath(0, x), np.log(x)).max() <= 1.0
    sp = orc.detmath(0, np.array([0.0, -0.0, -1.0, np.inf, np.nan, 1.0]))
    assert sp[0] == -np.inf and sp[1] == -np.inf and np.isnan(sp[2]) and sp[3] == np.inf and np.isnan(sp[4])
    assert sp[5] == 0.0


def test_det_exp_accuracy():
    rng = np.random.default_rng(1)
    x = rng.uniform(-700, 700, 100000)
    assert _ulps(orc.detmath(1, x), np.exp(x)).max() <= 1.0
    sp = orc.detmath(1, np.array([0.0, -1000.0, 1000.0, np.nan, -np.inf, np.inf]))
    assert sp[0] == 1.0 and sp[1] == 0.0 and sp[2] == np.inf and np.isnan(sp[3]) and sp[4] == 0 and sp[5] == np.inf


def test_exp_tab_accuracy():
    """det_exp_tab (logistic likelihood; table-driven, degree-6 polynomial): <= 1 ulp over the normal range;
    inf / 0 / NaN at the ends, as det_exp."""
    rng = np.random.default_rng(13)
    x = np.concatenate([rng.uniform(-708, 709.7, 200000), rng.uniform(-40, 40, 200000)])
    assert _ulps(orc.detmath(13, x), np.exp(x)).max() <= 1.0
    sp = orc.detmath(13, np.array([0.0, -1000.0, 1000.0, np.nan, -np.inf, np.inf, 710.0, -746.0]))
    assert sp[0] == 1.0 and sp[1] == 0.0 and sp[2] == np.inf and np.isnan(sp[3]) and sp[4] == 0.0
    assert sp[5] == np.inf and sp[6] == np.inf and sp[7] == 0.0


def test_log_tab_accuracy():
    """det_log_tab (logistic Bernoulli term; bm_log_u32's table for any double in [0, 1]): <= 1 ulp,
    subnormals included; log(0) = -inf, log(1) = 0, NaN passes."""
    rng = np.random.default_rng(14)
    v = np.concatenate([np.exp(rng.uniform(-744, 0, 200000)), rng.uniform(0, 1, 200000),
                        1 - np.exp(rng.uniform(-36, -1, 100000)), rng.uniform(5e-324, 2.2e-308, 20000)])
    v = v[v > 0]
    assert _ulps(orc.detmath(14, v), np.log(v)).max() <= 1.0
    sp = orc.detmath(14, np.array([0.0, 1.0, np.nan, 0.5]))
    assert sp[0] == -np.inf and sp[1] == 0.0 and np.isnan(sp[2]) and sp[3] == np.log(0.5)

def test_logistic_term_accuracy():
    """det_logi (round 5; the logistic Bernoulli term from one degree-9 segment polynomial and its derivative):
    term = -softplus(u) and rv = w sigmoid(u), u = -w eta, against extended precision: the term within 2 ulp plus
    2^-57 absolute (|u| > 40 holds f at f(40)), the weight within 3 ulp plus 2^-57 absolute, for both link signs
    and both responses (w = s (2y - 1))."""
    rng = np.random.default_rng(21)
    eta = np.concatenate([rng.uniform(-45, 45, 200000), rng.normal(0, 3, 100000), rng.uniform(-800, 800, 20000),
                          np.array([0.0, -0.0, 40.0, -40.0, 1e-300, 36.7368, 800.0])])
    L = np.longdouble
    for w in (1.0, -1.0):
        ww = np.full_like(eta, w)
        term, rv = orc.detmath(22, eta, ww), orc.detmath(23, eta, ww)
        u = -(w * eta).astype(L)
        sp = np.maximum(u, 0) + np.log1p(np.exp(-np.abs(u)))           # softplus(u)
        sig = 1 / (1 + np.exp(-u))
        t_ref, r_ref = (-sp).astype(float), (w * sig).astype(float)
        assert (np.abs(term - t_ref) <= 2 * np.spacing(np.abs(t_ref)) + 2.0**-57).all()
        assert (np.abs(rv - r_ref) <= 3 * np.spacing(np.abs(r_ref)) + 2.0**-57).all()
    # at u = 0 both branches of the weight give exactly 1/2; the term is -log 2
    assert orc.detmath(23, np.array([0.0, -0.0]), np.array([1.0, 1.0])).tolist() == [0.5, 0.5]
    assert orc.detmath(22, np.array([0.0]), np.array([-1.0]))[0] == -np.log(2.0)


@pytest.mark.parametrize("y", [0.0, 1.0])
def test_logistic_reference_minus_inf_rule(y):
    """The reference's p = 1/(1+exp(-X beta)) rounds to 1 (y = 0: log(1 - p) = -Inf) for X beta >= RU(53 ln 2) and
    to 0 (y = 1: log(p) = -Inf) past exp's overflow threshold; the oracle's evaluation is -Inf (LLAcc: zero gradient)
    from exactly those points on, and finite just before them."""
    T = float.fromhex("0x1.25e4f7b2737fbp+5") if y == 0.0 else float.fromhex("0x1.62e42fefa39f0p+9")
    sgn_eta = T if y == 0.0 else -T                         # u = -w eta = s eta (y = 0), -s eta (y = 1)
    X = np.array([[1.0], [1.0]])
    m = mc.model(mc.LogisticRegression(X, np.array([y, 1.0 - y]), prior_sigma=1e6), vars=np.zeros(1), gradient=True)
    pts = np.array([[sgn_eta, np.nextafter(sgn_eta, 0.0)]])
    lp, g = orc.eval_batch(m, pts)
    assert lp[0] == -np.inf and g[0, 0] == 0.0
    assert np.isfinite(lp[1]) and g[0, 1] != 0.0


def test_det_sincos2pi_accuracy():
    rng = np.random.default_rng(2)
    u = np.floor(rng.uniform(0, 2**32, 100000)) * 2.0**-32
    s, c = orc.detmath(2, u), orc.detmath(3, u)
    assert np.abs(s - np.sin(2 * np.pi * u)).max() < 2e-15
    assert np.abs(c - np.cos(2 * np.pi * u)).max() < 2e-15
    q = orc.detmath(2, np.array([0.0, 0.25, 0.5, 0.75]))
    assert np.allclose(q, [0, 1, 0, -1], atol=1e-16)


def test_sincos2pi_u32_accuracy():
    """Box-Muller angle sin/cos(2 pi w 2^-32), table-driven: within 4.5e-16 (2 ulp of 1) of a long-double reference,
    exact at the table nodes, including the wrap at w -> 2^32."""
    rng = np.random.default_rng(12)
    w = np.concatenate([np.floor(rng.uniform(0, 2**32, 300000)), np.arange(0, 3000), 2.0**32 - 1 - np.arange(0, 3000),
                        (np.arange(-40, 40) + 2.0**23 * np.arange(1, 512, 2)[:, None]).ravel() % 2**32])
    s, c = orc.detmath(10, w), orc.detmath(11, w)
    a = 2 * np.pi * (w.astype(np.longdouble) * np.longdouble(2.0)**-32)
    assert np.abs(s - np.sin(a)).max() < 4.5e-16
    assert np.abs(c - np.cos(a)).max() < 4.5e-16
    k = np.arange(0, 256) * 2.0**24
    np.testing.assert_array_equal(orc.detmath(10, k[[0, 64, 128, 192]]), [0.0, 1.0, 0.0, -1.0])


def test_round_ties_away_from_zero():
    x = np.array([0.5, 1.5, 2.5, -0.5, -2.5, 2.4999999999, 0.49999999999999994, 3.0])
    assert list(orc.detmath(7, x)) == [1, 2, 3, -1, -3, 2, 0, 3]      # Julia 0.2 round (HMCDA.jl:104)


def test_normals_are_standard_normal():
    n = 50000
    z = orc.detmath(6, np.arange(n, dtype=float), np.full(n, 3.0)).reshape(-1)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert stats.kstest(z, "norm").pvalue > 1e-3
    # 32-bit Box-Muller radius bound: sqrt(-2 log(2^-33)) = 6.76
    assert np.abs(z).max() < 6.77


def test_uniform52_range():
    u = orc.detmath(8, np.arange(20000, dtype=float))
    assert u.min() >= 0.0 and u.max() < 1.0
    assert stats.kstest(u, "uniform").pvalue > 1e-3


# ------------------------------------------------------------------ models
@pytest.mark.parametrize("mk", ["iso", "normal"])
def test_gradient_finite_difference(mk):
    """helper_diff.jl:8-37: DIFF_DELTA = 1e-9, relative error threshold 2e-2."""
    d = 5
    m = (mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True) if mk == "iso"
         else mc.model(mc.NormalDSL(1.0, 2.0), v=np.ones(d), gradient=True))
    rng = np.random.default_rng(3)
    x0 = rng.normal(size=(d, 4))
    lp0, g0 = orc.eval_batch(m, x0)
    delta = 1e-9
    for j in range(d):
        x1 = x0.copy()
        x1[j] += delta
        lp1, _ = orc.eval_batch(m, x1)
        gn = (lp1 - lp0) / delta
        err = np.abs(g0[j] - gn) / np.maximum(2e-2, np.abs(g0[j]))
        assert (err < 2e-2).all()


def test_normal_dsl_logpdf_and_out_of_support():
    m = mc.model(mc.NormalDSL(1.0, 2.0), v=np.zeros(3), gradient=True)
    x = np.array([[0.3], [-1.0], [2.5]])
    lp, g = orc.eval_batch(m, x)
    assert np.isclose(lp[0], stats.norm(1, 2).logpdf(x[:, 0]).sum(), rtol=1e-14)
    assert np.allclose(g[:, 0], (1.0 - x[:, 0]) / 4.0, rtol=1e-15)
    # LLAcc: a non-finite running sum -> (-Inf, zeros) (AccumulatorDerivRules.jl:14-16, modelparser.jl:68)
    lp, g = orc.eval_batch(m, np.array([[np.inf], [0.0], [0.0]]))
    assert lp[0] == -np.inf and (g == 0).all()


# ------------------------------------------------------------------ samplers: statistics
def _pool(samples, every=1):
    return samples[::every].reshape(-1)


@pytest.mark.parametrize("mu,sd", [(1.0, 1.0), (3.0, 12.0)])
@pytest.mark.parametrize("which", ["RWM", "HMC", "MALA"])
def test_ks_like_reference(mu, sd, which):
    """test_dists.jl:24-47: RWM(std), HMC(2, std/5), MALA(std) on x ~ Normal(mu, sd), SerialMC(1000:N),
    KS measure below the reference's threshold 10; here over 64 chains, one kept sample per chain and
    per 50 steps, against the 5 % critical value."""
    sampler = {"RWM": mc.RWM(sd), "HMC": mc.HMC(2, sd / 5), "MALA": mc.MALA(sd)}[which]
    m = mc.model(mc.NormalDSL(mu, sd), x=mu, gradient=True)
    oc = orc.OracleChains(m, sampler, nchains=64, seed=11)
    r = mc.SerialMC(range(1000, 6001))
    s, _, _ = oc.run(r)
    x = s[::50, 0, :].reshape(-1)                         # 101 x 64 draws, nearly independent
    xs = np.sort(x)
    dn = np.max(np.abs(np.arange(1, len(x) + 1) / len(x) - stats.norm(mu, sd).cdf(xs)))
    ksv = math.sqrt(len(x)) * dn
    assert ksv < 10.0                                      # the reference's KSTHRESHOLD (test_dists.jl:13)
    assert ksv < 2.5                                       # and a meaningful bound


def test_readme_hmc_statistics():
    """README.md:110-154: HMC(0.75) on -dot(v,v), d=3, SerialMC(steps=10000, burnin=1000): acceptance 79.76 %,
    AC time 1.687 -- the reference's numbers come from one dSFMT chain; here the mean over 16 Philox chains."""
    m = mc.model(mc.IsoNormalDot(), init=np.ones(3), grad=True)
    oc = orc.OracleChains(m, mc.HMC(0.75), nchains=16, seed=5)
    r = mc.SerialMC(steps=10000, burnin=1000)
    s, _, acc = oc.run(r)
    rate = acc.mean() * 100
    assert abs(rate - 79.76) < 1.5
    chain = type("C", (), {})()
    chain.samples = np.transpose(s, (2, 0, 1))
    act = mc.actime(chain)
    assert abs(act.mean() - 1.687) < 0.15
    assert np.allclose(s.reshape(-1, 3 * 16).std(axis=0), math.sqrt(0.5), atol=0.05)   # N(0, I/2)


def test_hmcda_adapts_towards_target_rate():
    m = mc.model(mc.IsoNormalDot(), init=np.ones(8), grad=True)
    oc = orc.OracleChains(m, mc.HMCDA(rate=0.65, len=1.0), nchains=32, seed=2)
    _, _, acc = oc.run(mc.SerialMC(steps=3000, burnin=1000))
    assert abs(acc.mean() - 0.65) < 0.1
    assert (oc.t_step == oc.t_bar).all()                    # after burn-in leapStep = dualLeapStep


def test_tuned_mala_and_hmc_adapt():
    m = mc.model(mc.NormalDSL(0.0, 1.0), v=np.zeros(4), gradient=True)
    oc = orc.OracleChains(m, mc.MALA(5.0, mc.EmpMCTuner(0.6, adaptStep=50)), nchains=16, seed=3)
    _, _, acc = oc.run(mc.SerialMC(steps=2000, burnin=1000))
    assert abs(acc.mean() - 0.6) < 0.15
    assert (oc.t_step != 5.0).all()
    oc = orc.OracleChains(m, mc.HMC(10, 2.0, mc.EmpMCTuner(0.7, adaptStep=50, maxStep=40)), nchains=16, seed=3)
    _, _, acc = oc.run(mc.SerialMC(steps=2000, burnin=1000))
    assert (oc.t_leaps <= 40).all() and (oc.t_leaps >= 1).all()


# ------------------------------------------------------------------ bookkeeping invariants
def test_serialmc_ranges():
    r = mc.SerialMC(steps=1000, burnin=100)
    assert (r.burnin, r.thinning, r.len, len(r.r)) == (100, 1, 1000, 900)
    r = mc.SerialMC(steps=1000, burnin=100, thinning=5)
    assert len(r.r) == 180 and r.r[0] == 101
    r = mc.SerialMC(range(101, 1001, 5))                    # SerialMC(101:5:1000)
    assert (r.burnin, r.thinning, r.len, len(r.r)) == (100, 5, 996, 180)
    with pytest.raises(AssertionError, match="Burnin rounds"):
        mc.SerialMC(steps=10, burnin=-1)
    with pytest.raises(AssertionError, match="Total MCMC length"):
        mc.SerialMC(steps=10, burnin=10)
    with pytest.raises(AssertionError, match="Thinning"):
        mc.SerialMC(steps=10, thinning=0)


def test_kept_steps_store_post_step_state():
    m = mc.model(mc.IsoNormalDot(), init=np.ones(3))
    oc = orc.OracleChains(m, mc.RWM(0.5), nchains=5, seed=4)
    s_all, _, a_all = oc.run(mc.SerialMC(steps=30))
    oc2 = orc.OracleChains(m, mc.RWM(0.5), nchains=5, seed=4)
    s_thin, _, a_thin = oc2.run(mc.SerialMC(steps=30, burnin=4, thinning=7))
    idx = np.arange(4, 30, 7)                                  # kept steps 5, 12, 19, 26 (1-based)
    assert np.array_equal(s_thin, s_all[idx]) and np.array_equal(a_thin, a_all[idx])
    assert np.array_equal(oc.x, oc2.x)


def test_continuation_equals_one_long_run():
    """run(chain) continues the same Markov chain (runners.jl:14): the counter-based stream makes
    two runs of 40 steps bit-identical to the last 40 of one 80-step run."""
    m = mc.model(mc.NormalDSL(0.5, 1.5), v=np.zeros(6), gradient=True)
    for sp in (mc.RWM(0.7), mc.MALA(0.3), mc.HMC(4, 0.3), mc.HMCDA(len=1.0)):
        a = orc.OracleChains(m, sp, nchains=7, seed=9)
        a.run(mc.SerialMC(steps=40, burnin=0))
        s2, _, acc2 = a.run(mc.SerialMC(steps=40, burnin=0))
        b = orc.OracleChains(m, sp, nchains=7, seed=9)
        s, _, acc = b.run(mc.SerialMC(steps=80, burnin=0))
        assert np.array_equal(s2, s[40:]) and np.array_equal(acc2, acc[40:])


def test_sharding_is_invisible():
    """Chains keyed by global id: two shards with chain_offset reproduce one batch."""
    m = mc.model(mc.IsoNormalDot(), init=np.ones(4), grad=True)
    full = orc.OracleChains(m, mc.HMC(3, 0.2), nchains=10, seed=8)
    s, _, acc = full.run(mc.SerialMC(steps=25, burnin=5))
    lo = orc.OracleChains(m, mc.HMC(3, 0.2), nchains=6, seed=8, chain_offset=0)
    hi = orc.OracleChains(m, mc.HMC(3, 0.2), nchains=4, seed=8, chain_offset=6)
    s_lo, _, a_lo = lo.run(mc.SerialMC(steps=25, burnin=5))
    s_hi, _, a_hi = hi.run(mc.SerialMC(steps=25, burnin=5))
    assert np.array_equal(np.concatenate([s_lo, s_hi], axis=2), s)
    assert np.array_equal(np.concatenate([a_lo, a_hi], axis=1), acc)


def test_wave_order_reduction_is_a_sum():
    """order 1 (wave-per-chain kernels) changes only the summation order."""
    m = mc.model(mc.NormalDSL(0.2, 1.3), v=np.zeros(300), gradient=True)
    x = np.random.default_rng(5).normal(size=(300, 3))
    lp0, g0 = orc.eval_batch(m, x, order=0)
    lp1, g1 = orc.eval_batch(m, x, order=1)
    assert np.allclose(lp0, lp1, rtol=1e-13) and np.array_equal(g0, g1)


def _fma(a, b, c):
    """correctly rounded a*b + c (Python 3.10 has no math.fma): exact rational arithmetic, one rounding"""
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


@pytest.mark.parametrize("d", [17, 20, 24, 29, 32])
def test_pair_order_is_the_two_halves(d):
    """ORDER_PAIR (two lanes per chain, 16 < d <= 32): the first 4 ceil(ceil(d/4)/2) coordinates left to right, the
    rest left to right, then the two partial sums -- restated here in that exact order, bitwise (fma chains as the
    kernels form them); it is also the default order at these widths (oracle_ref.kernel_order), RAM included."""
    x = np.random.default_rng(d).normal(size=(d, 5))
    S = 4 * ((((d + 3) // 4) + 1) // 2)
    m_iso = mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    lp, _ = orc.eval_batch(m_iso, x, order=orc.ORDER_PAIR)
    lp0, _ = orc.eval_batch(m_iso, x, order=0)
    for c in range(5):
        a = b = 0.0
        for j in range(d):
            if j < S:
                a = _fma(x[j, c], x[j, c], a)
            else:
                b = _fma(x[j, c], x[j, c], b)
        assert lp[c] == -(a + b)
        seq = 0.0
        for j in range(d):
            seq = _fma(x[j, c], x[j, c], seq)
        assert lp0[c] == -seq
    assert orc.kernel_order(m_iso, 1) == orc.ORDER_PAIR == orc.kernel_order(m_iso, 5)
    assert np.array_equal(orc.eval_batch(m_iso, x)[0], lp)           # the default is the library's order


@pytest.mark.parametrize("d", [33, 70, 128, 129, 256])
def test_half_wave_order_is_a_32_lane_butterfly(d):
    """ORDER_HALF (RAM on separable targets, 32 < d <= 256, two chains per wave): lane l of the chain's 32 owns
    coordinates 4 (l + 32 k) + e, an fma chain per lane in (k, e) order, then the xor butterfly 16, 8, 4, 2, 1 --
    restated here lane by lane, bitwise; the default order of RAM at these widths, the other samplers keep order 1."""
    x = np.random.default_rng(d).normal(size=(d, 3))
    m_iso = mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    lp, _ = orc.eval_batch(m_iso, x, order=orc.ORDER_HALF)
    for c in range(3):
        p = []
        for lane in range(32):
            a = 0.0
            for j0 in range(4 * lane, d, 128):
                for e in range(4):
                    if j0 + e < d:
                        a = _fma(x[j0 + e, c], x[j0 + e, c], a)
            p.append(a)
        for off in (16, 8, 4, 2, 1):
            p = [p[lane] + p[lane ^ off] for lane in range(32)]
        assert lp[c] == -p[0]
    assert orc.kernel_order(m_iso, 5) == orc.ORDER_HALF
    assert orc.kernel_order(m_iso, 1) == 1 == orc.kernel_order(m_iso)


def test_half_wave_ram_initial_lp_in_eval_order():
    """RAM chains at 33 <= d <= 256 start from the eval kernel's log-target (order 1, oracle.c orc_eval_order):
    a zero-step run leaves the oracle's lp equal to eval_batch in order 1."""
    d = 90
    x0 = np.random.default_rng(3).normal(size=d)
    m = mc.model(mc.IsoNormalDot(), init=x0, grad=True)
    oc = orc.OracleChains(m, mc.RAM(), nchains=3, seed=1)
    assert oc.order == orc.ORDER_HALF
    lp1, _ = orc.eval_batch(m, np.repeat(x0[:, None], 3, axis=1), order=1)
    assert np.array_equal(oc.lp, lp1)


def test_init_out_of_support_raises():
    m = mc.model(mc.NormalDSL(0.0, 1.0), v=np.zeros(2), gradient=True)
    with pytest.raises(AssertionError, match="out of model support"):
        orc.OracleChains(m, mc.RWM(0.1), nchains=2, init_x=np.array([[np.inf, 0.0], [0.0, 0.0]]))


# ------------------------------------------------------------------ regression models
def _logistic_data(n, d, seed=0, sign=1.0):
    """examples/logistic_regression.jl:10-13 with the build's synthetic generator (numpy here)."""
    rng = np.random.default_rng(seed)
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1))])
    beta0 = rng.normal(size=d)
    Y = (rng.random(n) < 1 / (1 + np.exp(-sign * (X @ beta0)))).astype(float)
    return X, Y


def _linear_data(n, d, seed=0):
    rng = np.random.default_rng(seed)
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1))])
    beta0 = rng.normal(size=d)
    return X, X @ beta0 + rng.normal(size=n)


@pytest.mark.parametrize("d", [10, 37, 130, 300])
def test_logistic_eval_matches_closed_form(d):
    X, Y = _logistic_data(200, d, seed=d)
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)
    B = np.random.default_rng(1).normal(size=(d, 5)) * 0.1
    lp, g = orc.eval_batch(m, B)
    eta = X @ B
    p = 1 / (1 + np.exp(-eta))
    ll = (Y[:, None] * np.log(p) + (1 - Y[:, None]) * np.log(1 - p)).sum(0)
    prior = stats.norm.logpdf(B).sum(0)
    np.testing.assert_allclose(lp, ll + prior, rtol=1e-12)
    np.testing.assert_allclose(g, -B + X.T @ (Y[:, None] - p), rtol=1e-9, atol=1e-11)


def test_logistic_link_sign_variant():
    """test/test_syntax.jl:13,18 writes prob = 1/(1+exp(X*vars))."""
    X, Y = _logistic_data(100, 6, seed=3, sign=-1.0)
    m = mc.model(mc.LogisticRegression(X, Y, link_sign=-1.0), vars=np.zeros(6), gradient=True)
    B = np.random.default_rng(2).normal(size=(6, 3)) * 0.2
    lp, g = orc.eval_batch(m, B)
    p = 1 / (1 + np.exp(X @ B))
    ll = (Y[:, None] * np.log(p) + (1 - Y[:, None]) * np.log(1 - p)).sum(0)
    np.testing.assert_allclose(lp, ll + stats.norm.logpdf(B).sum(0), rtol=1e-12)
    np.testing.assert_allclose(g, -B - X.T @ (Y[:, None] - p), rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("d", [10, 200])
def test_linear_eval_matches_closed_form(d):
    X, Y = _linear_data(150, d, seed=d)
    m = mc.model(mc.LinearRegression(X, Y, prior_sigma=1.5, noise_sigma=0.7), vars=np.zeros(d), gradient=True)
    B = np.random.default_rng(4).normal(size=(d, 4)) * 0.1
    lp, g = orc.eval_batch(m, B)
    R = Y[:, None] - X @ B
    np.testing.assert_allclose(lp, stats.norm(0, 0.7).logpdf(R).sum(0) + stats.norm(0, 1.5).logpdf(B).sum(0),
                               rtol=1e-12)
    np.testing.assert_allclose(g, -B / 1.5**2 + X.T @ R / 0.7**2, rtol=1e-9, atol=1e-10)


def test_glm_gradient_finite_difference():
    """helper_diff.jl:8-37 on the Bernoulli and Normal-residual rules (test_diff.jl:14,47)."""
    for kind in ("logistic", "linear"):
        d = 6
        X, Y = _logistic_data(80, d) if kind == "logistic" else _linear_data(80, d)
        tgt = mc.LogisticRegression(X, Y) if kind == "logistic" else mc.LinearRegression(X, Y)
        m = mc.model(tgt, vars=np.zeros(d), gradient=True)
        x0 = np.random.default_rng(5).normal(size=(d, 1)) * 0.3
        lp0, g0 = orc.eval_batch(m, x0)
        for j in range(d):
            x1 = x0.copy()
            x1[j] += 1e-7
            gn = (orc.eval_batch(m, x1)[0] - lp0) / 1e-7
            assert abs(g0[j, 0] - gn[0]) / max(2e-2, abs(g0[j, 0])) < 2e-2


def test_logistic_out_of_support():
    """p rounds to 1 with Y = 0: log(1-p) = -Inf -> LLAcc throws -> (-Inf, zeros)."""
    X = np.array([[1.0, 50.0], [1.0, -1.0]])
    Y = np.array([0.0, 1.0])
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(2), gradient=True)
    lp, g = orc.eval_batch(m, np.array([[0.0], [1.0]]))
    assert lp[0] == -np.inf and (g == 0).all()


def test_mala_logistic_recovers_posterior_mean():
    X, Y = _logistic_data(400, 4, seed=9)
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(4), gradient=True)
    oc = orc.OracleChains(m, mc.MALA(0.02), nchains=8, seed=3)
    s, _, acc = oc.run(mc.SerialMC(steps=3000, burnin=1000, thinning=5))
    post = s.mean(axis=(0, 2))
    # Laplace approximation of the posterior mean by Newton's method
    b = np.zeros(4)
    for _ in range(50):
        p = 1 / (1 + np.exp(-X @ b))
        gr = X.T @ (Y - p) - b
        H = -(X.T * (p * (1 - p))) @ X - np.eye(4)
        b = b - np.linalg.solve(H, gr)
    sd = np.sqrt(np.diag(np.linalg.inv(-H)))
    assert np.all(np.abs(post - b) < 0.25 * sd + 0.02)
    assert 0.2 < acc.mean() < 0.99


def test_ess_quotient_is_ieee_division(tmp_path):
    """k_ess_reg divides the autocovariance sums by n as two fmas around rn = 1/n (Markstein's correction); orc_ess
    uses the IEEE division.  Bitwise the same on 4 million quotients (n = 1..1024, near-exact ones included); the
    GPU ESS tests then compare the kernel with orc_ess on real series."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = os.path.join(os.path.dirname(__file__), "qdiv_check.c")
    exe = str(tmp_path / "qdiv_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"], check=True)
    r = subprocess.run([exe, "1024", "4000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("vtype,name", [(1, "imse"), (2, "ipse"), (3, "bm")])
@pytest.mark.parametrize("phi", [0.0, 0.7, 0.95, -0.5])
def test_oracle_ess_matches_numpy_stats(vtype, name, phi):
    """orc_ess restates ess.jl / var.jl; numpy stats.py (FFT autocovariances) agrees to rounding."""
    import mcmchip as mc
    rng = np.random.default_rng(5)
    n, d, C = 180, 2, 7
    e = rng.normal(size=(n, d, C))
    x = np.zeros_like(e)
    x[0] = e[0]
    for t in range(1, n):
        x[t] = phi * x[t - 1] + e[t]
    eo, vo = orc.ess(x, vtype, 0, 30)
    chain = type("Chain", (), {})()
    chain.samples = np.transpose(x, (2, 0, 1))
    kw = {"batchlen": 30} if name == "bm" else {}
    en = mc.stats.ess(chain, name, **kw)
    np.testing.assert_allclose(eo.T, en, rtol=1e-10)
    if phi == 0.7 and name == "imse":            # AR(1): ESS ~ n (1 - phi) / (1 + phi)
        assert abs(np.mean(eo) / (n * 0.3 / 1.7) - 1) < 0.35


def test_bm_log_u32_accuracy():
    """Box-Muller radius log((w + 1/2) 2^-32): <= 1 ulp against numpy's log, including near u = 1 and u -> 0."""
    rng = np.random.default_rng(9)
    w = np.concatenate([np.floor(rng.uniform(0, 2**32, 300000)), np.arange(0, 5000), 2.0**32 - 1 - np.arange(0, 5000),
                        (np.arange(-64, 64) + 2.0**26 * np.arange(1, 64)[:, None]).ravel()])
    got = orc.detmath(9, w)
    ref = np.log((w + 0.5) * 2.0**-32)
    err = np.abs(got - ref) / np.spacing(np.abs(ref))
    assert err.max() <= 1.0


def test_bm_radius_accuracy():
    """The Box-Muller radius sqrt(-2 log u), u = (w + 1/2) 2^-32, from the segment polynomials (op 17): every draw of
    the tail table's binades (v < 2^21 on both sides, 2^22 draws), 2 M random draws of the main table and every
    segment's ends, against an 80-bit long-double sqrt(-2 log u) (side 1: log1p(-(v + 1/2) 2^-32)).  a0 is one double
    (scripts/gen_bm_log_table.py), so the bound is its rounding plus the final one: <= 1 ulp, except on the few
    segments whose radius crosses a power of two, where a0's ulp is the coarser one (<= 1.4 ulp measured)."""
    rng = np.random.default_rng(17)
    e, k = np.meshgrid(np.arange(21, 31), np.arange(32))
    ends = (2 ** e * (1 + k / 32)).ravel().astype(np.int64)
    v = np.concatenate([np.arange(0, 2**21), rng.integers(2**21, 2**31, 2_000_000), ends - 1, ends, [2**31 - 1]])
    x = v.astype(np.longdouble) + np.longdouble(0.5)
    u = x * np.longdouble(2.0) ** -32
    for side, ref in ((0, np.sqrt(-2 * np.log(u))), (1, np.sqrt(-2 * np.log1p(-u)))):
        w = v if side == 0 else 2**32 - 1 - v
        got = orc.detmath(17, w.astype(np.float64))
        err = np.abs((got.astype(np.longdouble) - ref) / np.spacing(ref.astype(np.float64))).astype(np.float64)
        assert err.max() <= 1.45, (side, err.max(), v[np.argmax(err)])
        big = err > 1.0
        lg = np.log2(got[big])
        assert np.all(np.abs(lg - np.round(lg)) < 0.01), "above 1 ulp away from a power of two"
        assert err.mean() < 0.36


def test_abs_normal_dsl_closed_form_and_gradient():
    """y = abs(x); y ~ Normal(mu, sigma) (README.md:246-251): lp = sum logpdf(Normal, |x|), grad = sign(x) (mu-|x|)/s^2."""
    mu, sig = 1.0, 0.7
    m = mc.model(mc.AbsNormalDSL(mu, sig), x=np.zeros(5), gradient=True)
    x = np.array([[-1.3, 0.2, 2.0, -0.4, 1.1], [0.5, -0.5, 3.0, 1.0, -2.2]]).T
    lp, g = orc.eval_batch(m, x)
    ref = stats.norm.logpdf(np.abs(x), mu, sig).sum(axis=0)
    np.testing.assert_allclose(lp, ref, rtol=1e-13)
    np.testing.assert_allclose(g, np.sign(x) * (mu - np.abs(x)) / sig**2, rtol=1e-13)
    h = 1e-6
    for j in range(5):
        e = np.zeros((5, 1)); e[j] = h
        fd = (orc.eval_batch(m, x[:, :1] + e)[0] - orc.eval_batch(m, x[:, :1] - e)[0]) / (2 * h)
        assert abs(fd[0] - g[j, 0]) < 1e-6


DIST_CASES = [
    ("Normal", (0.3, 1.7), lambda p: stats.norm(p[0], p[1]), (-2.0, 2.0)),
    ("Uniform", (-1.0, 2.0), lambda p: stats.uniform(p[0], p[1] - p[0]), (-0.9, 1.9)),
    ("Weibull", (1.5, 2.0), lambda p: stats.weibull_min(p[0], scale=p[1]), (0.1, 4.0)),
    ("Beta", (2.0, 3.0), lambda p: stats.beta(p[0], p[1]), (0.05, 0.95)),
    ("TDist", (3.0,), lambda p: stats.t(p[0]), (-3.0, 3.0)),
    ("Exponential", (1.5,), lambda p: stats.expon(scale=p[0]), (0.1, 4.0)),
    ("Gamma", (2.5, 0.7), lambda p: stats.gamma(p[0], scale=p[1]), (0.1, 4.0)),
    ("Cauchy", (0.5, 1.3), lambda p: stats.cauchy(p[0], p[1]), (-3.0, 3.0)),
    ("LogNormal", (0.2, 0.6), lambda p: stats.lognorm(p[1], scale=np.exp(p[0])), (0.1, 4.0)),
    ("Laplace", (0.4, 0.9), lambda p: stats.laplace(p[0], p[1]), (-2.0, 2.0)),
]


@pytest.mark.parametrize("name,params,ref,rng_", DIST_CASES, ids=[c[0] for c in DIST_CASES])
def test_dist_dsl_logpdf_gradient_and_support(name, params, ref, rng_):
    """v ~ Dist(p1, p2) (MCMCDerivRules.jl:56-104): logpdf vs scipy, the x-derivative rule vs finite
    differences, and -Inf with zero gradient outside the support (LLAcc)."""
    d = 6
    m = mc.model(mc.DistDSL(name, *params), v=np.full(d, 0.5 if name == "Beta" else 1.0), gradient=True)
    x = np.random.default_rng(7).uniform(*rng_, size=(d, 9))
    lp, g = orc.eval_batch(m, x)
    np.testing.assert_allclose(lp, ref(params).logpdf(x).sum(axis=0), rtol=1e-12, atol=1e-12)
    h = 1e-6
    for j in range(d):
        e = np.zeros((d, 1))
        e[j] = h
        fd = (orc.eval_batch(m, x[:, :1] + e)[0] - orc.eval_batch(m, x[:, :1] - e)[0]) / (2 * h)
        if name != "Uniform":
            assert abs(fd[0] - g[j, 0]) < 1e-5 * max(1.0, abs(g[j, 0]))
    lo = {"Uniform": -1.5, "Weibull": -0.5, "Beta": 1.5, "Exponential": -0.1, "Gamma": -1.0, "LogNormal": -0.1}
    if name in lo:
        xo = x[:, :1].copy()
        xo[2] = lo[name]
        lpo, go = orc.eval_batch(m, xo)
        assert lpo[0] == -np.inf and np.all(go == 0.0)


def test_erfc_and_normal_logcdf_accuracy():
    """The probit model's erfc and logcdf(Normal(), z) (oracle/detmath.h orc_erfc / orc_normlogcdf; the device's
    det_erfc / det_normlogcdf are bitwise the same, test_gpu_parity.py) against 40-digit mpmath: relative error
    <= 8e-16 for erfc wherever it is normal, <= 2e-15 for the log-cdf of the rounded argument z/sqrt2 where
    |logcdf| > 1e-300 (z >= -1), of z itself below (StatsFuns's erfcx form, finite down to z^2 overflow)."""
    import mpmath as mp
    mp.mp.dps = 40
    rng = np.random.default_rng(18)
    x = np.concatenate([rng.uniform(-6, 26, 6000), rng.uniform(-0.6, 0.6, 1000),
                        2.0 ** np.arange(-1, 5)[:, None].ravel(), [0.0, 1e-300, 0.4999999999999999]])
    e = orc.detmath(18, x)
    ref = np.array([float(mp.erfc(mp.mpf(v))) for v in x])
    ok = ref > 2.3e-308
    rel = np.abs(e[ok] - ref[ok]) / ref[ok]
    assert rel.max() <= 8e-16, (rel.max(), x[ok][np.argmax(rel)])
    z = np.concatenate([rng.uniform(-37, 9, 6000), rng.uniform(-1.5, 1.5, 1000), -np.exp(rng.uniform(0, 300, 2000)),
                        [-1.0, np.nextafter(-1.0, 0), 0.0, -181.0, -181.1]])
    lc = orc.detmath(20, z)
    s2 = float.fromhex("0x1.6a09e667f3bcdp-1")   # RN(1/sqrt2): the argument's rounding is amplified by 2 x^2

    def exact(v):
        return mp.log(mp.ncdf(mp.mpf(v))) if v < -1 else mp.log1p(-mp.erfc(mp.mpf(v * s2)) / 2)
    rl = np.array([float(exact(v)) for v in z])
    ok = np.abs(rl) > 1e-300
    rel = np.abs(lc[ok] - rl[ok]) / np.abs(rl[ok])
    assert rel.max() <= 4e-15, (rel.max(), z[ok][np.argmax(rel)])
    assert orc.detmath(20, np.array([-1e200]))[0] == -np.inf
    assert orc.detmath(18, np.array([np.nan, -np.inf, np.inf])).tolist()[1:] == [2.0, 0.0]


# ------------------------------------------------------------------ probit regression (examples/probit_regression.jl)
VASO = os.path.join(os.path.dirname(__file__), "golden", "vaso.txt")     # the example's data file, kept as a fixture


def _probit_reference(X, Y, B, prior_sd=10.0):
    """examples/probit_regression.jl:18-40 restated with scipy: logpdf(MvNormal(0, priorvar I), pars) +
    dot(logcdf(N, X pars), y) + dot(logcdf(N, -X pars), 1 - y), and grad_log_posterior."""
    d = X.shape[1]
    lp, g = [], []
    mvn = stats.multivariate_normal(np.zeros(d), prior_sd**2 * np.eye(d))
    for b in B.T:
        xp = X @ b
        la, lb = stats.norm.logcdf(xp), stats.norm.logcdf(-xp)
        lp.append(mvn.logpdf(b) + la @ Y + lb @ (1 - Y))
        A = -(xp**2 + np.log(2 * np.pi)) / 2
        g.append(X.T @ (Y * np.exp(A - la) - (1 - Y) * np.exp(A - lb)) - b / prior_sd**2)
    return np.array(lp), np.array(g).T


def test_probit_eval_matches_reference_formula_on_vaso():
    """The probit example's own data (vaso.txt, standardised as the example does) and parameter points drawn from
    its prior (randprior, MvNormal(0, 100 I)) and around the posterior: the oracle's log-posterior and gradient
    against the example's formulas evaluated independently (scipy's logcdf and MvNormal)."""
    X, Y = mc.vaso_data(VASO)
    m = mc.model(mc.ProbitRegression(X, Y), vars=np.zeros(3), gradient=True)
    rng = np.random.default_rng(26)
    B = np.hstack([rng.normal(size=(3, 20)) * 10.0, rng.normal(size=(3, 20)) + np.array([[-2.9], [4.6], [3.6]]),
                   np.zeros((3, 1))])
    lp, g = orc.eval_batch(m, B)
    lr, gr = _probit_reference(X, Y, B)
    ok = np.isfinite(lr)
    np.testing.assert_allclose(lp[ok], lr[ok], rtol=1e-12)
    np.testing.assert_allclose(g[:, ok], gr[:, ok], rtol=1e-9, atol=1e-9)


def test_probit_gradient_finite_difference():
    """helper_diff.jl:8-37's check on the probit target."""
    X, Y = mc.vaso_data(VASO)
    m = mc.model(mc.ProbitRegression(X, Y), vars=np.zeros(3), gradient=True)
    x0 = np.array([[-1.0], [2.0], [1.5]])
    lp0, g0 = orc.eval_batch(m, x0)
    for j in range(3):
        x1 = x0.copy()
        x1[j] += 1e-7
        gn = (orc.eval_batch(m, x1)[0] - lp0) / 1e-7
        assert abs(g0[j, 0] - gn[0]) / max(2e-2, abs(g0[j, 0])) < 2e-3


def test_probit_posterior_mean_rwm():
    """The example's first run, RWM(0.5) x SerialMC(1001:10000) (probit_regression.jl:68), on 64 oracle chains from
    the posterior mode's neighbourhood: the pooled posterior mean agrees with a direct quadrature-free estimate, the
    importance-weighted mean of 200 000 prior-free draws from a wide normal (independent of the sampler)."""
    X, Y = mc.vaso_data(VASO)
    m = mc.model(mc.ProbitRegression(X, Y), vars=np.array([-2.0, 3.0, 2.5]), gradient=True)
    oc = orc.OracleChains(m, mc.RWM(0.5), nchains=64, seed=3)
    s, _, acc = oc.run(mc.SerialMC(steps=10000, burnin=1000, thinning=10))
    post = s.mean(axis=(0, 2))
    rng = np.random.default_rng(7)
    cen, sd = np.array([-2.9, 4.6, 3.6]), np.array([1.5, 2.5, 2.0])
    Z = cen + sd * rng.normal(size=(200000, 3))
    lq = stats.norm(cen, sd).logpdf(Z).sum(1)
    lp, _ = orc.eval_batch(m, Z.T)
    w = np.exp(lp - lq - (lp - lq).max())
    ref = (w[:, None] * Z).sum(0) / w.sum()
    np.testing.assert_allclose(post, ref, atol=0.35)
    assert 0.05 < acc.mean() < 0.6


# ------------------------------------------------------------------ y = x * v; y ~ D (bare_distribs.jl)
# benchmarks/benchunits/bare_distribs.jl:29-45: the 17 distributions, each started at its mean (Cauchy: 1.0)
BARE_DISTRIBS = [("Normal", (1, 1)), ("Normal", (3, 12)), ("Weibull", (1, 1)), ("Weibull", (3, 1)),
                 ("Uniform", (0, 2)), ("TDist", (2.2,)), ("TDist", (4,)), ("Beta", (1, 2)), ("Beta", (3, 2)),
                 ("Gamma", (1, 2)), ("Gamma", (3, 0.2)), ("Cauchy", (0, 1)), ("Cauchy", (-1, 0.2)),
                 ("Exponential", (3,)), ("Exponential", (0.2,)), ("LogNormal", (-1, 1)), ("LogNormal", (2, 0.1))]


def _scipy_dist(name, p):
    return {"Normal": lambda: stats.norm(p[0], p[1]), "Weibull": lambda: stats.weibull_min(p[0], scale=p[1]),
            "Uniform": lambda: stats.uniform(p[0], p[1] - p[0]), "TDist": lambda: stats.t(p[0]),
            "Beta": lambda: stats.beta(p[0], p[1]), "Gamma": lambda: stats.gamma(p[0], scale=p[1]),
            "Cauchy": lambda: stats.cauchy(p[0], p[1]), "Exponential": lambda: stats.expon(scale=p[0]),
            "LogNormal": lambda: stats.lognorm(p[1], scale=np.exp(p[0]))}[name]()


def bare_start(name, p):
    m = _scipy_dist(name, p).mean()
    return float(m) if np.isfinite(m) else 1.0                 # bare_distribs.jl:10-12


@pytest.mark.parametrize("name,p", BARE_DISTRIBS)
def test_dist_obs_eval_matches_scipy(name, p):
    """The benchmark unit's model at its start value and around it: lp = sum_i logpdf(D, x v_i) over a 1000-vector v
    (ones, as the unit, and a non-trivial v), gradient sum_i v_i dlogpdf; against scipy, and by finite differences."""
    D = _scipy_dist(name, p)
    x0 = bare_start(name, p)
    for v in (np.ones(1000), np.linspace(0.5, 1.5, 1000)):
        m = mc.model(mc.DistObsDSL(name, *p, v=v), x=x0, gradient=True)
        xs = np.array([[x0, x0 * 0.9, x0 * 1.1 + 0.01]])
        lp, g = orc.eval_batch(m, xs)
        ref = np.array([D.logpdf(x * v).sum() for x in xs[0]])
        ok = np.isfinite(ref)
        np.testing.assert_allclose(lp[ok], ref[ok], rtol=1e-11)
        assert (lp[~ok] == -np.inf).all() and (g[0, ~ok] == 0).all()
        for j in np.nonzero(ok)[0]:
            h = 1e-7 * max(1.0, abs(xs[0, j]))
            lp1, _ = orc.eval_batch(m, xs[:, j:j + 1] + h)
            if np.isfinite(lp1[0]):
                fd = (lp1[0] - lp[j]) / h
                assert abs(g[0, j] - fd) <= 2e-3 * max(1.0, abs(fd)), (name, p, xs[0, j], g[0, j], fd)


# ------------------------------------------------------------------ Ornstein-Uhlenbeck (examples/ornstein.jl:19-30)
def _ou_model(x=None, init=(0.05, 1.0, 1.0)):
    x = mc.ou_series() if x is None else x
    m = mc.model(mc.OrnsteinUhlenbeck(x), tau=init[0], sigma=init[1], mu=init[2], gradient=True)
    m.scale = np.array([1000.0, 1.0, 10.0])                 # ornstein.jl:30
    return m


def _ou_reference(x, B):
    """The example's formulas evaluated independently (numpy / scipy, vectorised): Uniform priors, the residual
    vector, sum(logpdf(Normal(0, sigma), resid)); gradient by hand-derived calculus."""
    out, grads = [], []
    for tau, sigma, mu in B.T:
        if not (0 <= tau <= 100 and 0 <= sigma <= 2 and 0 <= mu <= 20):
            out.append(-np.inf)
            grads.append(np.zeros(3))
            continue
        fac = np.exp(-1.0 / tau)
        r = x[1:] - x[:-1] * fac - mu * (1 - fac)
        out.append(-np.log(100) - np.log(2) - np.log(20) + stats.norm(0, sigma).logpdf(r).sum())
        dr = -r / sigma ** 2
        grads.append(np.array([np.sum(dr * (mu - x[:-1])) * fac / tau ** 2,
                               np.sum((r ** 2 / sigma ** 2 - 1) / sigma),
                               -np.sum(dr) * (1 - fac)]))
    return np.array(out), np.array(grads).T


def test_ou_eval_matches_reference_formula():
    """The oracle's OU log-target and gradient against the example's formulas (ornstein.jl:19-27), at points inside
    and outside the Uniform supports, including the example's init (0.05, 1, 1)."""
    x = mc.ou_series()
    m = _ou_model(x)
    rng = np.random.default_rng(19)
    B = np.column_stack([[0.05, 1.0, 1.0], [20.0, 0.1, 10.0], [100.0, 2.0, 20.0], [-1.0, 1.0, 1.0], [5.0, 2.5, 1.0],
                         [5.0, 1.0, 21.0]])
    B = np.hstack([B, np.vstack([rng.uniform(0.5, 99, 30), rng.uniform(0.05, 2, 30), rng.uniform(0, 20, 30)])])
    lp, g = orc.eval_batch(m, B)
    lr, gr = _ou_reference(x, B)
    assert np.array_equal(np.isfinite(lp), np.isfinite(lr))
    ok = np.isfinite(lr)
    assert not ok[3] and not ok[4] and not ok[5] and ok[2]           # Uniform bounds are closed (a <= x <= b)
    np.testing.assert_allclose(lp[ok], lr[ok], rtol=1e-12)
    np.testing.assert_allclose(g[:, ok], gr[:, ok], rtol=1e-9, atol=1e-9)
    assert np.all(g[:, ~ok] == 0.0)                                  # LLAcc: (-Inf, zero gradient)


def test_ou_gradient_finite_difference():
    """helper_diff.jl:8-37's check on the OU target, away from the support edges."""
    m = _ou_model()
    x0 = np.array([[18.0], [0.12], [9.5]])
    lp0, g0 = orc.eval_batch(m, x0)
    for j, h in enumerate((1e-5, 1e-8, 1e-7)):
        x1 = x0.copy()
        x1[j] += h
        gn = (orc.eval_batch(m, x1)[0] - lp0) / h
        assert abs(g0[j, 0] - gn[0]) / max(1.0, abs(g0[j, 0])) < 2e-3


def test_ou_example_posterior_ram():
    """ornstein.jl:33-34: run(m * RAM() * SerialMC(1000:10000)) from the example's init and scale hint, here on 8
    oracle chains: the posterior recovers the simulating parameters (mu0 = 10, tau0 = 20, sigma0 = 0.1)."""
    m = _ou_model()
    oc = orc.OracleChains(m, mc.RAM(), nchains=8, seed=34)
    s, _, acc = oc.run(mc.SerialMC(steps=10000, burnin=999, thinning=10))
    tail = s[len(s) // 2:]
    tau, sigma, mu = (tail[:, j, :].mean() for j in range(3))
    assert abs(mu - 10.0) < 0.5 and abs(tau - 20.0) < 6.0 and abs(sigma - 0.1) < 0.01, (tau, sigma, mu)
    assert 0.05 < acc[len(acc) // 2:].mean() < 0.6


def test_ou_init_out_of_support():
    m = _ou_model(init=(-1.0, 1.0, 1.0))
    with pytest.raises(AssertionError, match="out of model support"):
        orc.OracleChains(m, mc.RAM(), nchains=2, seed=1)
