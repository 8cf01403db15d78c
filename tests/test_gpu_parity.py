"""GPU parity: the HIP path (through the C ABI) against the oracle on the same seeds.

Bar (BASELINE.json north_star): samples within 1e-10 relative fp64 and accept
bits bit-identical.  The build's arithmetic is specified operation by operation
(DESIGN.md §3-4), so in practice samples are compared bit for bit; the 1e-10
tolerance is the stated fallback and is asserted too.
"""
import os

import numpy as np
import pytest

import mcmchip as mc
from mcmchip import _lib
import oracle_ref as orc

pytestmark = pytest.mark.gpu

RTOL = 1e-10


def _ctx():
    from mcmchip.api import _ctx
    return _ctx(0)


# ------------------------------------------------------------------ math layer
def test_device_philox_known_answers(gpu):
    import json, os, ctypes as ct
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "philox_kat.json")))["vectors"]
    ctr = np.array([[int(x, 16) for x in v["ctr"]] for v in kat], dtype=np.uint32)
    key = np.array([[int(x, 16) for x in v["key"]] for v in kat], dtype=np.uint32)
    out = np.zeros_like(ctr)
    P = ct.POINTER(ct.c_uint32)
    _lib.check(_lib.load().mcmc_debug_philox(_ctx(), len(ctr), ctr.ctypes.data_as(P), key.ctypes.data_as(P),
                                              out.ctypes.data_as(P)))
    assert [[format(int(x), "08x") for x in row] for row in out] == [v["out"] for v in kat]
    rng = np.random.default_rng(1)
    ctr = rng.integers(0, 2**32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    key = rng.integers(0, 2**32, size=(4096, 2), dtype=np.uint64).astype(np.uint32)
    out = np.zeros_like(ctr)
    _lib.check(_lib.load().mcmc_debug_philox(_ctx(), len(ctr), ctr.ctypes.data_as(P), key.ctypes.data_as(P),
                                              out.ctypes.data_as(P)))
    assert np.array_equal(out, orc.philox(ctr, key))


def _dev_math(op, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), dtype=np.float64)
    out = np.empty(4 * len(x) if op == 6 else len(x))
    _lib.check(_lib.load().mcmc_debug_detmath(_ctx(), op, len(x), _lib.dptr(x), _lib.dptr(y), _lib.dptr(out)))
    return out


@pytest.mark.parametrize("op,name", [(0, "log"), (1, "exp"), (2, "sin2pi"), (3, "cos2pi"), (4, "sqrt"),
                                     (5, "div"), (7, "round"), (9, "bm_log_u32"), (10, "sin2pi_u32"),
                                     (11, "cos2pi_u32"), (12, "sqrt_pos_normal"), (13, "exp_tab"),
                                     (14, "log_tab"), (16, "bm_rad2_u32"),
                                     (17, "bm_radius_u32"), (18, "erfc"), (19, "log1p"),
                                     (20, "normlogcdf"), (21, "bm_radius_u32_lds"), (22, "logi_term"),
                                     (23, "logi_weight")])
def test_device_detmath_bitwise(gpu, op, name):
    rng = np.random.default_rng(op)
    if op == 0:
        x = np.concatenate([np.exp(rng.uniform(-740, 709, 200000)), [0.0, -0.0, -1.0, np.inf, np.nan, 5e-324, 1.0]])
    elif op == 1:
        x = np.concatenate([rng.uniform(-750, 712, 200000), [0.0, np.inf, -np.inf, np.nan]])
    elif op in (2, 3):
        x = np.floor(rng.uniform(0, 2**32, 200000)) * 2.0**-32
    elif op == 4:
        x = np.exp(rng.uniform(-700, 700, 200000))
    elif op == 12:               # positive normals; dense over the Box-Muller radius argument [2.3e-10, 46]
        x = np.concatenate([np.exp(rng.uniform(-700, 700, 200000)), rng.uniform(2.3e-10, 46.0, 200000),
                            -2.0 * np.log((np.arange(0, 4000) + 0.5) * 2.0**-32),
                            -2.0 * np.log((2.0**32 - 0.5 - np.arange(0, 4000)) * 2.0**-32),
                            np.nextafter(np.arange(1.0, 47.0) ** 2, 0), np.arange(1.0, 47.0) ** 2])
    elif op in (18, 20):         # erfc / normal log-cdf: every interval edge, the underflow end, special values
        edges = np.concatenate([[0.5], (2.0 ** np.arange(-1, 8)[:, None] * (1 + np.arange(4) / 4)).ravel()])
        x = np.concatenate([rng.uniform(-40, 40, 200000), rng.uniform(-2, 2, 100000), edges, -edges,
                            np.nextafter(edges, 0), np.nextafter(-edges, 0), rng.uniform(-60, 60, 20000),
                            [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-300, -1e-300, 27.2, 26.6, -38.5, -37.6]])
        if op == 20:
            x = x * np.sqrt(2.0)
    elif op == 19:
        x = np.concatenate([-np.exp(rng.uniform(-745, -1e-9, 100000)), rng.uniform(-0.99, 0.0, 100000),
                            [0.0, -0.0, 1e-300, -1e-17, -0.5, -0.84, np.nan]])
    elif op in (9, 10, 11, 16, 17, 21):  # 32-bit draws; the device's integer quarter-turn reduction vs the oracle's
        x = np.concatenate([np.floor(rng.uniform(0, 2**32, 200000)), np.arange(0, 2000),
                            2.0**32 - 1 - np.arange(0, 2000), (np.arange(-40, 40) + 2**29 * np.arange(1, 8)[:, None]
                                                               ).ravel() % 2**32])
        if op in (17, 21):       # every polynomial segment's two ends on both sides, and the tail's edge (v = 2^21)
            e, k = np.meshgrid(np.arange(21, 31), np.arange(32))
            v = (2.0**e * (1 + k / 32)).ravel().astype(np.int64)
            v = np.concatenate([v - 2, v - 1, v, v + 1, [2**21 - 2, 2**21 - 1, 2**21, 2**21 + 1, 2**31 - 1]])
            x = np.concatenate([x, v, 2**32 - 1 - v]).astype(np.float64)
    elif op == 13:
        x = np.concatenate([rng.uniform(-750, 712, 200000), rng.uniform(-40, 40, 200000),
                            [0.0, np.inf, -np.inf, np.nan, 710.0, -746.0, -745.2, 709.79]])
    elif op == 14:
        x = np.concatenate([np.exp(rng.uniform(-745, 0, 200000)), rng.uniform(0, 1, 200000),
                            1 - np.exp(rng.uniform(-40, 0, 100000)), rng.uniform(5e-324, 2.3e-308, 20000),
                            [0.0, 1.0, 5e-324, 2.2250738585072014e-308, np.nan]])
    elif op == 5:
        x = rng.normal(size=200000) * np.exp(rng.uniform(-300, 300, 200000))
    elif op in (22, 23):         # eta over every table segment and both edges of each, beyond |u| = 40, specials
        j = np.arange(0, 321) / 8.0
        x = np.concatenate([rng.uniform(-45, 45, 200000), rng.normal(0, 3, 50000), rng.uniform(-800, 800, 5000),
                            j + 1 / 16, j - 1 / 16, np.nextafter(j + 1 / 16, 0), -(j + 1 / 16), -(j - 1 / 16),
                            [0.0, -0.0, 40.0, -40.0, 1e300, -1e300, np.inf, -np.inf]])
    else:
        x = np.concatenate([rng.uniform(-1e6, 1e6, 100000), np.arange(-50, 50) + 0.5])
    y = np.exp(rng.uniform(-300, 300, len(x))) if op == 5 else None
    if op in (22, 23):           # w = s (2y - 1) in {-1, +1}
        y = np.where(rng.random(len(x)) < 0.5, -1.0, 1.0)
    d, h = _dev_math(op, x, y), orc.detmath(op, x, y)
    same = (d.view(np.uint64) == h.view(np.uint64)) | (np.isnan(d) & np.isnan(h))
    assert same.all(), f"{name}: {np.count_nonzero(~same)} mismatches, e.g. x={x[~same][:3]}"


def test_screened_accept_test_is_exact(gpu):
    """gt_det_log (the RWM/MALA test ratio > log(rand()), RWM.jl:63, screened by an f32 log2) against the oracle's
    ratio > det_log(u): ratios at det_log(u) itself, one ulp either side, inside and just outside the screen's
    band E = 2^-16 (1 + |L|), far away, and the special values (u = 0 -> -inf; NaN, +-inf ratios; u near 1)."""
    rng = np.random.default_rng(15)
    u = np.concatenate([rng.uniform(0, 1, 20000), 1 - np.exp(rng.uniform(-36, -1, 5000)), np.exp(rng.uniform(-36, 0, 5000)),
                        [0.0, 2.0**-53, 1 - 2.0**-53, 0.5]])
    L = orc.detmath(0, u)
    E = 2.0**-16 * (1 + np.abs(np.where(np.isfinite(L), L, 0)))
    ratios = [L, np.nextafter(L, np.inf), np.nextafter(L, -np.inf), L + 0.3 * E, L - 0.3 * E, L + 0.999 * E,
              L - 0.999 * E, L + 3 * E, L - 3 * E, L + 1.0, L - 1.0, np.zeros_like(u), np.full_like(u, np.nan),
              np.full_like(u, -np.inf), np.full_like(u, np.inf)]
    r = np.concatenate(ratios)
    uu = np.tile(u, len(ratios))
    d, h = _dev_math(15, r, uu), orc.detmath(15, r, uu)
    assert np.array_equal(d, h), f"{np.count_nonzero(d != h)} decisions differ"
    assert 0 < h.mean() < 1


def test_device_normals_bitwise(gpu):
    n = 50000
    a = np.arange(n, dtype=float) + 2.0**32 * 3
    z, zh = _dev_math(6, a, np.full(n, 17.0)), orc.detmath(6, a, np.full(n, 17.0))
    assert np.array_equal(z.view(np.uint64), zh.view(np.uint64))
    u, uh = _dev_math(8, np.arange(n, dtype=float)), orc.detmath(8, np.arange(n, dtype=float))
    assert np.array_equal(u, uh)


# ------------------------------------------------------------------ samplers
def _model(kind, d):
    if kind == "iso":
        return mc.model(mc.IsoNormalDot(), init=np.linspace(0.5, 1.5, d), grad=True,
                        scale=np.linspace(0.8, 1.2, d))
    if kind == "abs":
        return mc.model(mc.AbsNormalDSL(1.0, 0.7), x=np.linspace(-1, 1, d), gradient=True)
    return mc.model(mc.NormalDSL(0.3, 1.7), v=np.linspace(-1, 1, d), gradient=True)


SAMPLERS = {
    "rwm": lambda: mc.RWM(0.6),
    "mala": lambda: mc.MALA(0.4),
    "mala_tuned": lambda: mc.MALA(2.0, mc.EmpMCTuner(0.6, adaptStep=7)),
    "hmc": lambda: mc.HMC(4, 0.3),
    "hmc_tuned": lambda: mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9)),
    "hmcda": lambda: mc.HMCDA(len=0.8),
}


def assert_parity(chain, s_ref, g_ref, acc_ref, kind):
    s = chain._samples
    assert s.shape == s_ref.shape
    acc = chain.diagnostics["accept"].T
    assert np.array_equal(acc, acc_ref.astype(bool)), f"accept bits differ in {np.count_nonzero(acc != acc_ref)}"
    np.testing.assert_allclose(s, s_ref, rtol=RTOL, atol=0)
    assert np.array_equal(s.view(np.uint64), s_ref.view(np.uint64)), "samples not bit-identical"
    if g_ref is not None and kind != "rwm":
        np.testing.assert_allclose(chain._gradients, g_ref, rtol=RTOL, atol=0)


def order_for(d):
    """None: the oracle takes the library's own order (oracle_ref.kernel_order): lane-per-chain kernels (d <= 16)
    sum left to right; two-lanes-per-chain kernels (16 < d <= 32) each half, then the halves; wave-per-chain kernels
    (d <= 2048) per lane + butterfly; block-per-chain kernels (d <= 8192: 4 waves, d <= 16384: 8 waves) per lane,
    per wave, then waves left to right; RAM lane per chain up to d = 32."""
    return None


@pytest.mark.parametrize("sname", list(SAMPLERS))
@pytest.mark.parametrize("mkind", ["iso", "normal"])
@pytest.mark.parametrize("d", [2049, 5000, 8192, 8193, 16384])
def test_block_per_chain_parity(gpu, sname, mkind, d):
    """d > 2048 (the reference's model() takes any d, likmodel.jl:100-143): one chain per block of 4 (d <= 8192) or
    8 (d <= 16384) waves, sums per lane, per wave, then over the waves -- bitwise against the oracle in that order,
    every sampler, both separable model families, partial and full last blocks."""
    m = _model(mkind, d)
    C = 5
    r = mc.SerialMC(steps=6, burnin=1, thinning=2)
    t = (m * SAMPLERS[sname]() * r).batch(C, seed=2024 + d)
    chain = mc.run(t)
    assert t.step_kernel.startswith("bpc_")
    oc = orc.OracleChains(m, SAMPLERS[sname](), nchains=C, seed=2024 + d, order=order_for(d))
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname)
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    lp, g = m.evalallg(chain.final_x)                       # model.eval at this d (bpc_eval)
    lp_r, g_r = orc.eval_batch(m, chain.final_x, order=order_for(d))
    assert np.array_equal(lp, lp_r) and np.array_equal(g, g_r)


@pytest.mark.parametrize("sname", list(SAMPLERS))
@pytest.mark.parametrize("mkind", ["iso", "normal", "abs"])
@pytest.mark.parametrize("d", [1, 3, 7, 16, 32, 33, 100, 256, 257, 1024])
def test_sampler_parity(gpu, sname, mkind, d):
    m = _model(mkind, d)
    C = 200 if d <= 256 else 67                          # not a multiple of 64 / of 4: tail wave, tail block
    r = mc.SerialMC(steps=45 if d <= 256 else 20, burnin=6, thinning=3)
    task = m * SAMPLERS[sname]() * r
    chain = mc.run(task, nchains=C, seed=12345 + d)
    oc = orc.OracleChains(m, SAMPLERS[sname](), nchains=C, seed=12345 + d, order=order_for(d))
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname)
    assert np.array_equal(chain.final_x, oc.x, equal_nan=True) and np.array_equal(chain.final_lp, oc.lp, equal_nan=True)
    assert chain.task.evals == int(oc.n_evals.sum())        # leapfrog / evaluation bookkeeping


@pytest.mark.parametrize("d", [5, 70])
@pytest.mark.parametrize("sname", ["rwm", "mala_tuned", "hmc_tuned", "hmcda"])
def test_continue_run_matches_oracle(gpu, sname, d):
    """run(chain) continues the same chains (runners.jl:14); tuners keep adapting only while i <= burnin."""
    m = _model("normal", d)
    r = mc.SerialMC(steps=30, burnin=12, thinning=2)
    task = (m * SAMPLERS[sname]() * r).batch(130, seed=77)
    c1 = mc.run(task)
    c2 = mc.run(c1)
    oc = orc.OracleChains(m, SAMPLERS[sname](), nchains=130, seed=77, order=order_for(d))
    s1, g1, a1 = oc.run(r)
    s2, g2, a2 = oc.run(r)
    assert_parity(c1, s1, g1, a1, sname)
    assert_parity(c2, s2, g2, a2, sname)
    assert task.steps_done == 60


@pytest.mark.parametrize("d", [8, 96])
@pytest.mark.parametrize("spl", [1, 7])
def test_steps_per_launch_is_invisible(gpu, spl, d):
    m = _model("iso", d)
    r = mc.SerialMC(steps=40, burnin=5, thinning=4)
    a = mc.run((m * mc.MALA(0.3) * r).batch(150, seed=3))
    b = mc.run((m * mc.MALA(0.3) * r).batch(150, seed=3, steps_per_launch=spl))
    assert np.array_equal(a._samples, b._samples)
    assert np.array_equal(a.diagnostics["accept"], b.diagnostics["accept"])


@pytest.mark.parametrize("d", [4, 130])
def test_chain_offset_sharding_is_invisible(gpu, d):
    m = _model("iso", d)
    r = mc.SerialMC(steps=25, burnin=3)
    full = mc.run((m * mc.HMC(3, 0.25) * r).batch(300, seed=5))
    lo = mc.run((m * mc.HMC(3, 0.25) * r).batch(170, seed=5, chain_offset=0))
    hi = mc.run((m * mc.HMC(3, 0.25) * r).batch(130, seed=5, chain_offset=170))
    assert np.array_equal(np.concatenate([lo._samples, hi._samples], axis=2), full._samples)
    assert np.array_equal(np.concatenate([lo.diagnostics["accept"], hi.diagnostics["accept"]]),
                          full.diagnostics["accept"])


def test_single_chain_readme_example(gpu):
    """README.md:85: run(mymodel1, RWM(0.1), SerialMC(steps=1000, burnin=100)) -> 900 samples."""
    m1 = mc.model(mc.IsoNormalDot(), init=np.ones(3))
    ch = mc.run(m1, mc.RWM(0.1), mc.SerialMC(steps=1000, burnin=100))
    assert ch.samples.shape == (1, 900, 3) and np.isnan(ch.gradients).all()
    # the chain is drawn from the global stream (MCMC.jl:33-39): its key is drawn_key(the global seed), its id the
    # stream's next; the oracle takes the task's own
    assert ch.task.seed == mc.drawn_key(ch.task.seed)
    oc = orc.OracleChains(m1, mc.RWM(0.1), nchains=1, seed=ch.task.seed, chain_offset=ch.task.chain_offset)
    s, _, acc = oc.run(mc.SerialMC(steps=1000, burnin=100))
    assert np.array_equal(ch._samples, s) and np.array_equal(ch.diagnostics["accept"].T, acc.astype(bool))
    assert ch.diagnostics["step"] == list(range(101, 1001))
    rate = mc.acceptance(ch)[0]
    assert rate == pytest.approx(100 * acc.mean(), rel=1e-14)      # 100 * count / n and 100 * mean round apart


def test_resume_restarts_from_init(gpu):
    """resume (SerialMC.jl:93-97) spins a new task from model.init whose chains come from the global stream: not a
    replay of the original run's first steps, but bitwise the oracle's chains at the ids it drew."""
    m = _model("iso", 3)
    ch = mc.run((m * mc.RWM(0.5) * mc.SerialMC(steps=20, thinning=2)).batch(64, seed=9))
    ch2 = mc.resume(ch, steps=30)
    assert ch2.samples.shape == (64, 15, 3) and ch2.task.steps_done == 30
    t2 = ch2.task
    oc = orc.OracleChains(m, mc.RWM(0.5), nchains=64, seed=t2.seed, chain_offset=t2.chain_offset)
    s_ref, g_ref, acc_ref = oc.run(mc.SerialMC(steps=30, thinning=2))
    assert_parity(ch2, s_ref, g_ref, acc_ref, "rwm")
    assert not np.array_equal(ch2._samples[:10], ch._samples[:10])     # a fresh stream, not the original's


@pytest.mark.parametrize("d", [9, 300])
def test_model_eval_matches_oracle(gpu, d):
    for kind in ("iso", "normal"):
        m = _model(kind, d)
        x = np.random.default_rng(0).normal(size=(d, 333)) * 3
        lp, g = m.evalallg(x)
        lp_r, g_r = orc.eval_batch(m, x, order=order_for(d))
        assert np.array_equal(lp, lp_r) and np.array_equal(g, g_r)


def test_init_out_of_support(gpu):
    m = mc.model(mc.NormalDSL(0, 1), v=np.zeros(2), gradient=True)
    bad = np.array([[np.inf, 0.0, 0.0], [0.0, 0.0, 0.0]])
    with pytest.raises(mc.OutOfSupportError, match="Initial values out of model support"):
        mc.run((m * mc.RWM(0.1) * mc.SerialMC(steps=5)).batch(3, init_x=bad))
    with pytest.raises(mc.OutOfSupportError):
        mc.model(mc.NormalDSL(0, 1), v=np.array([np.inf]), gradient=True)._handle(0)


@pytest.mark.parametrize("d", [4, 40])
def test_divergent_hmc_rejects(gpu, d):
    """Huge leapfrog steps on the DSL target: out-of-support trajectories (-Inf, zero grad) must reject."""
    m = mc.model(mc.NormalDSL(0.0, 1.0), v=np.ones(d), gradient=True)
    r = mc.SerialMC(steps=20)
    ch = mc.run((m * mc.HMC(30, 1e150) * r).batch(70, seed=4))
    oc = orc.OracleChains(m, mc.HMC(30, 1e150), nchains=70, seed=4, order=order_for(d))
    s, g, acc = oc.run(r)
    assert_parity(ch, s, g, acc, "hmc")
    assert not ch.diagnostics["accept"].any()


# ------------------------------------------------------------------ regression models (fp64 MFMA)
def _glm_model(kind, d, n=50, seed=0):
    rng = np.random.default_rng(seed + d)
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1))])
    beta0 = rng.normal(size=d) * 0.3
    if kind == "logistic":
        Y = (rng.random(n) < 1 / (1 + np.exp(-X @ beta0))).astype(float)
        return mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)
    if kind == "probit":
        Y = (rng.normal(size=n) < X @ beta0).astype(float)
        return mc.model(mc.ProbitRegression(X, Y, prior_sigma=10.0), vars=np.zeros(d), gradient=True)
    Y = X @ beta0 + rng.normal(size=n)
    return mc.model(mc.LinearRegression(X, Y, prior_sigma=1.0, noise_sigma=1.0), vars=np.zeros(d), gradient=True)


GLM_SAMPLERS = {
    "rwm": lambda: mc.RWM(0.05),
    "mala": lambda: mc.MALA(0.002),
    "mala_tuned": lambda: mc.MALA(0.01, mc.EmpMCTuner(0.6, adaptStep=3)),
    "hmc": lambda: mc.HMC(3, 0.02),
    "hmc_tuned": lambda: mc.HMC(2, 0.05, mc.EmpMCTuner(0.7, adaptStep=3, maxStep=6)),
    "hmcda": lambda: mc.HMCDA(len=0.1),
}


@pytest.mark.parametrize("sname", list(GLM_SAMPLERS))
@pytest.mark.parametrize("kind", ["logistic", "linear"])
@pytest.mark.parametrize("d", [3, 16, 37, 64, 100, 200, 300, 600, 1024])     # 600, 1024: 8 slices of 128, one X buffer
def test_glm_sampler_parity(gpu, sname, kind, d):
    m = _glm_model(kind, d)
    C = 40                                               # not a multiple of 16: tail tile
    r = mc.SerialMC(steps=14, burnin=4, thinning=2)
    chain = mc.run((m * GLM_SAMPLERS[sname]() * r).batch(C, seed=99 + d))
    oc = orc.OracleChains(m, GLM_SAMPLERS[sname](), nchains=C, seed=99 + d)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname)
    assert np.array_equal(chain.final_x, oc.x, equal_nan=True) and np.array_equal(chain.final_lp, oc.lp, equal_nan=True)
    assert chain.task.evals == int(oc.n_evals.sum())        # leapfrog / evaluation bookkeeping


@pytest.mark.parametrize("sname", list(GLM_SAMPLERS))
@pytest.mark.parametrize("d", [3, 37, 200])              # single slice (NM = 1, 4) and d-sliced (4 x 64)
def test_probit_sampler_parity(gpu, sname, d):
    """examples/probit_regression.jl's target on every gradient sampler, bitwise against the oracle."""
    test_glm_sampler_parity(gpu, sname, "probit", d)


def test_probit_vaso_example_bitwise(gpu):
    """The probit example itself (probit_regression.jl:7-16, 68): vaso.txt standardised, MvNormal(0, 100 I) prior,
    RWM(0.5) x SerialMC(1001:10000), 64 chains from a prior draw (randprior), bitwise against the oracle."""
    X, Y = mc.vaso_data(os.path.join(os.path.dirname(__file__), "golden", "vaso.txt"))
    init = np.random.default_rng(68).normal(size=3) * 10.0
    m = mc.model(mc.ProbitRegression(X, Y), vars=init, gradient=True)
    r = mc.SerialMC(steps=10000, burnin=1000)
    chain = mc.run((m * mc.RWM(0.5) * r).batch(64, seed=68))
    oc = orc.OracleChains(m, mc.RWM(0.5), nchains=64, seed=68)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, "rwm")
    assert 0.05 < acc_ref.mean() < 0.6


@pytest.mark.parametrize("kind", ["logistic", "linear", "probit"])
@pytest.mark.parametrize("d", [10, 130, 700])
def test_glm_eval_matches_oracle(gpu, kind, d):
    m = _glm_model(kind, d, n=70)
    x = np.random.default_rng(3).normal(size=(d, 37)) * 0.2
    lp, g = m.evalallg(x)
    lp_r, g_r = orc.eval_batch(m, x)
    assert np.array_equal(lp, lp_r) and np.array_equal(g, g_r)


def test_glm_width_cap(gpu):
    """d = 1024 is the widest regression shape (8 slices of 128 coordinates, one 128 KB X tile in LDS); wider models
    are refused at model() with the cap in the message."""
    with pytest.raises(Exception, match="d <= 1024"):
        _glm_model("linear", 1025, n=20).evalallg(np.zeros((1025, 1)))


def test_glm_continue_and_shard(gpu):
    m = _glm_model("logistic", 20)
    r = mc.SerialMC(steps=10, burnin=3)
    t = (m * mc.MALA(0.01, mc.EmpMCTuner(0.5, adaptStep=2)) * r).batch(50, seed=5)
    c1, c2 = mc.run(t), None
    c2 = mc.run(c1)
    oc = orc.OracleChains(m, mc.MALA(0.01, mc.EmpMCTuner(0.5, adaptStep=2)), nchains=50, seed=5)
    s1, g1, a1 = oc.run(r)
    s2, g2, a2 = oc.run(r)
    assert_parity(c1, s1, g1, a1, "mala")
    assert_parity(c2, s2, g2, a2, "mala")
    lo = mc.run((m * mc.HMC(2, 0.05) * r).batch(23, seed=5, chain_offset=0))
    hi = mc.run((m * mc.HMC(2, 0.05) * r).batch(27, seed=5, chain_offset=23))
    full = mc.run((m * mc.HMC(2, 0.05) * r).batch(50, seed=5))
    assert np.array_equal(np.concatenate([lo._samples, hi._samples], axis=2), full._samples)


@pytest.mark.parametrize("sname", ["hmcda", "hmc_tuned"])
@pytest.mark.parametrize("kind,d", [("linear", 20), ("logistic", 200)])
def test_glm_trajectory_order_continue(gpu, sname, kind, d):
    """Regression HMC / HMCDA launch their chains sorted by trajectory length (runtime.cpp glm_trajectory_order):
    after an adapting run the per-chain leapStep (HMCDA) or nLeaps (tuned HMC) differ, so the continued run's tile
    -> chain map is a real permutation; samples, gradients, accept bits, final state, evaluation counts and the
    adapted state stay bitwise the oracle's (which knows nothing of tiles)."""
    import ctypes as ct
    mk = {"hmcda": lambda: mc.HMCDA(len=1.0),                # adapted leapSteps differ from chain to chain
          "hmc_tuned": lambda: mc.HMC(2, 0.05, mc.EmpMCTuner(0.7, adaptStep=2, maxStep=9))}[sname]
    m = _glm_model(kind, d)
    C = 70                                                     # four full 16-chain tiles and a tail of 6
    r1, r2 = mc.SerialMC(steps=8, burnin=6), mc.SerialMC(steps=6, burnin=1)
    t = (m * mk() * r1).batch(C, seed=13)
    c1 = mc.run(t)
    ts1 = t.tuner_state()
    t.runner = r2
    c2 = mc.run(t)
    used, order = ct.c_int32(0), (ct.c_int32 * C)()
    _lib.check(_lib.load().mcmc_debug_chains_order(t.handle(), ct.byref(used), order))
    assert used.value == 1
    order = np.frombuffer(order, dtype=np.int32)
    key = ts1["step"] if sname == "hmcda" else -ts1["nleaps"].astype(float)   # longest trajectory first
    assert np.array_equal(order, np.argsort(key, kind="stable"))
    if np.unique(key).size > 1:                               # (tuned HMC may leave every nLeaps at maxStep)
        assert not np.array_equal(order, np.arange(C))
    oc = orc.OracleChains(m, mk(), nchains=C, seed=13)
    s1, g1, a1 = oc.run(r1)
    s2, g2, a2 = oc.run(r2)
    assert_parity(c1, s1, g1, a1, sname)
    assert_parity(c2, s2, g2, a2, sname)
    assert np.array_equal(c2._gradients.view(np.uint64), g2.view(np.uint64))
    assert np.array_equal(c2.final_x.view(np.uint64), oc.x.view(np.uint64))
    assert t.evals == int(oc.n_evals.sum())
    ts = t.tuner_state()
    assert np.array_equal(ts["step"].view(np.uint64), oc.t_step.view(np.uint64))


@pytest.mark.parametrize("kind,d,C,sname", [("logistic", 200, 96, "hmcda"), ("linear", 300, 64, "hmcda"),
                                            ("probit", 160, 160, "hmc_tuned")])
def test_glm_tile_pairing_and_skip(gpu, kind, d, C, sname):
    """d-sliced regression HMCDA with two chain tiles a workgroup (128 < d <= 512) and whole 32-chain workgroups: the
    runtime gives workgroup w the w-th longest and the w-th shortest sorted tile (runtime.cpp glm_trajectory_order),
    and glm_hmc's tiles whose chains have all ended their trajectories skip their evaluations (GLM_TILE_SKIP) while
    the other tile of their workgroup runs on.  Samples, gradients, accept bits, final state, evaluation counts and
    the adapted leapSteps stay bitwise the oracle's."""
    import ctypes as ct
    mk = {"hmcda": lambda: mc.HMCDA(len=1.0),
          "hmc_tuned": lambda: mc.HMC(2, 0.05, mc.EmpMCTuner(0.7, adaptStep=2, maxStep=9))}[sname]
    m = _glm_model(kind, d)                                    # C / 32 two-tile workgroups (d = 160, 200: 64-wide
    r1, r2 = mc.SerialMC(steps=8, burnin=6), mc.SerialMC(steps=6, burnin=1)   # slices; d = 300: 128-wide)
    t = (m * mk() * r1).batch(C, seed=21)
    c1 = mc.run(t)
    ts1 = t.tuner_state()
    t.runner = r2
    c2 = mc.run(t)
    used, order = ct.c_int32(0), (ct.c_int32 * C)()
    _lib.check(_lib.load().mcmc_debug_chains_order(t.handle(), ct.byref(used), order))
    assert used.value == 1
    key = ts1["step"] if sname == "hmcda" else -ts1["nleaps"].astype(float)   # longest trajectory first
    srt = np.argsort(key, kind="stable").reshape(C // 16, 16)
    nt = C // 16
    paired = np.concatenate([srt[w if h == 0 else nt - 1 - w] for w in range(nt // 2) for h in range(2)])
    assert np.array_equal(np.frombuffer(order, dtype=np.int32), paired)
    oc = orc.OracleChains(m, mk(), nchains=C, seed=21)
    s1, g1, a1 = oc.run(r1)
    s2, g2, a2 = oc.run(r2)
    assert_parity(c1, s1, g1, a1, sname)
    assert_parity(c2, s2, g2, a2, sname)
    assert np.array_equal(c2._gradients.view(np.uint64), g2.view(np.uint64))
    assert np.array_equal(c2.final_x.view(np.uint64), oc.x.view(np.uint64))
    assert t.evals == int(oc.n_evals.sum())
    assert np.array_equal(t.tuner_state()["step"].view(np.uint64), oc.t_step.view(np.uint64))


def test_logistic_out_of_support_rejects(gpu):
    """Huge proposals push prob to exactly 0/1: log(0) -> LLAcc throws -> (-Inf, 0) -> reject."""
    X = np.hstack([np.ones((30, 1)), np.random.default_rng(1).normal(size=(30, 3)) * 30])
    Y = (np.random.default_rng(2).random(30) < 0.5).astype(float)
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(4), gradient=True)
    r = mc.SerialMC(steps=8)
    ch = mc.run((m * mc.RWM(50.0) * r).batch(20, seed=1))
    oc = orc.OracleChains(m, mc.RWM(50.0), nchains=20, seed=1)
    s, g, acc = oc.run(r)
    assert_parity(ch, s, g, acc, "rwm")


@pytest.mark.parametrize("obs", [3, 12, 15])
def test_logistic_mala_minus_inf_rule_each_row(gpu, obs):
    """The reference's -Inf (p rounds to 1 with y = 0) triggered by one observation in row obs // 4 of a 16-
    observation tile (obs 3, 12: the first tile's rows 0 and 3; 15: its last lane quarter), in glm_mala1ws' V wave;
    samples, gradients and accept bits bitwise against the oracle, both outcomes present."""
    rng = np.random.default_rng(40 + obs)
    d, n = 8, 20
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1)) * 0.3])
    X[obs] *= 100.0                                           # 400: every proposal rejected (oracle), 100: mixed
    Y = (rng.random(n) < 0.5).astype(float)
    Y[obs] = 0.0
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)
    r = mc.SerialMC(steps=12, burnin=0)
    ch = mc.run((m * mc.MALA(0.02) * r).batch(96, seed=9))
    assert ch.task.step_kernel.startswith("glm_mala1ws")
    oc = orc.OracleChains(m, mc.MALA(0.02), nchains=96, seed=9)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(ch, s_ref, g_ref, acc_ref, "mala")
    assert np.array_equal(ch._gradients.view(np.uint64), g_ref.view(np.uint64))
    a = ch.diagnostics["accept"]
    assert 0 < a.mean() < 1                                   # both outcomes, the rejections by the -Inf rule
    eta = np.einsum("j,sjc->sc", X[obs], s_ref)
    assert eta.max() < 36.8 and np.abs(eta).max() > 100       # kept states stay below the rule's p == 1 edge


@pytest.mark.parametrize("kind", ["logistic", "probit"])
def test_covariates_that_can_overflow_to_nan_are_refused(gpu, kind):
    """X vars overflowing with mixed signs gives a NaN eta, which the reference's LLAcc turns into -Inf; the kernels
    clamp |eta| into their tables, so mcmc_model_create refuses data whose row L1 norm times the largest |vars| of
    finite prior density can reach 2^1022 (runtime.cpp), and accepts the same rows scaled into range."""
    from mcmchip import _lib
    X = np.array([[1.0, 1e200], [1.0, -1e200], [1.0, 3.0]])
    Y = np.array([0.0, 1.0, 1.0])
    T = mc.LogisticRegression if kind == "logistic" else mc.ProbitRegression
    m = mc.model(T(X, Y), vars=np.zeros(2), gradient=True)
    with pytest.raises(_lib.MCMCError, match="overflow to NaN"):
        mc.run((m * mc.RWM(0.1) * mc.SerialMC(steps=4)).batch(64, seed=1))
    m = mc.model(T(X * 1e-100, Y), vars=np.zeros(2), gradient=True)
    mc.run((m * mc.RWM(0.1) * mc.SerialMC(steps=4)).batch(64, seed=1))


@pytest.mark.parametrize("sname", ["rwm", "hmc"])
def test_glm_nonzero_init_few_coords_many_chains(gpu, sname):
    """d << C with a non-zero start: the coordinate-major state must be broadcast per coordinate row."""
    d = 5
    rng = np.random.default_rng(11)
    X = np.hstack([np.ones((60, 1)), rng.normal(size=(60, d - 1))])
    Y = X @ (rng.normal(size=d) * 0.3) + rng.normal(size=60)
    m = mc.model(mc.LinearRegression(X, Y), vars=0.1 * np.arange(1, d + 1), gradient=True)
    r = mc.SerialMC(steps=9, burnin=1, thinning=2)
    ch = mc.run((m * GLM_SAMPLERS[sname]() * r).batch(200, seed=3))
    oc = orc.OracleChains(m, GLM_SAMPLERS[sname](), nchains=200, seed=3)
    s, g, acc = oc.run(r)
    assert_parity(ch, s, g, acc, sname)


def test_model_released_before_its_chains(gpu):
    """A host that finalizes the model before its chains (any GC order) must not free it under them."""
    from mcmchip import _lib
    m = _glm_model("logistic", 6)
    r = mc.SerialMC(steps=5)
    t = (m * mc.HMC(2, 0.05) * r).batch(32, seed=2)
    t.handle()
    for h in m._dev.values():
        _lib.check(_lib.load().mcmc_model_destroy(h))
    m._dev.clear()
    ch = mc.run(t)                          # the chains still own a live model
    oc = orc.OracleChains(m, mc.HMC(2, 0.05), nchains=32, seed=2)
    s, g, acc = oc.run(r)
    assert_parity(ch, s, g, acc, "hmc")
    del t, ch                               # last chains gone: the model is freed now


@pytest.mark.parametrize("vtype,name", [(1, "imse"), (2, "ipse"), (3, "bm")])
# k_ess_reg<32/64/96> (n <= 96, IMSE/IPSE; 32 and 64 at the bucket edges), k_ess_tile (batch means, 96 < n <= 618,
# > 64 KB of LDS from 241) / k_ess_col
@pytest.mark.parametrize("n", [20, 32, 33, 41, 64, 65, 90, 96, 97, 300, 618, 619])
def test_device_ess_bitwise(gpu, vtype, name, n):
    import torch
    rng = np.random.default_rng(n + vtype)
    d, C = 3, 130
    e = rng.normal(size=(n, d, C))
    x = np.zeros_like(e)
    x[0] = e[0]
    for t in range(1, n):
        x[t] = 0.6 * x[t - 1] + e[t]
    bl = 20 if n >= 40 else n // 2                          # batch means need two batches
    ref, vref = orc.ess(x, vtype, 0, bl)
    chain = type("Chain", (), {})()
    chain._samples = x
    got, v = mc.stats.ess_device(chain, name, batchlen=bl, return_var=True)
    assert np.array_equal(got.T, ref) and np.array_equal(v.T, vref)
    xt = torch.from_numpy(x).cuda()
    got_d = mc.stats.ess_device(xt, name, batchlen=bl)     # device pointers, no PCIe
    assert np.array_equal(got_d.cpu().numpy(), ref)


@pytest.mark.parametrize("n,maxlag", [(2, 0), (3, 0), (3, 1), (17, 5), (64, 63), (65, 2), (90, 6), (90, 7), (90, 89),
                                      (96, 95), (400, 9)])
def test_device_ess_short_series_and_maxlag(gpu, n, maxlag):
    """short series, maxlag below n - 1 (k = floor((maxlag - 1) / 2) pairs), white noise (Geyer stops at the first
    pairs) next to strongly autocorrelated series (it runs to k), in one batch"""
    rng = np.random.default_rng(n * 7 + maxlag)
    d, C = 2, 200
    x = rng.normal(size=(n, d, C))
    for t in range(1, n):
        x[t, 1] = 0.95 * x[t - 1, 1] + 0.1 * x[t, 1]
    chain = type("Chain", (), {})()
    chain._samples = x
    for vtype, name in ((1, "imse"), (2, "ipse")):
        ref, vref = orc.ess(x, vtype, maxlag, 0)
        got, v = mc.stats.ess_device(chain, name, maxlag=maxlag, return_var=True)
        assert np.array_equal(got.T.view(np.uint64), ref.view(np.uint64))
        assert np.array_equal(v.T.view(np.uint64), vref.view(np.uint64))


def test_device_ess_of_a_run(gpu):
    m = _model("iso", 4)
    ch = mc.run(m * mc.HMC(0.75) * mc.SerialMC(steps=600, burnin=100), nchains=70, seed=3)
    ref, _ = orc.ess(ch._samples, 1)
    assert np.array_equal(mc.stats.ess_device(ch), ref.T)
    np.testing.assert_allclose(mc.stats.ess_device(ch), mc.stats.ess(ch), rtol=1e-9)
    with pytest.raises(mc.MCMCError, match="greather than one"):
        mc.stats.ess_device(ch, "bm", batchlen=400)


DIST_MODELS = [("Gamma", (2.5, 0.7), 1.2), ("Beta", (2.0, 3.0), 0.4), ("TDist", (3.0,), 0.1), ("Weibull", (1.5, 2.0), 1.0),
               ("LogNormal", (0.2, 0.6), 1.1), ("Laplace", (0.4, 0.9), 0.3), ("Cauchy", (0.5, 1.3), 0.2),
               ("Uniform", (-1.0, 2.0), 0.5), ("Exponential", (1.5,), 0.8), ("Normal", (0.3, 1.7), 0.0)]


@pytest.mark.parametrize("sname", ["rwm", "mala", "hmc", "hmcda"])
@pytest.mark.parametrize("dist,params,x0", DIST_MODELS, ids=[c[0] for c in DIST_MODELS])
@pytest.mark.parametrize("d", [5, 40])
def test_dist_dsl_sampler_parity(gpu, sname, dist, params, x0, d):
    """v ~ Dist(p1, p2) through the lane-per-chain (d=5) and wave-per-chain (d=40) kernels; proposals
    leave the support (Gamma/Beta/... -> LLAcc -Inf) and must reject exactly as in the oracle."""
    if dist == "Uniform" and sname != "rwm":
        pytest.skip("zero gradient: MALA/HMC reduce to random walks; covered by RWM")
    m = mc.model(mc.DistDSL(dist, *params), v=np.full(d, x0), gradient=True)
    sp = {"rwm": lambda: mc.RWM(0.4), "mala": lambda: mc.MALA(0.05), "hmc": lambda: mc.HMC(3, 0.1),
          "hmcda": lambda: mc.HMCDA(len=0.3)}[sname]
    r = mc.SerialMC(steps=24, burnin=4, thinning=2)
    chain = mc.run((m * sp() * r).batch(130, seed=77 + d))
    oc = orc.OracleChains(m, sp(), nchains=130, seed=77 + d, order=order_for(d))
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname)


# ------------------------------------------------------------------ RAM (RAM.jl)
def _ram_model(mkind, d):
    if mkind == "dist":
        return mc.model(mc.DistDSL("Gamma", 2.5, 0.7), v=np.full(d, 1.2))
    return _model(mkind, d)


def _assert_ram_factor(task, oc, d):
    S = task.ram_factor()
    S_ref = mc.api.unpack_ram_factor(oc.ram_L, d)
    assert np.array_equal(S.view(np.uint64), S_ref.view(np.uint64)), "jump factors not bit-identical"


@pytest.mark.parametrize("mkind", ["iso", "normal", "abs", "dist"])
@pytest.mark.parametrize("d", [1, 3, 7, 16, 17, 28, 30, 32])
def test_ram_parity(gpu, mkind, d):
    """lane-per-chain RAM: samples, accept bits, final state and every chain's jump factor S bit-identical
    to the oracle (proposals out of the Gamma support -> -Inf -> downdates of S)."""
    m = _ram_model(mkind, d)
    C = 200
    r = mc.SerialMC(steps=45, burnin=6, thinning=3)
    task = (m * mc.RAM(0.7, 0.3) * r).batch(C, seed=4242 + d)
    chain = mc.run(task)
    oc = orc.OracleChains(m, mc.RAM(0.7, 0.3), nchains=C, seed=4242 + d)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert g_ref is None and chain._gradients is None
    assert_parity(chain, s_ref, None, acc_ref, "ram")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    assert task.evals == int(oc.n_evals.sum())
    _assert_ram_factor(task, oc, d)


@pytest.mark.parametrize("kind", ["logistic", "linear"])
@pytest.mark.parametrize("d", [3, 10, 16, 17, 32])
def test_glm_ram_parity(gpu, kind, d):
    """RAM on the regression targets (examples/linear_regression.jl:28): the four lanes of a chain
    rebuild S z, lane 0 stores the updated factor."""
    m = _glm_model(kind, d)
    C = 40
    r = mc.SerialMC(steps=30, burnin=4, thinning=2)
    task = (m * mc.RAM(1.0, 0.3) * r).batch(C, seed=31 + d)
    chain = mc.run(task)
    oc = orc.OracleChains(m, mc.RAM(1.0, 0.3), nchains=C, seed=31 + d)
    s_ref, _, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, None, acc_ref, "ram")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    _assert_ram_factor(task, oc, d)


@pytest.mark.parametrize("kind,d", [("linear", 33), ("logistic", 64), ("linear", 128), ("probit", 100),
                                    ("logistic", 256), ("linear", 257), ("logistic", 300), ("linear", 600),
                                    ("linear", 1024)])
def test_glm_ram_wave_parity(gpu, kind, d):
    """RAM on the regression targets for 32 < d <= 1024 (round 5): per step the regression eval kernel and the
    wave-per-chain accept / factor-update kernel (glm_ram_wave.hip; two chains a wave for d <= 256, round 6); samples,
    accept bits, final state, the evaluation count and every factor bitwise against the oracle (|rvec|^2 in the
    half-wave order for d <= 256, the 64-lane wave order above); 37 chains: a half-live tail wave, several launches,
    a continuation."""
    m = _glm_model(kind, d, n=40)
    C = 37
    r = mc.SerialMC(steps=12 if d <= 300 else 6, burnin=2, thinning=2)
    sc = 0.1 / np.sqrt(d)                                      # proposals of norm ~0.1: both accepts and rejects
    task = (m * mc.RAM(sc, 0.3) * r).batch(C, seed=55 + d, steps_per_launch=5)
    chain = mc.run(task)
    assert task.step_kernel.startswith("glm_ram_update<"), task.step_kernel
    oc = orc.OracleChains(m, mc.RAM(sc, 0.3), nchains=C, seed=55 + d)
    s_ref, _, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, None, acc_ref, "ram")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    assert task.evals == int(oc.n_evals.sum())
    assert chain.diagnostics["accept"].sum() > 0
    _assert_ram_factor(task, oc, d)
    c2 = mc.run(chain)
    s2, _, a2 = oc.run(r)
    assert_parity(c2, s2, None, a2, "ram")
    _assert_ram_factor(task, oc, d)


@pytest.mark.parametrize("kind,d,sampler", [("logistic", 6, "mala"), ("linear", 300, "rwm")])
def test_glm_state_rows_past_d_at_large_batch(gpu, kind, d, sampler):
    """The regression kernels load the state unconditionally and zero the slots past d (round 6); such a slot reads
    the chain's row 0, never the lane's own row, which lies past the d state rows when d is not a multiple of the
    slice geometry (d = 6: rows 8 and 12 of glm_mala1ws's lanes; d = 300: rows 300..511 of the eval kernel's).  At
    20 000 chains those rows would be megabytes past the state buffer; samples bitwise against the oracle."""
    m = _glm_model(kind, d, n=40)
    smp = mc.MALA(0.002) if sampler == "mala" else mc.RWM(0.05)
    C = 20000
    r = mc.SerialMC(steps=3, burnin=0)
    task = (m * smp * r).batch(C, seed=3 + d)
    chain = mc.run(task)
    oc = orc.OracleChains(m, smp, nchains=C, seed=3 + d)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref if sampler == "mala" else None, acc_ref, sampler)


@pytest.mark.parametrize("kind,d", [("linear", 64), ("logistic", 300)])
def test_glm_ram_wave_two_streams(gpu, kind, d):
    """At C >= 8192 chains glm_ram_wave runs the batch as two halves on two streams (the eval kernel of one beside
    the factor update of the other, round 6); the split is invisible: samples, accept bits, the final state and
    every factor bitwise against the oracle, the second half's tail wave half-live (8293 chains)."""
    m = _glm_model(kind, d, n=24)
    C = 8293
    r = mc.SerialMC(steps=4, burnin=1, thinning=1)
    sc = 0.1 / np.sqrt(d)
    task = (m * mc.RAM(sc, 0.3) * r).batch(C, seed=7 + d, steps_per_launch=2)
    chain = mc.run(task)
    assert task.step_kernel.startswith("glm_ram_update<"), task.step_kernel
    oc = orc.OracleChains(m, mc.RAM(sc, 0.3), nchains=C, seed=7 + d)
    s_ref, _, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, None, acc_ref, "ram")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    assert task.evals == int(oc.n_evals.sum())
    _assert_ram_factor(task, oc, d)


def test_ram_continue_spl_and_shards(gpu):
    """S lives on the device between runs; steps per launch and chain offsets are invisible."""
    d = 6
    m = _model("normal", d)
    r = mc.SerialMC(steps=30, burnin=5, thinning=5)
    task = (m * mc.RAM() * r).batch(150, seed=8)
    c1 = mc.run(task)
    c2 = mc.run(c1)
    oc = orc.OracleChains(m, mc.RAM(), nchains=150, seed=8)
    s1, _, a1 = oc.run(r)
    s2, _, a2 = oc.run(r)
    assert_parity(c1, s1, None, a1, "ram")
    assert_parity(c2, s2, None, a2, "ram")
    _assert_ram_factor(task, oc, d)
    b = mc.run((m * mc.RAM() * mc.SerialMC(steps=60, burnin=5, thinning=5)).batch(150, seed=8, steps_per_launch=7))
    lo = mc.run((m * mc.RAM() * mc.SerialMC(steps=60, burnin=5, thinning=5)).batch(70, seed=8))
    hi = mc.run((m * mc.RAM() * mc.SerialMC(steps=60, burnin=5, thinning=5)).batch(80, seed=8, chain_offset=70))
    full = orc.OracleChains(m, mc.RAM(), nchains=150, seed=8)
    s, _, _ = full.run(mc.SerialMC(steps=60, burnin=5, thinning=5))
    assert np.array_equal(b._samples, s)
    assert np.array_equal(np.concatenate([lo._samples, hi._samples], axis=2), s)


@pytest.mark.parametrize("mkind", ["iso", "normal", "abs", "dist"])
@pytest.mark.parametrize("d", [33, 64, 100, 128, 129, 200, 256, 257, 513, 1024])
def test_ram_wave_parity(gpu, mkind, d):
    """32 < d <= 1024 (RAM.jl:41-80 has no d cap): wave-per-chain RAM, the factor column-major per chain and its
    rows spread over the lanes; samples, accept bits, final state and every factor bit-identical to the oracle in
    the kernel's order (d <= 256: two chains per wave, one / two slot groups per lane, ORDER_HALF, 7 chains so the
    last wave has a dead half; 257..512: one chain per wave, two slot groups, 513..1024: four; tail wave and tail
    block)."""
    m = _ram_model(mkind, d)
    C = 7
    r = mc.SerialMC(steps=14 if d <= 256 else 8, burnin=2, thinning=2)
    task = (m * mc.RAM(0.7, 0.3) * r).batch(C, seed=777 + d, steps_per_launch=5)
    chain = mc.run(task)
    assert task.step_kernel.startswith("wpc_ram2<" if d <= 256 else "wpc_ram<")
    oc = orc.OracleChains(m, mc.RAM(0.7, 0.3), nchains=C, seed=777 + d, order=order_for(d))
    s_ref, _, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, None, acc_ref, "ram")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    assert task.evals == int(oc.n_evals.sum())
    _assert_ram_factor(task, oc, d)


def test_ram_wave_continue_and_shards(gpu):
    """wave-per-chain RAM: the factor lives on the device between runs, and chain offsets are invisible"""
    d = 70
    m = _model("normal", d)
    r = mc.SerialMC(steps=12, burnin=2, thinning=3)
    task = (m * mc.RAM() * r).batch(9, seed=21)
    c1 = mc.run(task)
    c2 = mc.run(c1)
    oc = orc.OracleChains(m, mc.RAM(), nchains=9, seed=21, order=order_for(d))
    s1, _, a1 = oc.run(r)
    s2, _, a2 = oc.run(r)
    assert_parity(c1, s1, None, a1, "ram")
    assert_parity(c2, s2, None, a2, "ram")
    _assert_ram_factor(task, oc, d)
    lo = mc.run((m * mc.RAM() * r).batch(5, seed=21))
    hi = mc.run((m * mc.RAM() * r).batch(4, seed=21, chain_offset=5))
    assert np.array_equal(np.concatenate([lo._samples, hi._samples], axis=2), s1)


def test_ram_limits(gpu):
    m = _model("iso", 1025)
    with pytest.raises(mc.MCMCError, match="RAM is built for d <= 1024"):
        mc.run((m * mc.RAM() * mc.SerialMC(steps=5)).batch(64))
    with pytest.raises(mc.MCMCError, match="d <= 1024"):      # regression targets: RAM up to the models' own cap
        m2 = mc.model(mc.LinearRegression(np.ones((20, 1025)), np.ones(20)), vars=np.zeros(1025), gradient=True)
        mc.run((m2 * mc.RAM() * mc.SerialMC(steps=5)).batch(64))


# ------------------------------------------------------------------ storeLeaps (HMC.jl:145-150, HMCDA.jl:110-117)
def _store_leaps_case(m, sp, C, seed, order, cap, steps=16, burnin=5, thinning=3):
    r = mc.SerialMC(steps=steps, burnin=burnin, thinning=thinning)
    chain = mc.run((m * sp * r).batch(C, seed=seed))
    lv = chain.diagnostics["leaps"]
    oc = orc.OracleChains(m, sp, nchains=C, seed=seed, order=order)
    s_ref, g_ref, acc_ref, lv_ref = oc.run_leaps(r, cap)
    assert np.array_equal(chain._samples.view(np.uint64), s_ref.view(np.uint64))   # the run itself is unchanged
    assert np.array_equal(chain.diagnostics["accept"].T, acc_ref.astype(bool))
    assert np.array_equal(lv["nleaps"], lv_ref["nleaps"])
    for k in ("pars", "grad", "m", "logTarget", "H"):
        a, b = lv[k], lv_ref[k]
        assert a.shape == b.shape
        assert np.array_equal(np.isnan(a), np.isnan(b)), k                         # NaN past nLeaps
        assert np.array_equal(np.nan_to_num(a).view(np.uint64), np.nan_to_num(b).view(np.uint64)), k


@pytest.mark.parametrize("sname", ["hmc", "hmc_tuned", "hmcda"])
@pytest.mark.parametrize("mkind,d", [("iso", 3), ("normal", 16), ("iso", 40), ("abs", 300)])
def test_store_leaps_bitwise(gpu, sname, mkind, d):
    """the trajectory record of every kept step, lane-per-chain (d <= 32) and wave-per-chain kernels"""
    sp = {"hmc": lambda: mc.HMC(4, 0.3, storeLeaps=True),
          "hmc_tuned": lambda: mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9), storeLeaps=True),
          "hmcda": lambda: mc.HMCDA(len=0.8, storeLeaps=True, max_leaps=40)}[sname]()
    _store_leaps_case(_model(mkind, d), sp, C=70, seed=31 + d, order=order_for(d), cap=sp.leaps_cap())


@pytest.mark.parametrize("sname", ["hmc", "hmcda"])
@pytest.mark.parametrize("kind,d", [("logistic", 5), ("linear", 37), ("linear", 200)])
def test_store_leaps_regression_bitwise(gpu, sname, kind, d):
    """the trajectory record on the fp64-MFMA regression kernels (single-slice and d-sliced)"""
    sp = mc.HMC(3, 0.02, storeLeaps=True) if sname == "hmc" else mc.HMCDA(len=0.1, storeLeaps=True, max_leaps=30)
    _store_leaps_case(_glm_model(kind, d), sp, C=40, seed=5 + d, order=0, cap=sp.leaps_cap())


@pytest.mark.parametrize("d", [4, 40])
@pytest.mark.parametrize("eps,nl", [(1e150, 30), (3.0, 250), (3.0, 262)])
def test_iso_hmc_overflowing_trajectories(gpu, d, eps, nl):
    """IsoDot HMC takes the half kick as (-x) eps (samplers.hpp trajectory_halfneg); trajectories whose |x| reaches
    2^1023, where -2x overflows, fall back to the model's gradient: bitwise the oracle's either way.  eps = 3 makes
    the leapfrog map unstable (|lambda| ~ 16): 250 leapfrogs stay just below the overflow, 262 cross it."""
    m = mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    r = mc.SerialMC(steps=12)
    ch = mc.run((m * mc.HMC(nl, eps) * r).batch(70, seed=6))
    oc = orc.OracleChains(m, mc.HMC(nl, eps), nchains=70, seed=6, order=order_for(d))
    s, g, acc = oc.run(r)
    assert_parity(ch, s, g, acc, "hmc")
    assert ch.task.evals == int(oc.n_evals.sum())


# ------------------------------------------------------------------ y = x * v; y ~ D (bare_distribs.jl)
from test_oracle import BARE_DISTRIBS, bare_start  # noqa: E402


@pytest.mark.parametrize("name,p", BARE_DISTRIBS)
def test_dist_obs_rwm100_bitwise(gpu, name, p):
    """benchmarks/benchunits/bare_distribs.jl's "100 RWM steps" unit (run(m * RWM(0.1), steps=100) from the
    distribution's mean) on 300 chains, and its "loglik and gradient eval", bitwise against the oracle."""
    m = mc.model(mc.DistObsDSL(name, *p), x=bare_start(name, p), gradient=True)
    r = mc.SerialMC(steps=100)
    chain = mc.run((m * mc.RWM(0.1) * r).batch(300, seed=13))
    oc = orc.OracleChains(m, mc.RWM(0.1), nchains=300, seed=13)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, "rwm")
    xs = bare_start(name, p) * np.linspace(0.8, 1.2, 33)[None, :]
    lp, g = m.evalallg(xs)
    lp_r, g_r = orc.eval_batch(m, xs)
    assert np.array_equal(lp, lp_r) and np.array_equal(g, g_r)


@pytest.mark.parametrize("sname", ["mala", "hmc", "hmcda"])
@pytest.mark.parametrize("name,p", [("Normal", (1, 1)), ("Gamma", (3, 0.2)), ("LogNormal", (2, 0.1))])
def test_dist_obs_gradient_samplers_bitwise(gpu, sname, name, p):
    v = np.linspace(0.5, 1.5, 200)
    m = mc.model(mc.DistObsDSL(name, *p, v=v), x=bare_start(name, p), gradient=True)
    sp = {"mala": lambda: mc.MALA(0.001), "hmc": lambda: mc.HMC(3, 0.005), "hmcda": lambda: mc.HMCDA(len=0.05)}[sname]
    r = mc.SerialMC(steps=30, burnin=5, thinning=2)
    chain = mc.run((m * sp() * r).batch(130, seed=4))
    oc = orc.OracleChains(m, sp(), nchains=130, seed=4)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname)


# ------------------------------------------------------------------ Ornstein-Uhlenbeck (examples/ornstein.jl:19-30)
from test_oracle import _ou_model  # noqa: E402

OU_SAMPLERS = {"rwm": lambda: mc.RWM(0.05), "mala": lambda: mc.MALA(1e-5), "hmc": lambda: mc.HMC(5, 0.002),
               "hmc_tuned": lambda: mc.HMC(3, 0.002, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9)),
               "hmcda": lambda: mc.HMCDA(len=0.01), "ram": lambda: mc.RAM()}


@pytest.mark.parametrize("sname", list(OU_SAMPLERS))
def test_ou_sampler_parity(gpu, sname):
    """The OU target (a joint, non-separable log-target over (tau, sigma, mu) and a 1 000-point series) on every
    sampler from the example's init and scale hint (ornstein.jl:29-30), 70 chains (a tail wave): samples,
    gradients, accept bits, final state and evaluation counts bitwise against the oracle."""
    m = _ou_model()
    r = mc.SerialMC(steps=40, burnin=6, thinning=3)
    task = (m * OU_SAMPLERS[sname]() * r).batch(70, seed=29)
    chain = mc.run(task)
    assert task.step_kernel.startswith("lpc_") and "OUDSL" in task.step_kernel
    oc = orc.OracleChains(m, OU_SAMPLERS[sname](), nchains=70, seed=29)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, sname.split("_")[0])
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    assert task.evals == int(oc.n_evals.sum())
    if sname == "ram":
        _assert_ram_factor(task, oc, 3)


def test_ou_example_runs_bitwise(gpu):
    """ornstein.jl:33-38 as written: one chain, run(m * RAM() * SerialMC(1000:10000)) and run(m * HMC(5, 0.002) *
    SerialMC(1000:10000)), bitwise against the oracle; RAM's chain recovers the simulating parameters."""
    m = _ou_model()
    r = mc.SerialMC(steps=10000, burnin=999)
    for sp in (mc.RAM, lambda: mc.HMC(5, 0.002)):
        chain = mc.run((m * sp() * r).batch(1, seed=1))
        oc = orc.OracleChains(m, sp(), nchains=1, seed=1)
        s_ref, g_ref, acc_ref = oc.run(r)
        assert np.array_equal(chain._samples, s_ref)
        assert np.array_equal(chain.diagnostics["accept"].T, acc_ref.astype(bool))
    chain = mc.run((m * mc.RAM() * r).batch(1, seed=1))
    tail = chain._samples[5000:, :, 0].mean(axis=0)
    assert abs(tail[2] - 10.0) < 0.5 and abs(tail[0] - 20.0) < 8.0 and abs(tail[1] - 0.1) < 0.02, tail


@pytest.mark.parametrize("C", [1, 5])
def test_ou_few_chain_rwm_bitwise(gpu, C):
    """RWM on the joint OU target with one chain (the path-speculation kernel lpc_rwm_spec, chosen for C == 1) and
    with a few chains (lpc_rwm_la): the joint log-target, not a per-coordinate sum, decides every step (ADVICE r4:
    a per-coordinate sum of a joint model is 0 and accepted every proposal), bitwise against the oracle."""
    m = _ou_model()
    r = mc.SerialMC(steps=400, burnin=50, thinning=7)
    task = (m * mc.RWM(0.05) * r).batch(C, seed=41)
    chain = mc.run(task)
    assert task.step_kernel.startswith("lpc_rwm_spec" if C == 1 else "lpc_rwm_la"), task.step_kernel
    oc = orc.OracleChains(m, mc.RWM(0.05), nchains=C, seed=41)
    s_ref, g_ref, acc_ref = oc.run(r)
    assert_parity(chain, s_ref, g_ref, acc_ref, "rwm")
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)
    acc = chain.diagnostics["accept"]
    assert 0 < acc.sum() < acc.size                           # some proposals rejected (out of support, or worse)


def test_ou_eval_and_limits(gpu):
    """model.eval / evalallg of the OU target on a batch (inside and outside the supports) bitwise against the
    oracle; a model with d != 3 or a series shorter than 2 is refused."""
    m = _ou_model()
    rng = np.random.default_rng(5)
    B = np.hstack([np.array([[0.05, 20.0, 100.0, -1.0, 5.0], [1.0, 0.1, 2.0, 1.0, 2.5], [1.0, 10.0, 20.0, 1.0, 1.0]]),
                   np.vstack([rng.uniform(0.5, 99, 60), rng.uniform(0.05, 2, 60), rng.uniform(0, 20, 60)])])
    lp, g = m.evalallg(B)
    lp_r, g_r = orc.eval_batch(m, B)
    assert np.array_equal(lp, lp_r) and np.array_equal(g, g_r)
    bad = mc.model(mc.OrnsteinUhlenbeck(mc.ou_series()), init=np.ones(4), gradient=True)
    with pytest.raises(mc.MCMCError, match="3 parameters"):
        bad.eval(np.ones(4))
    with pytest.raises(ValueError):
        mc.OrnsteinUhlenbeck([1.0])
