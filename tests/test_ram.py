"""RAM sampler (src/samplers/RAM.jl) -- constructors, the oracle's restatement against a literal
numpy transcription of RAM.jl, and the sampler's coerced acceptance rate.  CPU only."""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc
from mcmchip.api import unpack_ram_factor


def test_ram_constructors_and_asserts():
    """RAM.jl:22-34: RAM(), RAM(x), RAM(x, r), RAM(; scale, rate) and the two @asserts."""
    assert (mc.RAM().scale, mc.RAM().rate) == (1.0, 0.234)
    assert (mc.RAM(2.0).scale, mc.RAM(2.0).rate) == (2.0, 0.234)
    assert (mc.RAM(1.0, 0.3).scale, mc.RAM(1.0, 0.3).rate) == (1.0, 0.3)
    assert (mc.RAM(scale=0.5, rate=0.4).scale, mc.RAM(scale=0.5, rate=0.4).rate) == (0.5, 0.4)
    with pytest.raises(AssertionError, match="scale should be > 0"):
        mc.RAM(0.0)
    for r in (0.0, 1.0, -0.1, 1.5):
        with pytest.raises(AssertionError, match=r"target acceptance rate \(.*\) should be between 0 and 1"):
            mc.RAM(1.0, r)
    assert not mc.RAM().uses_gradient                  # RAM needs only model.eval (RAM.jl:52,61)


def _normals(chain, step, d):
    """the oracle's normals of (chain, step) with seed 0 (detmath op 6: blocks of 4)."""
    nb = (d + 3) // 4
    a = np.array([chain + (b << 32) for b in range(nb)], dtype=np.float64)
    return orc.detmath(6, a, np.full(nb, float(step)))[:d]


def _accept_u(chain, step):
    w = orc.philox(np.array([[chain, step, 0, 1]], dtype=np.uint32), np.zeros((1, 2), dtype=np.uint32))[0]
    m = (int(w[0]) >> 5 << 26) | (int(w[1]) >> 6)
    return m * 2.0 ** -53


def _ram_literal(m, sampler, chain, steps):
    """RAM.jl:50-78 transcribed literally in numpy: proposal pars + S*rvec, ratio > 0 || ratio > log(rand()),
    eta = min(1, d*i^(-2/3)), SS = S*(I + rvec*rvec'/dot(rvec,rvec)*eta*(min(1,exp(ratio))-rate))*S',
    S = chol(SS)'.  LAPACK's Cholesky replaces Julia's chol: agreement is to rounding, not bitwise."""
    d = m.size
    S = np.diag(np.asarray(m.scale, dtype=float) * sampler.scale)
    pars = np.asarray(m.init, dtype=float).copy()
    lt = orc.eval_batch(m, pars[:, None])[0][0]
    out, accs = [], []
    for i in range(1, steps + 1):
        rvec = _normals(chain, i, d)
        prop = pars + S @ rvec
        plt = orc.eval_batch(m, prop[:, None])[0][0]
        ratio = plt - lt
        acc = ratio > 0 or ratio > np.log(_accept_u(chain, i))
        if acc:
            pars, lt = prop, plt
        out.append(pars.copy())
        accs.append(acc)
        eta = min(1.0, d * i ** (-2.0 / 3.0))
        SS = np.outer(rvec, rvec) / rvec.dot(rvec) * eta * (min(1.0, np.exp(ratio)) - sampler.rate)
        SS = S @ (np.eye(d) + SS) @ S.T
        S = np.linalg.cholesky(SS)
    return np.array(out), np.array(accs), S


@pytest.mark.parametrize("mk,d", [("normal", 1), ("normal", 3), ("iso", 6), ("dist", 4)])
def test_oracle_ram_matches_literal_reference(mk, d):
    if mk == "normal":
        m = mc.model(mc.NormalDSL(0.3, 1.7), v=np.linspace(-1, 1, d), gradient=True)
    elif mk == "iso":
        m = mc.model(mc.IsoNormalDot(), init=np.linspace(0.5, 1.5, d), scale=np.linspace(0.8, 1.2, d))
    else:
        m = mc.model(mc.DistDSL("Gamma", 2.5, 0.7), v=np.full(d, 1.2))   # support edge: -Inf proposals
    sp = mc.RAM(0.8, 0.3)
    C, steps = 3, 120
    oc = orc.OracleChains(m, sp, nchains=C, seed=0)
    s, g, acc = oc.run(mc.SerialMC(steps=steps))
    assert g is None
    S_orc = unpack_ram_factor(oc.ram_L, d)
    for c in range(C):
        ref, racc, S_ref = _ram_literal(m, sp, c, steps)
        assert np.array_equal(acc[:, c].astype(bool), racc)
        np.testing.assert_allclose(s[:, :, c], ref, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(S_orc[c], S_ref, rtol=1e-9, atol=1e-12)
    assert (acc == 0).any() and (acc == 1).any()


def test_ram_factor_starts_at_scaled_diagonal():
    d = 5
    m = mc.model(mc.IsoNormalDot(), init=np.ones(d), scale=np.arange(1.0, d + 1))
    oc = orc.OracleChains(m, mc.RAM(0.5), nchains=4, seed=1)
    S = unpack_ram_factor(oc.ram_L, d)
    assert np.array_equal(S, np.broadcast_to(np.diag(0.5 * np.arange(1.0, d + 1)), (4, d, d)))


@pytest.mark.parametrize("rate", [0.234, 0.5])
def test_ram_coerces_acceptance_rate(rate):
    """Vihola (2012): the adapted factor drives the acceptance rate to the target."""
    m = mc.model(mc.NormalDSL(0.0, 2.0), v=np.zeros(4))
    oc = orc.OracleChains(m, mc.RAM(0.1, rate), nchains=32, seed=7)
    _, _, acc = oc.run(mc.SerialMC(steps=4000))
    assert abs(acc[2000:].mean() - rate) < 0.03


def test_linear_regression_example_acceptance():
    """examples/linear_regression.jl:26-30: RAM(1., 0.3) on 1000 obs x 10 vars, acceptance ~29.7 %."""
    rng = np.random.default_rng(1)
    n, d = 1000, 10
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1))])
    Y = X @ rng.normal(size=d) + rng.normal(size=n)
    m = mc.model(mc.LinearRegression(X, Y), vars=np.zeros(d), gradient=True)
    oc = orc.OracleChains(m, mc.RAM(1.0, 0.3), nchains=8, seed=3)
    s, _, acc = oc.run(mc.SerialMC(steps=6000, burnin=1000))
    assert abs(acc.mean() - 0.3) < 0.03
    beta_hat = np.linalg.solve(X.T @ X + np.eye(d), X.T @ Y)       # posterior mean with the N(0,1) prior
    np.testing.assert_allclose(s.mean(axis=(0, 2)), beta_hat, atol=0.02)


def test_ram_continuation_and_sharding():
    """S persists across run(chain) continuations (the task keeps it) and chains are keyed by global id."""
    m = mc.model(mc.NormalDSL(0.5, 1.5), v=np.zeros(5))
    a = orc.OracleChains(m, mc.RAM(), nchains=7, seed=9)
    a.run(mc.SerialMC(steps=40))
    s2, _, acc2 = a.run(mc.SerialMC(steps=40))
    b = orc.OracleChains(m, mc.RAM(), nchains=7, seed=9)
    s, _, acc = b.run(mc.SerialMC(steps=80))
    assert np.array_equal(s2, s[40:]) and np.array_equal(acc2, acc[40:])
    assert np.array_equal(a.ram_L, b.ram_L)
    lo = orc.OracleChains(m, mc.RAM(), nchains=3, seed=9)
    hi = orc.OracleChains(m, mc.RAM(), nchains=4, seed=9, chain_offset=3)
    s_lo, _, _ = lo.run(mc.SerialMC(steps=80))
    s_hi, _, _ = hi.run(mc.SerialMC(steps=80))
    assert np.array_equal(np.concatenate([s_lo, s_hi], axis=2), s)
