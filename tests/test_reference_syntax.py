"""The reference's own smoke configuration, test/test_syntax.jl:7-34, on the HIP path.

n = 1000 observations, nbeta = 10: X = [ones(n) randn(n, 9)], beta0 = randn(10),
Y = rand(n) .< 1 ./ (1 + exp(X * beta0)) (:8-13), and the DSL model with prob = 1 / (1 + exp(X * vars)) (:16-22):
the sign variant of examples/logistic_regression.jl (MCMC_MODEL_LOGISTIC, link_sign = -1).  Its samplers and
runners (:25-34): RWM(0.05), HMC(2, 0.1), MALA(0.001) under SerialMC(100:1000); RWM() under
SerialMC(steps=1000, thinning=10, burnin=0); HMC(2, 0.1) under SerialMC(thinning=10, burnin=0) and
SerialMC(burnin=20).  (NUTS, :27, is outside the hot path: SURVEY.md §2.)  The reference only runs them;
here every case runs on the GPU for a batch of chains and is compared bit for bit with the oracle.  The data
come from numpy's Philox (srand(1)'s dSFMT stream cannot be replayed).
"""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc

pytestmark = pytest.mark.gpu


def syntax_model():
    g = np.random.Generator(np.random.Philox(key=1))
    n, nbeta = 1000, 10
    X = np.hstack([np.ones((n, 1)), g.standard_normal((n, nbeta - 1))])
    beta0 = g.standard_normal(nbeta)
    Y = (g.random(n) < 1.0 / (1.0 + np.exp(X @ beta0))).astype(np.float64)
    return mc.model(mc.LogisticRegression(X, Y, link_sign=-1.0), vars=np.zeros(nbeta), gradient=True)


CASES = {
    "rwm_100:1000": (lambda: mc.RWM(0.05), lambda: mc.SerialMC(range(100, 1001))),
    "hmc_100:1000": (lambda: mc.HMC(2, 0.1), lambda: mc.SerialMC(range(100, 1001))),
    "mala_100:1000": (lambda: mc.MALA(0.001), lambda: mc.SerialMC(range(100, 1001))),
    "rwm_default_thin10": (lambda: mc.RWM(), lambda: mc.SerialMC(steps=1000, thinning=10, burnin=0)),
    "hmc_thin10": (lambda: mc.HMC(2, 0.1), lambda: mc.SerialMC(thinning=10, burnin=0)),
    "hmc_burnin20": (lambda: mc.HMC(2, 0.1), lambda: mc.SerialMC(burnin=20)),
}


@pytest.mark.parametrize("case", list(CASES))
def test_syntax_cases_bitwise(gpu, case):
    m = syntax_model()
    sf, rf = CASES[case]
    C = 100                                              # not a multiple of 16 or 64: tail tiles
    ch = mc.run((m * sf() * rf()).batch(C, seed=17))
    oc = orc.OracleChains(m, sf(), nchains=C, seed=17)
    s, g, acc = oc.run(rf())
    assert np.array_equal(ch._samples.view(np.uint64), s.view(np.uint64))
    assert np.array_equal(ch.diagnostics["accept"].T, acc.astype(bool))
    if ch._gradients is not None:
        assert np.array_equal(ch._gradients.view(np.uint64), g.view(np.uint64))
    assert np.isfinite(ch._samples).all()
    assert ch.diagnostics["step"] == list(rf().r)


def test_syntax_model_posterior_sign(gpu):
    """With prob = 1/(1+exp(X*vars)) the posterior mean of vars has the sign of the generating beta0 (the
    data were drawn with the same link): checks the link_sign = -1 branch end to end on the device."""
    m = syntax_model()
    g = np.random.Generator(np.random.Philox(key=1))
    g.standard_normal((1000, 9))
    beta0 = g.standard_normal(10)
    ch = mc.run((m * mc.MALA(0.001) * mc.SerialMC(range(500, 3001))).batch(256, seed=3))
    post = ch._samples.mean(axis=(0, 2))
    big = np.abs(beta0) > 0.3
    assert np.all(np.sign(post[big]) == np.sign(beta0[big])), (post, beta0)
