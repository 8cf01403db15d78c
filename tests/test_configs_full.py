"""BASELINE.json configs 4 and 5 at their own sizes, bitwise against the oracle on the GPU.

- config 5: Bayesian linear regression n=4096, d=512 (examples/linear_regression.jl:14-20; bench.py's
  `regression_data("linear", 4096, 512)`), `HMCDA()` with the reference defaults (HMCDA.jl:42-43: rate 0.65,
  len 2, shrinkage 0.05, t0 10, step 0.75).  d = 512 is the only regression width with no zero-padded columns of
  the d-sliced kernel `glm_hmc<8, 4, true>` (4 waves of 128 coordinates per 16 chains, two tiles a workgroup), and n = 4096 runs 256 observation tiles
  per evaluation.  With the NaN-initialised step (epsilon_0 = 1, HMCDA.jl:86-92) the first dual-averaging steps
  take trajectories of 2, 1, 2, 7 leapfrogs; by the fifth adapted step epsilon is ~0.07 and a step takes ~28
  leapfrogs of the default len = 2 -- so SerialMC(steps=7, burnin=5) runs the default trajectory length, not the
  one-leapfrog degenerate chain a 2-step burnin gives.  Samples, gradients, accept bits, final state, evaluation
  counts and the adapted step sizes (leapStep and dualLeapStep, HMCDA.jl:136-140) are compared bit for bit.
- the same workload over a group of 8 blocks (mcmc_group_*, 512 chains = 8 x 64), equal to one context bit for
  bit, and the last block's tail tile against the oracle.
- config 4: d = 1024 iso-Normal, HMC(10, 0.1), init ones(1024) (the wave-per-chain kernel
  `wpc_hmc<4, true, IsoDot, false>`).
"""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc

pytestmark = pytest.mark.gpu

ORC_THREADS = 16            # the GPU box's CPU share


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def _config5_model():
    from bench import regression_data
    X, Y = regression_data("linear", 4096, 512)
    return mc.model(mc.LinearRegression(X, Y), vars=np.zeros(512), gradient=True)


def _check_chain(chain, oc, s_ref, g_ref, acc_ref, grads=True):
    acc = chain.diagnostics["accept"].T
    assert np.array_equal(acc, acc_ref.astype(bool)), f"accept bits differ in {np.count_nonzero(acc != acc_ref)}"
    np.testing.assert_allclose(chain._samples, s_ref, rtol=1e-10, atol=0)          # north_star tolerance
    assert _bits_equal(chain._samples, s_ref), "samples not bit-identical"
    if grads:
        assert _bits_equal(chain._gradients, g_ref), "gradients not bit-identical"
    assert _bits_equal(chain.final_x, oc.x) and _bits_equal(chain.final_lp, oc.lp)


def test_config5_linear512_hmcda_defaults(gpu):
    m = _config5_model()
    C = 40                                   # two full 16-chain tiles and a tail tile of 8
    r = mc.SerialMC(steps=7, burnin=5)
    t = (m * mc.HMCDA() * r).batch(C, seed=5)
    chain = mc.run(t)
    assert t.step_kernel == "glm_hmc<8, 4, true>"
    oc = orc.OracleChains(m, mc.HMCDA(), nchains=C, seed=5)
    s_ref, g_ref, acc_ref = oc.run(r, nthreads=ORC_THREADS)
    _check_chain(chain, oc, s_ref, g_ref, acc_ref)
    assert t.evals == int(oc.n_evals.sum())
    ts = t.tuner_state()
    assert _bits_equal(ts["step"], oc.t_step), "adapted leapStep differs"
    assert _bits_equal(ts["step_bar"], oc.t_bar), "dualLeapStep differs"
    # the default trajectory length is exercised: after the adaptation steps a step takes len/eps >> 2 leapfrogs
    assert np.all(np.round(2.0 / oc.t_step) >= 10), oc.t_step
    assert t.evals / (C * r.len) > 10


def test_config5_group_of_8_blocks(gpu):
    m = _config5_model()
    C = 512
    r = mc.SerialMC(steps=7, burnin=5)
    one_t = (m * mc.HMCDA() * r).batch(C, seed=9)
    one = mc.run(one_t)
    task = (m * mc.HMCDA() * r).batch(C, seed=9, devices=(0,) * 8)
    grp = mc.run(task)
    assert [b[2] for b in task.blocks()] == [64] * 8
    assert _bits_equal(grp._samples, one._samples) and _bits_equal(grp._gradients, one._gradients)
    assert np.array_equal(grp.diagnostics["accept"], one.diagnostics["accept"])
    assert _bits_equal(grp.final_x, one.final_x) and task.evals == one_t.evals
    assert _bits_equal(task.tuner_state()["step_bar"], one_t.tuner_state()["step_bar"])
    # the last block's last 32 chains (a tile boundary inside the block) against the oracle, keyed by global id
    c0 = 480
    oc = orc.OracleChains(m, mc.HMCDA(), nchains=32, seed=9, chain_offset=c0)
    s_ref, g_ref, acc_ref = oc.run(r, nthreads=ORC_THREADS)
    assert _bits_equal(grp._samples[:, :, c0:], s_ref) and _bits_equal(grp._gradients[:, :, c0:], g_ref)
    assert np.array_equal(grp.diagnostics["accept"][c0:].T, acc_ref.astype(bool))
    assert _bits_equal(grp.final_x[:, c0:], oc.x)


def test_config4_hmc1024_as_configured(gpu):
    d = 1024
    m = mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    C = 130                                  # 32 full 4-chain workgroups and a partial one
    r = mc.SerialMC(steps=40, burnin=10, thinning=6)
    t = (m * mc.HMC(10, 0.1) * r).batch(C, seed=4)
    chain = mc.run(t)
    assert t.step_kernel == "wpc_hmc<4, true, IsoDot, false>"
    oc = orc.OracleChains(m, mc.HMC(10, 0.1), nchains=C, seed=4, order=1)
    s_ref, g_ref, acc_ref = oc.run(r, nthreads=ORC_THREADS)
    _check_chain(chain, oc, s_ref, g_ref, acc_ref)
    assert t.evals == int(oc.n_evals.sum())
    assert 0.2 < acc_ref.mean() < 1.0
