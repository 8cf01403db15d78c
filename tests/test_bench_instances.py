"""The exact kernel instances the benchmarks dispatch, parity-tested on the GPU.

bench.py's RWM workloads use README.md:60's model (`-dot(v,v)`, init `ones(d)`, no model scale) under
`RWM(0.1)` (README.md:85): every coordinate's effective scale `model.scale .* sampler.scale` (RWM.jl:52) is the
same, so the runtime launches the uniform-scale specialisations (`scale1` in a scalar register).  These tests
run those workloads' own configurations, read back which step kernel ran (`mcmc_chains_step_kernel`), and
compare the HIP results with the oracle bit for bit:

- config 2 (d=3) -> `lpc_rwm<1, false, IsoDot, true>`; the metric (d=32) -> `lpp_rwm<4, true, IsoDot, true>` (two
  lanes per chain, samplers.hpp PairChain);
- config 1 (one chain, d <= 4) -> the path-speculation kernel `lpc_rwm_spec`; C <= 64 -> the
  look-ahead kernel `lpc_rwm_la`; both also across launches
  (`steps_per_launch`) and continued runs, where a launch starts mid-way through the kept range;
- the metric at its full size: 2^20 chains, d=32, SerialMC(1000, 100, 10) with device-resident outputs,
  checked bitwise on 4 096 chains spread over the batch and on every chain's accept bits' statistics.
"""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc

pytestmark = pytest.mark.gpu


def _readme_model(d):
    return mc.model(mc.IsoNormalDot(), init=np.ones(d))          # README.md:60 (d = 3), bench.py's RWM model


def _check(chain, s_ref, acc_ref):
    acc = chain.diagnostics["accept"].T
    assert np.array_equal(acc, acc_ref.astype(bool)), f"accept bits differ in {np.count_nonzero(acc != acc_ref)}"
    np.testing.assert_allclose(chain._samples, s_ref, rtol=1e-10, atol=0)      # north_star tolerance
    assert np.array_equal(chain._samples.view(np.uint64), s_ref.view(np.uint64)), "samples not bit-identical"


@pytest.mark.parametrize("d,C,kernel", [
    (3, 1000, "lpc_rwm<1, false, IsoDot, true>"),      # config 2's instance
    (32, 1000, "lpp_rwm<4, true, IsoDot, true>"),      # the metric's instance
    (4, 300, "lpc_rwm<1, true, IsoDot, true>"),
    (16, 300, "lpc_rwm<4, true, IsoDot, true>"),       # the last lane-per-chain width
    (17, 130, "lpp_rwm<3, false, IsoDot, true>"),
    (24, 130, "lpp_rwm<3, true, IsoDot, true>"),
    (30, 97, "lpp_rwm<4, false, IsoDot, true>"),
    (32, 65, "lpp_rwm<4, true, IsoDot, true>"),        # one chain past the look-ahead limit
    (32, 64, "lpc_rwm_la<8, IsoDot, true>"),           # the look-ahead kernel in the pair kernels' sum order
])
def test_uniform_scale_rwm_instances(gpu, d, C, kernel):
    m = _readme_model(d)
    r = mc.SerialMC(steps=200, burnin=20, thinning=10)
    t = (m * mc.RWM(0.1) * r).batch(C, seed=1)
    chain = mc.run(t)
    assert t.step_kernel == kernel
    oc = orc.OracleChains(m, mc.RWM(0.1), nchains=C, seed=1)
    s_ref, _, acc_ref = oc.run(r)
    _check(chain, s_ref, acc_ref)
    assert np.array_equal(chain.final_x, oc.x) and np.array_equal(chain.final_lp, oc.lp)


def test_nonuniform_scale_takes_the_generic_instance(gpu):
    m = mc.model(mc.IsoNormalDot(), init=np.ones(32), scale=np.linspace(0.8, 1.2, 32))
    t = (m * mc.RWM(0.1) * mc.SerialMC(steps=10)).batch(128, seed=1)
    mc.run(t)
    assert t.step_kernel == "lpp_rwm<4, true, IsoDot, false>"


@pytest.mark.parametrize("uniform", [True, False])
@pytest.mark.parametrize("spl", [0, 1, 7])
@pytest.mark.parametrize("C", [1, 2, 5, 32, 33, 37, 64])
def test_lookahead_rwm_across_launches_and_runs(gpu, C, spl, uniform):
    """few-chain RWM kernels: lpc_rwm_spec (one chain, d <= 4: path speculation, 6 steps per block, blocks cut
    by launch boundaries) and lpc_rwm_la (C <= 64).  With steps_per_launch 1 or 7 and a continued
    run, launches begin inside the kept range (the kept-step counter restarts from step_begin - run_step0 >
    burnin + 1)."""
    d = 3
    m = (_readme_model(d) if uniform else
         mc.model(mc.IsoNormalDot(), init=np.ones(d), scale=np.array([0.8, 1.0, 1.3])))
    r = mc.SerialMC(steps=150, burnin=20, thinning=7)
    t = (m * mc.RWM(0.1) * r).batch(C, seed=3, steps_per_launch=spl)
    c1 = mc.run(t)
    c2 = mc.run(c1)                                               # runners.jl:14: the same chains continue
    us = "true" if uniform else "false"
    assert t.step_kernel == (f"lpc_rwm_spec<3, IsoDot, {us}>" if C == 1 else f"lpc_rwm_la<1, IsoDot, {us}>")
    oc = orc.OracleChains(m, mc.RWM(0.1), nchains=C, seed=3)
    s1, _, a1 = oc.run(r)
    s2, _, a2 = oc.run(r)
    _check(c1, s1, a1)
    _check(c2, s2, a2)
    assert t.steps_done == 300


def test_readme_config1_instance(gpu):
    """config 1 exactly: README.md:60,85 run(mymodel1, RWM(0.1), SerialMC(steps=1000, burnin=100)), one chain."""
    m1 = _readme_model(3)
    t = (m1 * mc.RWM(0.1) * mc.SerialMC(steps=1000, burnin=100)).batch(1, seed=1)
    ch = mc.run(t)
    assert t.step_kernel == "lpc_rwm_spec<3, IsoDot, true>"
    oc = orc.OracleChains(m1, mc.RWM(0.1), nchains=1, seed=1)
    s, _, acc = oc.run(mc.SerialMC(steps=1000, burnin=100))
    _check(ch, s, acc)
    assert ch.samples.shape == (1, 900, 3)


def test_full_size_metric_run(gpu):
    """The metric workload at its full size (BASELINE.json metric; bench.py --config metric --steps 1000):
    2^20 chains, d=32, init ones(32), RWM(0.1), SerialMC(steps=1000, burnin=100, thinning=10), seed 1, outputs
    resident on the device.  4 096 chains -- 64 blocks of 64 spread over the batch, the first and last chain
    included -- are compared bit for bit with the oracle (the oracle keys its stream by global chain id, so a
    block at chain_offset k is exactly chains k..k+63 of the full run).  Every chain: the accept fraction and
    the final moments agree with the subset's within their sampling error."""
    import ctypes as ct
    import torch
    from mcmchip import _lib

    d, C = 32, 1 << 20
    m = _readme_model(d)
    r = mc.SerialMC(steps=1000, burnin=100, thinning=10)
    t = (m * mc.RWM(0.1) * r).batch(C, seed=1)
    h = t.handle()
    lib = _lib.load()
    nk = len(r.r)
    dev = torch.device("cuda", 0)
    samples = torch.empty((nk, d, C), dtype=torch.float64, device=dev)
    bits = torch.empty((nk, C // 64), dtype=torch.int64, device=dev)
    fx = torch.empty((d, C), dtype=torch.float64, device=dev)
    out = _lib.Outputs()
    out.samples, out.accept_bits, out.final_x = samples.data_ptr(), bits.data_ptr(), fx.data_ptr()
    out.on_device = 1
    cfg = r.cfg()
    _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(out)))
    torch.cuda.synchronize(dev)
    assert t.step_kernel == "lpp_rwm<4, true, IsoDot, true>"
    assert out.nkept == 90

    starts = np.unique(np.linspace(0, C - 64, 64).astype(np.int64) // 64 * 64)
    assert len(starts) == 64 and starts[0] == 0 and starts[-1] == C - 64
    acc_sub = []
    for c0 in starts:
        oc = orc.OracleChains(m, mc.RWM(0.1), nchains=64, seed=1, chain_offset=int(c0))
        s_ref, _, a_ref = oc.run(r)
        s_gpu = samples[:, :, c0:c0 + 64].cpu().numpy()
        assert np.array_equal(s_gpu.view(np.uint64), s_ref.view(np.uint64)), f"samples of chains {c0}.. differ"
        w = bits[:, c0 // 64].cpu().numpy().view(np.uint64)
        a_gpu = ((w[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8)
        assert np.array_equal(a_gpu, a_ref), f"accept bits of chains {c0}.. differ"
        assert np.array_equal(fx[:, c0:c0 + 64].cpu().numpy(), oc.x)
        acc_sub.append(a_ref)
    acc_sub = np.concatenate(acc_sub, axis=1)
    # every chain: accept fraction per kept step and overall, from the ballot words
    b = bits.view(torch.uint8)
    table = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.float64, device=dev)
    pop = table[b.long()].sum(dim=1)
    rate_all = float(pop.sum()) / (nk * C)
    rate_sub = acc_sub.mean()
    se = np.sqrt(rate_sub * (1 - rate_sub) / acc_sub.size)
    assert abs(rate_all - rate_sub) < 6 * se + 1e-3, (rate_all, rate_sub)
    # final state moments over all chains vs the 4 096-chain subset (chains are i.i.d. replicas)
    mean_all = fx.mean(dim=1).cpu().numpy()
    var_all = fx.var(dim=1).cpu().numpy()
    sub = np.concatenate([fx[:, c0:c0 + 64].cpu().numpy() for c0 in starts], axis=1)
    se_mean = np.sqrt(sub.var(axis=1) / sub.shape[1])
    assert np.all(np.abs(mean_all - sub.mean(axis=1)) < 6 * se_mean)
    assert np.all(np.abs(var_all / sub.var(axis=1) - 1) < 6 * np.sqrt(2 / sub.shape[1]))
    assert bool(torch.isfinite(samples).all())


@pytest.mark.parametrize("d", [1, 3, 4, 5, 8, 9])
@pytest.mark.parametrize("C", [1, 3, 16])
def test_few_chain_rwm_models_and_sizes(gpu, C, d):
    """the few-chain kernels on every separable model, d across the lpc_rwm_spec / lpc_rwm_la boundary (d <= 4),
    out-of-support proposals included (AbsNormal's -Inf branch does not arise; DistDSL Gamma rejects x <= 0)"""
    models = [mc.model(mc.IsoNormalDot(), init=np.linspace(0.5, 1.5, d), grad=True),
              mc.model(mc.NormalDSL(0.3, 1.7), v=np.linspace(-1, 1, d), gradient=True),
              mc.model(mc.DistDSL("Gamma", 3, 0.2), x=np.full(d, 0.6), gradient=True)]
    r = mc.SerialMC(steps=97, burnin=9, thinning=4)
    for m in models:
        sp = mc.RWM(0.4)
        ch = mc.run((m * sp * r).batch(C, seed=8))
        assert ch.task.step_kernel.startswith("lpc_rwm_spec" if d <= 4 and C == 1 else "lpc_rwm_la")
        oc = orc.OracleChains(m, mc.RWM(0.4), nchains=C, seed=8)
        s, _, acc = oc.run(r)
        _check(ch, s, acc)
        assert np.array_equal(ch.final_x, oc.x) and np.array_equal(ch.final_lp, oc.lp)
        assert ch.task.evals == C * 97


@pytest.mark.parametrize("tuned", [False, True])
@pytest.mark.parametrize("link_sign", [1.0, -1.0])
@pytest.mark.parametrize("prior", [1.0, 2.5])
def test_config3_logistic_mala_instance(gpu, tuned, link_sign, prior):
    """config 3's kernel: logistic regression n=1000, d=128 under MALA(0.001) (test/test_syntax.jl:28's sampler),
    the wave-specialised glm_mala1ws<8> (M and V waves on one SIMD); 200 chains (a partial 64-chain workgroup),
    bitwise against the oracle over several launches (one step per launch), tuned and untuned, both link signs, the
    unit prior (its instance skips the exact x / 1 divisions) and another."""
    from test_gpu_parity import _glm_model
    m0 = _glm_model("logistic", 128, n=1000)
    X, Y = m0.target.X, m0.target.Y
    m = mc.model(mc.LogisticRegression(X, Y, prior_sigma=prior, link_sign=link_sign), vars=np.zeros(128),
                 gradient=True)
    smp = (lambda: mc.MALA(0.001, mc.EmpMCTuner(0.6, adaptStep=2))) if tuned else (lambda: mc.MALA(0.001))
    r = mc.SerialMC(steps=5, burnin=1, thinning=2)
    t = (m * smp() * r).batch(200, seed=31)
    chain = mc.run(t)
    assert t.step_kernel == ("glm_mala1ws<8, true>" if prior == 1.0 else "glm_mala1ws<8>")
    oc = orc.OracleChains(m, smp(), nchains=200, seed=31)
    s_ref, g_ref, acc_ref = oc.run(r)
    _check(chain, s_ref, acc_ref)
    assert np.array_equal(chain._gradients.view(np.uint64), g_ref.view(np.uint64)), "gradients not bit-identical"
    assert np.array_equal(chain.final_lp, oc.lp)


@pytest.mark.parametrize("d,scale,spl", [(2, 1.5, 0), (4, 1.5, 0), (3, 0.1, 0), (3, 0.6, 700), (1, 3.0, 999)])
def test_speculation_long_and_rejecting(gpu, d, scale, spl):
    """lpc_rwm_spec (one chain, d <= 4): 2 500 steps (13 stage halves of pre-drawn increments), at acceptance rates
    from ~96 % down to ~10 %, over one launch or launches of 700 / 999 steps (blocks cut by launch boundaries);
    thinning 3 with a burnin that ends inside a 6-step block."""
    m = mc.model(mc.IsoNormalDot(), init=np.linspace(0.5, 1.0, d))
    r = mc.SerialMC(steps=2500, burnin=37, thinning=3)
    t = (m * mc.RWM(scale) * r).batch(1, seed=11, steps_per_launch=spl)
    ch = mc.run(t)
    assert t.step_kernel.startswith("lpc_rwm_spec")
    oc = orc.OracleChains(m, mc.RWM(scale), nchains=1, seed=11)
    s, _, acc = oc.run(r)
    _check(ch, s, acc)
    assert np.array_equal(ch.final_x, oc.x) and np.array_equal(ch.final_lp, oc.lp)
    assert t.evals == 2500
