"""Multi-GPU through the C ABI (include/mcmc_hip.h, mcmc_group_*): one host thread drives a node's GPUs.

Replaces the reference's prun -> pmap of independent tasks over processes (src/runners/runners.jl:35-42,
examples/parallel_serialmc.jl:1-8).  A group splits one chain batch into contiguous blocks of whole 64-chain
groups, one per listed device, runs every block's step loop concurrently (a library worker thread per block)
and gathers the outputs device -> host into the caller's buffers.  The Philox streams are keyed by global chain
id, so a group run must equal a one-context run of the same batch bit for bit, whatever the split.  The box has
one GPU, so the GPU tests list device 0 several times: several contexts on one GPU, driven concurrently by
their worker threads -- the same code path as one block per GPU.  The CPU tests cover the block plan (host
arithmetic only).
"""
import ctypes as ct
import threading

import numpy as np
import pytest

import mcmchip as mc
from mcmchip import _lib


def plan(C, G):
    f = (ct.c_int64 * G)()
    n = (ct.c_int64 * G)()
    _lib.check(_lib.load().mcmc_group_plan(C, G, f, n))
    return list(f), list(n)


@pytest.mark.parametrize("C,G", [(1, 1), (1, 8), (64, 2), (100, 2), (1000, 3), (1 << 20, 8), (524288, 8),
                                 (65536, 8), (200, 3), (129, 2), (4097, 8)])
def test_plan_contiguous_64_aligned(C, G):
    f, n = plan(C, G)
    assert sum(n) == C
    pos = 0
    for g in range(G):
        assert f[g] == min(pos, C) and n[g] >= 0
        assert f[g] % 64 == 0 or n[g] == 0
        pos = f[g] + n[g]
    assert max(n) - min(x for x in n if x > 0) <= 64 * G or G == 1
    if C % (64 * G) == 0:                                       # the BASELINE shards: equal blocks
        assert len(set(n)) == 1


def test_plan_rejects_bad_arguments():
    f = (ct.c_int64 * 2)()
    assert _lib.load().mcmc_group_plan(0, 2, f, f) == _lib.MCMC_E_INVALID_ARG
    assert _lib.load().mcmc_group_plan(10, 0, f, f) == _lib.MCMC_E_INVALID_ARG


def _same(a, b):
    assert np.array_equal(a._samples.view(np.uint64), b._samples.view(np.uint64))
    if a._gradients is not None or b._gradients is not None:
        assert np.array_equal(a._gradients.view(np.uint64), b._gradients.view(np.uint64))
    assert np.array_equal(a.diagnostics["accept"], b.diagnostics["accept"])
    assert np.array_equal(a.final_x.view(np.uint64), b.final_x.view(np.uint64))
    assert np.array_equal(a.final_lp.view(np.uint64), b.final_lp.view(np.uint64))


def _logistic(d=8, n=40):
    rng = np.random.default_rng(4)
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, d - 1))])
    Y = (rng.random(n) < 0.5).astype(float)
    return mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(d), gradient=True)


CASES = {
    # (model, sampler, runner, nchains): lane-per-chain, wave-per-chain and regression layouts
    "rwm32": lambda: (mc.model(mc.IsoNormalDot(), init=np.ones(32), grad=True), mc.RWM(0.1),
                      mc.SerialMC(steps=60, burnin=10, thinning=5), 1000),
    "hmc3": lambda: (mc.model(mc.IsoNormalDot(), init=np.ones(3), grad=True), mc.HMC(3, 0.2),
                     mc.SerialMC(steps=30, burnin=5, thinning=3), 200),
    "mala64": lambda: (mc.model(mc.IsoNormalDot(), init=np.ones(64), grad=True), mc.MALA(0.05),
                       mc.SerialMC(steps=20, burnin=2, thinning=2), 300),
    "logistic_mala": lambda: (_logistic(), mc.MALA(0.01), mc.SerialMC(steps=10, burnin=2, thinning=3), 257),
    "hmcda_dist": lambda: (mc.model(mc.DistDSL("Gamma", 3, 0.2), x=0.6, gradient=True), mc.HMCDA(),
                           mc.SerialMC(steps=40, burnin=20), 130),
}


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0)])
@pytest.mark.parametrize("case", list(CASES))
def test_group_equals_one_context(gpu, case, devices):
    m, s, r, C = CASES[case]()
    one = mc.run((m * s * r).batch(C, seed=11))
    task = (m * s * r).batch(C, seed=11, devices=devices)
    grp = mc.run(task)
    _same(grp, one)
    assert grp.diagnostics["gather_s"] >= 0.0
    assert task.evals == one.task.evals
    assert task.steps_done == one.task.steps_done == r.len
    # continue (run(chain), runners.jl:14) and resume (SerialMC.jl:93-97) on the group
    _same(mc.run(grp), mc.run(one))
    _same(mc.resume(grp, steps=7), mc.resume(one, steps=7))


@pytest.mark.gpu
def test_group_per_chain_init_and_offset(gpu):
    m = mc.model(mc.IsoNormalDot(), init=np.ones(4), grad=True)
    C = 333
    x0 = np.random.default_rng(2).normal(size=(4, C))
    r = mc.SerialMC(steps=25, burnin=5, thinning=4)
    one = mc.run((m * mc.MALA(0.1) * r).batch(C, seed=3, init_x=x0, chain_offset=1000))
    grp = mc.run((m * mc.MALA(0.1) * r).batch(C, seed=3, init_x=x0, chain_offset=1000, devices=(0, 0, 0)))
    _same(grp, one)


@pytest.mark.gpu
def test_group_blocks_are_the_plan(gpu):
    m, s, r, C = CASES["hmc3"]()
    task = (m * s * r).batch(C, seed=1, devices=(0, 0, 0))
    bl = task.blocks()
    f, n = plan(C, 3)
    assert [(b[1], b[2]) for b in bl] == list(zip(f, n))
    assert bl[2][0] is None and n[2] == 0                      # 200 chains over 3: 128 + 72 + an empty block


@pytest.mark.gpu
def test_group_bad_device_fails_loudly(gpu):
    g = ct.c_void_p()
    devs = (ct.c_int32 * 2)(0, 999)
    rc = _lib.load().mcmc_group_create(devs, 2, ct.byref(g))
    assert rc == _lib.MCMC_E_INVALID_ARG
    assert b"device ordinal" in _lib.load().mcmc_last_error()


@pytest.mark.gpu
def test_group_rejects_device_outputs(gpu):
    m, s, r, C = CASES["hmc3"]()
    task = (m * s * r).batch(C, seed=1, devices=(0, 0))
    out = _lib.Outputs()
    out.on_device = 1
    cfg = r.cfg()
    rc = _lib.load().mcmc_group_run_serialmc(task.handle(), ct.byref(cfg), ct.byref(out), None)
    assert rc == _lib.MCMC_E_INVALID_ARG


@pytest.mark.gpu
def test_two_host_threads_two_contexts_one_gpu(gpu):
    """Distinct contexts are independent: two host threads each drive their own context on the same GPU at
    once (ctypes releases the GIL inside the C calls); each result equals the same run done alone."""
    lib = _lib.load()
    m = mc.model(mc.IsoNormalDot(), init=np.ones(32), grad=True)
    r = mc.SerialMC(steps=200, burnin=20, thinning=10)
    C = 4096
    alone = [mc.run((m * mc.RWM(0.1) * r).batch(C, seed=s)) for s in (1, 2)]
    res = [None, None]
    err = []

    def worker(i, seed):
        try:
            ctx, mh, ch = ct.c_void_p(), ct.c_void_p(), ct.c_void_p()
            _lib.check(lib.mcmc_ctx_create(0, ct.byref(ctx)))
            desc = m._desc()
            _lib.check(lib.mcmc_model_create(ctx, ct.byref(desc), ct.byref(mh)))
            cfg = mc.RWM(0.1).cfg()
            _lib.check(lib.mcmc_chains_create(mh, ct.byref(cfg), C, 0, seed, None, ct.byref(ch)))
            nk = len(r.r)
            s = np.empty((nk, 32, C))
            b = np.zeros((nk, C // 64), dtype=np.uint64)
            out = _lib.Outputs()
            out.samples = s.ctypes.data
            out.accept_bits = b.ctypes.data
            rc = r.cfg()
            for _ in range(3):                                   # overlap several runs of both threads
                _lib.check(lib.mcmc_chains_reset(ch))
                _lib.check(lib.mcmc_run_serialmc(ch, ct.byref(rc), ct.byref(out)))
            res[i] = (s, b)
            lib.mcmc_chains_destroy(ch)
            lib.mcmc_model_destroy(mh)
            lib.mcmc_ctx_destroy(ctx)
        except Exception as e:                                   # surfaced in the main thread
            err.append(e)

    th = [threading.Thread(target=worker, args=(i, s)) for i, s in enumerate((1, 2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    for i in range(2):
        assert np.array_equal(res[i][0].view(np.uint64), alone[i]._samples.view(np.uint64))
        bits = np.unpackbits(res[i][1].view(np.uint8).reshape(len(r.r), -1), axis=1, bitorder="little")
        assert np.array_equal(bits.astype(bool).T, alone[i].diagnostics["accept"])
