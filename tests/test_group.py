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
    # RAM (RAM.jl:41-79): per-block jump factors, assembled by MCMCTask.ram_factor from every block's
    # mcmc_chains_ram_factor -- wave per chain (d = 70) and the regression layout (d = 10)
    "ram70": lambda: (mc.model(mc.IsoNormalDot(), init=np.ones(70), grad=True), mc.RAM(1.0, 0.234),
                      mc.SerialMC(steps=30, burnin=5, thinning=5), 150),
    "ram_linear10": lambda: (_linear10(), mc.RAM(1.0, 0.3), mc.SerialMC(steps=25, burnin=5, thinning=4), 200),
}


def _linear10(n=60):
    rng = np.random.default_rng(6)
    X = np.hstack([np.ones((n, 1)), rng.normal(size=(n, 9))])
    Y = X @ rng.normal(size=10) + rng.normal(size=n)
    return mc.model(mc.LinearRegression(X, Y), vars=np.zeros(10), gradient=True)


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
    if isinstance(s, mc.RAM):
        assert np.array_equal(task.ram_factor().view(np.uint64), one.task.ram_factor().view(np.uint64))
    # continue (run(chain), runners.jl:14) and resume (SerialMC.jl:93-97) on the group
    _same(mc.run(grp), mc.run(one))
    _same(mc.resume(grp, steps=7, seed=11, chain_offset=4096), mc.resume(one, steps=7, seed=11, chain_offset=4096))
    a = mc.resume(grp, steps=7)                                      # chains drawn from the global stream
    _same(a, mc.resume(one, steps=7, seed=a.task.seed, chain_offset=a.task.chain_offset))
    assert mc.resume(one, steps=7).task.chain_offset != a.task.chain_offset


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


@pytest.mark.gpu
def test_group_failed_block_blocks_further_runs(gpu):
    """A run in which one block fails leaves the blocks at different steps: the error names the block, and the
    chains refuse further runs (and steps_done) until reset; after mcmc_group_chains_reset (resume) the group is
    again bit-identical to one context."""
    lib = _lib.load()
    m, s, r, C = CASES["hmc3"]()
    task = (m * s * r).batch(C, seed=11, devices=(0, 0, 0))
    mc.run(task)
    _lib.check(lib.mcmc_debug_group_inject_failure(task.handle(), 1))
    with pytest.raises(_lib.MCMCError, match="block 1"):
        mc.run(task)
    with pytest.raises(_lib.MCMCError, match="different steps"):
        task.steps_done
    with pytest.raises(_lib.MCMCError, match="failed"):
        mc.run(task)
    task.reset()
    assert task.steps_done == 0
    _same(mc.run(task), mc.run((m * s * r).batch(C, seed=11)))


@pytest.mark.gpu
def test_group_gather_rate_at_metric_size(gpu):
    """The end gather at 2^20 chains (d = 32, 20 kept rows: 5.4 GB of samples into one host buffer), two blocks:
    the caller's pageable buffers are page-locked for the run (hipHostRegister), so each block's strided copy
    is direct DMA.  Prints the measured gather time and rate; DESIGN.md §8 quotes it."""
    import json
    import time
    C, d = 1 << 20, 32
    m = mc.model(mc.IsoNormalDot(), init=np.ones(d))
    r = mc.SerialMC(steps=20, burnin=0, thinning=1)
    task = (m * mc.RWM(0.1) * r).batch(C, seed=1, devices=(0, 0))
    h = task.handle()
    lib = _lib.load()
    nk = len(r.r)
    samples = np.empty((nk, d, C))
    bits = np.empty((nk, C // 64), dtype=np.uint64)
    samples[:, :, ::4096] = 0.0                                  # touch nothing else: registration faults pages in
    out = _lib.Outputs()
    out.samples, out.accept_bits = samples.ctypes.data, bits.ctypes.data
    cfg = r.cfg()
    gs = ct.c_double(0.0)
    t0 = time.perf_counter()
    _lib.check(lib.mcmc_group_run_serialmc(h, ct.byref(cfg), ct.byref(out), ct.byref(gs)))
    wall = time.perf_counter() - t0
    nbytes = samples.nbytes + bits.nbytes
    pin = ct.c_double(-1.0)
    _lib.check(lib.mcmc_group_last_pin_s(h, ct.byref(pin)))
    assert pin.value >= 0.0
    line = {"test": "group_gather", "chains": C, "d": d, "kept": nk, "blocks": 2, "bytes": nbytes,
            "gather_s": gs.value, "gather_GBps": nbytes / gs.value / 1e9, "pin_s": pin.value,
            "gather_with_pin_GBps": nbytes / (gs.value + pin.value) / 1e9, "step_loop_s": out.runtime_s,
            "call_wall_s": wall}
    print(json.dumps(line))
    assert np.isfinite(samples[-1]).all() and samples[-1, :, ::65536].std() > 0
    assert nbytes / gs.value > 5e9, line                         # direct DMA, not staged pageable copies
