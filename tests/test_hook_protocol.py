"""The Julia hook's call pattern through the C ABI (GPU): a spun GPU task is a 1-chain batch that julia/mcmc_jl_hook.jl
runs in chunks with every step kept (SerialMC(steps=chunk): burnin 0, thinning 1), producing one MCMCSample per
consume; run_serialmc (SerialMC.jl:37-85) applies the task runner's kept range itself.  The samplers' adaptation reads
the task's own runner -- EmpiricalMALATune / EmpiricalHMCTune while i <= runner.burnin (MALA.jl:116, HMC.jl:167),
HMCDA's dual averaging while i < runner.burnin (HMCDA.jl:133-141) -- so the hook sets the task runner's burnin as the
tuners' burnin (mcmc_chains_set_tuner_burnin) apart from the chunks' kept range.  Here the hook's loop is driven
exactly so (chunk = min(1000, r.len) as the hook picks it, and shorter chunks that cut the burnin and the adaptation
windows) and the rows (burnin+1):len, the accept flags, the continuation run(c) and the adapted step sizes are checked
bit for bit against the oracle's SerialMC(steps=1000, burnin=100) of the same chain.
"""
import ctypes as ct

import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc
from mcmchip import _lib
from test_gpu_parity import _glm_model, _model

pytestmark = pytest.mark.gpu

CASES = {
    "mala_tuned": (lambda: _model("normal", 5), lambda: mc.MALA(2.0, mc.EmpMCTuner(0.6, adaptStep=7))),
    "hmc_tuned": (lambda: _model("iso", 7), lambda: mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9))),
    "hmcda": (lambda: _model("iso", 4), lambda: mc.HMCDA(len=0.8)),
    "logistic_mala_tuned": (lambda: _glm_model("logistic", 6), lambda: mc.MALA(0.05, mc.EmpMCTuner(0.6, adaptStep=9))),
    "logistic_hmcda": (lambda: _glm_model("logistic", 6), lambda: mc.HMCDA(len=0.3)),
}


def _hook_task(m, sp, chunk, seed, offset, tuner_burnin):
    """hip_chains + hip_ensure!: a 1-chain batch whose runs keep every step; the tuners' burnin set from the task's
    runner (None: not set, the chunk runner's burnin 0 applies -- the round-5 hook)"""
    t = mc.MCMCTask(m, sp, mc.SerialMC(steps=chunk), nchains=1, seed=seed, chain_offset=offset)
    if tuner_burnin is not None:
        _lib.check(_lib.load().mcmc_chains_set_tuner_burnin(t.handle(), tuner_burnin))
    return t


def _consume(t, nsteps):
    """hip_produce_loop: `nsteps` consumes, a new chunk whenever the buffer is empty (leftover steps stay buffered
    for the next call, as the Julia task keeps them).  Returns per-step ppars, pgrads, accept."""
    buf = getattr(t, "_hook_buf", None)
    xs, gs, acc = [], [], []
    for _ in range(nsteps):
        if buf is None or buf[3] >= buf[0].shape[0]:
            ch = mc.run(t)
            buf = [ch._samples[:, :, 0], None if ch._gradients is None else ch._gradients[:, :, 0],
                   ch.diagnostics["accept"][0], 0]
        j = buf[3]
        xs.append(buf[0][j])
        gs.append(None if buf[1] is None else buf[1][j])
        acc.append(bool(buf[2][j]))
        buf[3] += 1
    t._hook_buf = buf
    return np.array(xs), (None if gs[0] is None else np.array(gs)), np.array(acc)


@pytest.mark.parametrize("chunk", [1000, 250, 37])
@pytest.mark.parametrize("case", list(CASES))
def test_hook_chunked_task_matches_serialmc(gpu, case, chunk):
    mkm, mks = CASES[case]
    m, sp = mkm(), mks()
    r = mc.SerialMC(steps=1000, burnin=100)
    seed, off = 5, 3
    t = _hook_task(m, sp, min(chunk, r.len), seed, off, r.burnin)
    oc = orc.OracleChains(m, mks(), nchains=1, seed=seed, chain_offset=off)
    for rnd in range(2):                                  # run(t), then the continuation run(c) (runners.jl:14)
        xs, gs, acc = _consume(t, r.len)
        s, g, a = oc.run(r)
        kept = np.arange(r.burnin, r.len)                 # rows (burnin+1):len of the consumed steps
        assert np.array_equal(xs[kept].view(np.uint64), s[:, :, 0].view(np.uint64)), f"round {rnd}: samples"
        assert np.array_equal(gs[kept].view(np.uint64), g[:, :, 0].view(np.uint64)), f"round {rnd}: gradients"
        assert np.array_equal(acc[kept], a[:, 0].astype(bool)), f"round {rnd}: accept flags"
    st = t.tuner_state()
    want = oc.t_bar if sp.kind == 4 else oc.t_step
    got = st["step_bar"] if sp.kind == 4 else st["step"]
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))        # the adapted step, bitwise
    start = 1.0 if sp.kind == 4 else (sp.cfg().drift_step if sp.kind == 2 else sp.cfg().leap_step)
    assert got[0] != start                                                  # ... and it did adapt


@pytest.mark.parametrize("case", ["mala_tuned", "hmcda"])
def test_hook_without_tuner_burnin_does_not_adapt(gpu, case):
    """The round-5 hook (every chunk a burnin-0 run, no tuner burnin): the tuners never adapt, so the chain is not
    the reference's SerialMC(1000, 100) chain -- the defect the tuner burnin removes."""
    mkm, mks = CASES[case]
    m, sp = mkm(), mks()
    r = mc.SerialMC(steps=1000, burnin=100)
    t = _hook_task(m, sp, 1000, 5, 3, None)
    xs, _, _ = _consume(t, r.len)
    s, _, _ = orc.OracleChains(m, mks(), nchains=1, seed=5, chain_offset=3).run(r)
    assert not np.array_equal(xs[r.burnin:], s[:, :, 0])


def test_tuner_burnin_validation_and_fork(gpu):
    """-1 restores the runner's burnin; below -1 is refused; mcmc_chains_fork copies the setting."""
    lib = _lib.load()
    m = _model("normal", 5)
    sp = mc.MALA(2.0, mc.EmpMCTuner(0.6, adaptStep=7))
    t = mc.MCMCTask(m, sp, mc.SerialMC(steps=300), nchains=8, seed=2)
    h = t.handle()
    with pytest.raises(_lib.MCMCError, match="tuner burnin"):
        _lib.check(lib.mcmc_chains_set_tuner_burnin(h, -2))
    _lib.check(lib.mcmc_chains_set_tuner_burnin(h, 120))
    f = ct.c_void_p()
    _lib.check(lib.mcmc_chains_fork(h, 2, 3, ct.byref(f)))
    ft = mc.MCMCTask(m, sp, mc.SerialMC(steps=300), nchains=3, seed=2, chain_offset=2)
    ft._h = f                                             # the fork as a task of its own (MCMCTask owns the handle)
    ch = mc.run(ft)
    oc = orc.OracleChains(m, sp, nchains=3, seed=2, chain_offset=2)
    s, _, _ = oc.run(mc.SerialMC(steps=300, burnin=120))  # the fork adapts to 120 with every step kept
    assert np.array_equal(ch._samples[120:].view(np.uint64), s.view(np.uint64))
