"""Task semantics at the drop-in boundary (GPU): arrays of tasks, prun, resume and MCMC.reset.

The reference's tasks draw from Julia's global RNG as they run, so every spun task samples a chain of its own
(MCMC.jl:87-98); run(t::Array{MCMCTask}) runs them in turn (runners.jl:17-33), prun maps run_serialmc_exit over
them (runners.jl:35-42, SerialMC.jl:87-91), run(c::MCMCChain) continues c.task (runners.jl:14), resume spins a fresh
task from model.init (SerialMC.jl:93-97), and MCMC.reset(t, x) moves a task's chain (MCMC.jl:39; the samplers'
:reset hooks).  Here like tasks run as ONE chain batch; every check is bitwise against the oracle at the global
chain ids the tasks drew.
"""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc
from test_gpu_parity import _glm_model, _model, _ram_model, assert_parity

pytestmark = pytest.mark.gpu


def _oracle_chain(m, sp, task, r):
    oc = orc.OracleChains(m, sp, nchains=task.nchains, seed=task.seed, chain_offset=task.chain_offset)
    return oc, oc.run(r)


def test_array_of_tasks_gives_independent_chains(gpu):
    """run(m * [RWM(0.1), RWM(0.1)] * r): two different chains, each bitwise the oracle's chain at its id, run as
    one batch (consecutive ids, one launch sequence)."""
    mc.srand(1)
    m = _model("iso", 3)
    r = mc.SerialMC(steps=200, burnin=20, thinning=3)
    ts = m * [mc.RWM(0.1), mc.RWM(0.1)] * r
    chs = mc.run(ts)
    assert len(chs) == 2 and chs[0].task is ts[0] and chs[1].task is ts[1]
    assert ts[0].seed == ts[1].seed == mc.drawn_key(1) and ts[1].chain_offset == ts[0].chain_offset + 1
    assert not np.array_equal(chs[0]._samples, chs[1]._samples)
    for t, ch in zip(ts, chs):
        _, (s, g, acc) = _oracle_chain(m, mc.RWM(0.1), t, r)
        assert_parity(ch, s, g, acc, "rwm")
        assert ch.samples.shape == (1, len(r.r), 3)


def test_respun_tasks_draw_new_streams(gpu):
    """run(m * s * r) twice: the second task's chain is not the first's (the global stream advanced)."""
    mc.srand(7)
    m = _model("iso", 3)
    r = mc.SerialMC(steps=50)
    a = mc.run(m * mc.RWM(0.3) * r)
    b = mc.run(m * mc.RWM(0.3) * r)
    assert (a.task.seed, a.task.chain_offset) == (mc.drawn_key(7), 0)
    assert (b.task.seed, b.task.chain_offset) == (mc.drawn_key(7), 1)
    assert not np.array_equal(a._samples, b._samples)
    mc.srand(7)
    c = mc.run(m * mc.RWM(0.3) * r)                     # srand restarts the stream
    assert np.array_equal(a._samples, c._samples)


def test_explicit_seed_and_drawn_streams_do_not_overlap(gpu):
    """MCMCTask(m, s, r, nchains=4) (seed 1, chain ids 0..3) and a later run(m * s * r) under srand(1) (the global
    stream's ids 0, 1, ...) sample different chains: drawn keys have their own key space."""
    mc.srand(1)
    m = _model("iso", 3)
    r = mc.SerialMC(steps=60)
    a = mc.run(mc.MCMCTask(m, mc.RWM(0.3), r, nchains=4))
    b = mc.run(m * mc.RWM(0.3) * r)
    assert (b.task.seed, b.task.chain_offset) == (mc.drawn_key(1), 0)
    assert not np.array_equal(a._samples[:, :, 0], b._samples[:, :, 0])
    c = mc.resume(a, steps=60)                           # a new task from model.init on the drawn stream
    assert not any(np.array_equal(c._samples[:, :, k], a._samples[:, :, k]) for k in range(4))
    _, (s, g, acc) = _oracle_chain(m, mc.RWM(0.3), b.task, r)
    assert_parity(b, s, g, acc, "rwm")


SAMPLERS = {
    "rwm": (lambda: _model("iso", 30), lambda: mc.RWM(0.6)),
    "mala_tuned": (lambda: _model("normal", 5), lambda: mc.MALA(2.0, mc.EmpMCTuner(0.6, adaptStep=7))),
    "hmc_tuned": (lambda: _model("iso", 7), lambda: mc.HMC(3, 0.9, mc.EmpMCTuner(0.7, adaptStep=5, maxStep=9))),
    "hmcda": (lambda: _model("iso", 40), lambda: mc.HMCDA(len=0.8)),
    "ram": (lambda: _ram_model("dist", 5), lambda: mc.RAM(0.7, 0.3)),
    "ram_wave": (lambda: _ram_model("iso", 48), lambda: mc.RAM(0.7, 0.3)),
    "glm_mala_tuned": (lambda: _glm_model("logistic", 20), lambda: mc.MALA(0.01, mc.EmpMCTuner(0.6, adaptStep=3))),
    "glm_hmcda": (lambda: _glm_model("linear", 200, n=40), lambda: mc.HMCDA(len=0.1)),
}


@pytest.mark.parametrize("sname", list(SAMPLERS))
def test_batched_chain_continues_chain_k(gpu, sname):
    """70 one-chain tasks run as one batch; continuing chains 67 and 3 (run(c) = run(c.task)) equals the oracle's
    continuation of those chains of the batch -- position, log-target, tuner state, HMCDA step and RAM factor all
    carried over -- in either order; the tasks not continued keep their batch state."""
    mm, ms = SAMPLERS[sname]
    m = mm()
    mc.srand(3)
    r = mc.SerialMC(steps=30, burnin=4, thinning=2)
    ts = m * [ms() for _ in range(70)] * r
    chs = mc.run(ts)
    off = ts[0].chain_offset
    assert [t.chain_offset for t in ts] == list(range(off, off + 70))
    oc = orc.OracleChains(m, ms(), nchains=70, seed=ts[0].seed, chain_offset=off)
    s1, g1, a1 = oc.run(r)
    kind = "rwm" if sname.startswith(("rwm", "ram")) else "grad"           # gradients compared unless rwm
    for k in (0, 41, 69):
        assert_parity(chs[k], s1[:, :, k:k + 1], None if g1 is None else g1[:, :, k:k + 1], a1[:, k:k + 1], kind)
    s2, g2, a2 = oc.run(r)
    for k in (67, 3):
        c2 = mc.run(chs[k])
        assert_parity(c2, s2[:, :, k:k + 1], None if g2 is None else g2[:, :, k:k + 1], a2[:, k:k + 1], kind)
        assert np.array_equal(c2.final_x[:, 0], oc.x[:, k]) and c2.final_lp[0] == oc.lp[k]
        assert ts[k].steps_done == 2 * r.len
    assert ts[5].steps_done == r.len and ts[5]._h is None                  # not forked until it runs
    if sname.startswith("ram"):
        S = ts[67].ram_factor()[0]
        S_ref = mc.api.unpack_ram_factor(oc.ram_L, m.size)[67]
        assert np.array_equal(S.view(np.uint64), S_ref.view(np.uint64))


def test_unlike_tasks_run_one_by_one(gpu):
    """m * [RWM(0.1), MALA(0.1)] * r: different samplers cannot share a batch; each task still draws its own chain
    and matches the oracle there."""
    mc.srand(11)
    m = _model("iso", 4)
    r = mc.SerialMC(steps=40)
    sps = [mc.RWM(0.1), mc.MALA(0.1)]
    ts = m * sps * r
    chs = mc.run(ts)
    assert ts[0].chain_offset != ts[1].chain_offset
    for t, ch, sp, kind in zip(ts, chs, sps, ("rwm", "mala")):
        _, (s, g, acc) = _oracle_chain(m, sp, t, r)
        assert_parity(ch, s, g, acc, kind)


def test_prun_runs_one_batch_and_stops(gpu):
    """prun(tasks): the same chains as run(tasks) would give, then stopped (run_serialmc_exit)."""
    m = _model("iso", 3)
    r = mc.SerialMC(steps=60, thinning=4)
    mc.srand(21)
    chs = mc.prun(m * [mc.HMC(3, 0.2) for _ in range(5)] * r)
    mc.srand(21)
    ref = mc.run(m * [mc.HMC(3, 0.2) for _ in range(5)] * r)
    for a, b in zip(chs, ref):
        assert np.array_equal(a._samples, b._samples) and np.array_equal(a.diagnostics["accept"],
                                                                        b.diagnostics["accept"])
    with pytest.raises(AssertionError, match="stopped"):
        mc.run(chs[0])


@pytest.mark.parametrize("case", ["iso_hmc", "normal_rwm", "glm_mala", "ram"])
def test_reset_moves_every_chain(gpu, case):
    """MCMC.reset(t, x): the chains jump to x with lp = eval(x) (and the gradient there); the next run continues
    from x with the step counter, tuners and RAM factor as they were -- bitwise the oracle doing the same."""
    if case == "iso_hmc":
        m, sp = _model("iso", 6), lambda: mc.HMC(4, 0.3)
    elif case == "normal_rwm":
        m, sp = _model("normal", 20), lambda: mc.RWM(0.6)
    elif case == "glm_mala":
        m, sp = _glm_model("logistic", 12), lambda: mc.MALA(0.01, mc.EmpMCTuner(0.6, adaptStep=3))
    else:
        m, sp = _ram_model("iso", 9), lambda: mc.RAM(0.7, 0.3)
    C = 70
    r = mc.SerialMC(steps=25, burnin=3, thinning=2)
    task = (m * sp() * r).batch(C, seed=5)
    mc.run(task)
    oc = orc.OracleChains(m, sp(), nchains=C, seed=5)
    oc.run(r)
    xs = np.random.default_rng(2).normal(size=(m.size, C)) * 0.3 + np.asarray(m.init)[:, None]
    lp = mc.reset(task, xs)
    lp_ref, _ = orc.eval_batch(m, xs, order=oc.order if oc.order != orc.ORDER_HALF else 1)
    assert np.array_equal(lp, lp_ref)
    oc.x[:] = xs
    oc.lp[:] = lp_ref
    ch = mc.run(task)
    s, g, acc = oc.run(r)
    kind = "rwm" if case in ("normal_rwm", "ram") else "mala" if case == "glm_mala" else "hmc"
    assert_parity(ch, s, g, acc, kind)
    assert task.steps_done == 2 * r.len
    one = mc.reset(task, np.asarray(m.init))                   # one point for every chain
    assert np.all(one == one[0])
