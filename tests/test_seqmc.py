"""SeqMC population runner (src/runners/SeqMC.jl): oracle behaviour on CPU, HIP parity on the GPU.

The README's SeqMC example (README.md:240-266): 10 tempered targets y = abs(x); y ~ Normal(1, s_i),
s_i = logspace(1, -1, 10), RWM(s_i) each, SeqMC(steps=10, burnin=0), 1000 particles; the weighted
particles approximate |x| ~ Normal(1, 0.1), i.e. x near +-1.
"""
import numpy as np
import pytest

import mcmchip as mc
import oracle_ref as orc
from mcmchip.seqmc import target_seed


def _readme_targets(nmod=10, steps=10, burnin=0, trigger=1e-10):
    sts = np.logspace(1, -1, nmod)
    mods = [mc.model(mc.AbsNormalDSL(1.0, s), x=0.0) for s in sts]
    return [mods[i] * mc.RWM(sts[i]) * mc.SeqMC(steps=steps, burnin=burnin, trigger=trigger) for i in range(nmod)]


def _oracle(targets, particles, seed):
    r = targets[-1].runner
    return orc.seqmc([(t.model, t.sampler) for t in targets], particles, r.steps, r.burnin, r.trigger, seed,
                     [target_seed(seed, k) for k in range(len(targets))])


def test_seqmc_validation_messages():
    with pytest.raises(AssertionError, match="Burnin rounds"):
        mc.SeqMC(steps=3, burnin=-1)
    with pytest.raises(AssertionError, match="should be > to burnin"):
        mc.SeqMC(steps=3, burnin=3)


def test_oracle_seqmc_readme_example_statistics():
    """Weighted resampling of the final particles concentrates on |x| ~ 1 (README.md:258-266)."""
    targets = _readme_targets()
    rng = np.random.default_rng(0)
    particles = rng.standard_normal((1000, 1))
    s, w, flags = _oracle(targets, particles, seed=3)
    x = s[-1, 0]
    ww = w[-1] / w[-1].sum()
    draws = rng.choice(x, size=4000, p=ww)                 # wsample(samples, weigths, n)
    assert abs(np.mean(np.abs(draws)) - 1.0) < 0.1
    assert np.all(np.isfinite(s))


def test_oracle_seqmc_resampling_triggers():
    """A huge trigger resamples after every target; weights reset to exp(0) = 1."""
    targets = _readme_targets(nmod=3, steps=4, trigger=1e300)
    particles = np.random.default_rng(1).standard_normal((200, 1))
    s, w, flags = _oracle(targets, particles, seed=5)
    assert flags.all()
    assert np.array_equal(w, np.ones_like(w))


@pytest.mark.gpu
@pytest.mark.parametrize("trigger", [1e-10, 1e300, 0.05])
@pytest.mark.parametrize("npart", [7, 1000, 3000])
def test_seqmc_matches_oracle(gpu, trigger, npart):
    targets = _readme_targets(nmod=4, steps=6, burnin=2, trigger=trigger)
    particles = np.random.default_rng(npart).standard_normal((npart, 1))
    ch = mc.run(targets, particles=particles, seed=11)
    s, w, flags = _oracle(targets, particles, seed=11)
    assert np.array_equal(ch.diagnostics["resampled"], flags.astype(bool))
    assert np.array_equal(ch._samples, s)
    assert np.array_equal(ch.diagnostics["weigths"], w.reshape(-1))
    assert ch.samples.shape == (4 * npart, 1)


@pytest.mark.gpu
def test_seqmc_multidim_mala_targets(gpu):
    """d = 5 NormalDSL targets with MALA and HMC mutations (gradient samplers inside SeqMC)."""
    mods = [mc.model(mc.NormalDSL(0.5 * k, 1.0 + k), v=np.zeros(5), gradient=True) for k in range(3)]
    targets = [mods[0] * mc.MALA(0.3) * mc.SeqMC(steps=4), mods[1] * mc.HMC(2, 0.2) * mc.SeqMC(steps=4),
               mods[2] * mc.RWM(0.5) * mc.SeqMC(steps=4, trigger=0.5)]
    particles = np.random.default_rng(2).standard_normal((333, 5))
    ch = mc.run(targets, particles=particles, seed=4)
    s, w, flags = _oracle(targets, particles, seed=4)
    assert np.array_equal(ch._samples, s) and np.array_equal(ch.diagnostics["weigths"], w.reshape(-1))
