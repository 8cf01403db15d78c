"""Golden chain fixtures (tests/golden/chains_*.npz, made by tests/golden/gen_golden.py).

CPU: the oracle still reproduces every committed fixture bit for bit (a change to the oracle's
arithmetic or RNG consumption shows up here).  GPU: the HIP path, through the C ABI, reproduces the
same fixtures bit for bit -- samples, kept gradients, accept flags and the evaluation count -- without
running the oracle.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import gen_golden as gg  # noqa: E402
import mcmchip as mc  # noqa: E402

IDS = [c[0] for c in gg.CASES]
CASES = {c[0]: c for c in gg.CASES}


def _fixture(name):
    with np.load(gg.fixture_path(name)) as f:
        return {k: f[k] for k in f.files}


def test_every_case_has_a_fixture():
    missing = [n for n in IDS if not os.path.exists(gg.fixture_path(n))]
    assert not missing, f"run tests/golden/gen_golden.py: missing {missing}"


@pytest.mark.parametrize("name", IDS)
def test_oracle_reproduces_fixture(name):
    _, spec, sname, runner, C, seed = CASES[name]
    fx = _fixture(name)
    s, g, acc, ev = gg.oracle_run(spec, sname, runner, C, seed)
    assert np.array_equal(s.view(np.uint64), fx["samples"].view(np.uint64))
    assert np.array_equal(acc, fx["accept"])
    assert np.array_equal(ev, fx["evals"])
    if "gradients" in fx:
        assert np.array_equal(g.view(np.uint64), fx["gradients"].view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("name", IDS)
def test_hip_reproduces_fixture(gpu, name):
    _, spec, sname, runner, C, seed = CASES[name]
    fx = _fixture(name)
    m = gg.make_model(spec)
    r = mc.SerialMC(steps=runner[0], burnin=runner[1], thinning=runner[2])
    chain = mc.run((m * gg.case_sampler(spec, sname) * r).batch(C, seed=seed))
    s = chain._samples
    acc = chain.diagnostics["accept"].T
    assert np.array_equal(acc, fx["accept"].astype(bool)), f"accept flags differ in {np.count_nonzero(acc != fx['accept'])}"
    np.testing.assert_allclose(s, fx["samples"], rtol=1e-10, atol=0)            # north_star tolerance
    assert np.array_equal(s.view(np.uint64), fx["samples"].view(np.uint64)), "samples not bit-identical"
    if "gradients" in fx and sname not in ("rwm", "ram"):
        assert np.array_equal(chain._gradients.view(np.uint64), fx["gradients"].view(np.uint64))
    assert chain.task.evals == int(fx["evals"].sum())
