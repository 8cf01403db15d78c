"""Sharded runs on the GPU: the union of per-rank shards equals a one-GPU run of all chains.

World size 1 over RCCL (the box has one GPU) and world size 2 over gloo with both ranks on cuda:0
(two processes, the gather goes through host copies): in both cases rank 0's assembled MCMCChain must
be bit-identical to mc.run of all chains, because the Philox stream is keyed by the global chain id.
"""
import os
import socket

import numpy as np
import pytest

import mcmchip as mc

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(kind):
    if kind == "iso":
        m = mc.model(mc.IsoNormalDot(), init=np.ones(5), grad=True)
        return m, mc.HMC(3, 0.2), mc.SerialMC(steps=12, burnin=2, thinning=2)
    rng = np.random.default_rng(4)
    X = np.hstack([np.ones((40, 1)), rng.normal(size=(40, 7))])
    Y = (rng.random(40) < 0.5).astype(float)
    m = mc.model(mc.LogisticRegression(X, Y), vars=np.zeros(8), gradient=True)
    return m, mc.MALA(0.01), mc.SerialMC(steps=10, burnin=2, thinning=3)


def _worker(rank, world, port, backend, kind, nchains, q):
    import torch
    import torch.distributed as dist
    from mcmchip.sharded import run_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, s, r = _setup(kind)
        ch = run_sharded(m, s, r, nchains, seed=21, device=0)
        if rank == 0:
            q.put({"samples": ch._samples, "grads": ch._gradients, "accept": ch.diagnostics["accept"],
                   "final_x": ch.final_x, "final_lp": ch.final_lp})
        else:
            q.put(ch)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(1, "nccl"), (2, "gloo")])
@pytest.mark.parametrize("kind", ["iso", "logistic"])
def test_sharded_equals_single_gpu(gpu, world, backend, kind):
    import torch.multiprocessing as tmp
    nchains = 150
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, kind, nchains, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = next(x for x in res if isinstance(x, dict))
    m, s, r = _setup(kind)
    ref = mc.run((m * s * r).batch(nchains, seed=21))
    assert np.array_equal(got["samples"], ref._samples)
    assert np.array_equal(got["accept"], ref.diagnostics["accept"])
    assert np.array_equal(got["final_x"], ref.final_x) and np.array_equal(got["final_lp"], ref.final_lp)
    if ref._gradients is not None:
        assert np.array_equal(got["grads"], ref._gradients)
