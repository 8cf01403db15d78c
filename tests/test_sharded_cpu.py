"""Multi-process (gloo, world_size 2) tests of the chain sharding and the end-of-run gather.

The sharded run (mcmchip/sharded.py) steps each rank's block with the GPU kernels; these CPU tests
cover what is independent of the device: the block partition (global chain ids, 64-aligned so accept
bit words concatenate) and the gather/assembly of per-rank shards on the destination rank.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from conftest import PKG  # noqa: F401  (puts mcmc.jl_amd on sys.path)
from mcmchip.sharded import gather_shards, shard


def test_shard_partition_covers_all_chains():
    for total in (1, 63, 64, 65, 1000, 1 << 20, 524288):
        for world in (1, 2, 3, 4, 8):
            blocks = [shard(total, world, r) for r in range(world)]
            assert blocks[0][0] == 0
            for (o, c, b), (o2, c2, b2) in zip(blocks, blocks[1:]):
                assert b == b2 and b % 64 == 0
                if c2 > 0:
                    assert o + c == o2
            assert sum(c for _, c, _ in blocks) == total
            assert all(o % 64 == 0 for o, c, _ in blocks if c > 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_shard(off, cnt, nk, d):
    """Arrays a rank would produce for global chains off..off+cnt-1 (values encode the global id)."""
    c = np.arange(off, off + cnt)
    samples = (np.arange(nk)[:, None, None] * 1e6 + np.arange(d)[None, :, None] * 1e3 + c[None, None, :])
    acc = ((c[None, :] * 7 + np.arange(nk)[:, None]) % 3 == 0)
    words = np.zeros((nk, max(1, (cnt + 63) // 64)), dtype=np.uint64)
    for k in range(nk):
        for j in range(cnt):
            if acc[k, j]:
                words[k, j // 64] |= np.uint64(1) << np.uint64(j % 64)
    return samples, acc, words


def _worker(rank, world, port, total, nk, d, q, chunk=None, slots=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt, block = shard(total, world, rank)
        s, _, words = _fake_shard(off, cnt, nk, d)
        parts = {"samples": torch.from_numpy(s), "accept_bits": torch.from_numpy(words.view(np.int64)),
                 "final_lp": torch.from_numpy(s[-1, 0].copy())}
        stats = {}
        kw = {"slots": slots} if chunk is None else {"chunk_bytes": chunk, "slots": slots}
        full = gather_shards(parts, cnt, block, total, dst=0, stats=stats, **kw)
        if rank == 0:
            res = {k: v.copy() for k, v in full.items()}
            res["_stats"] = stats
            q.put(res)
        else:
            q.put(None if full is None else "unexpected")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,chunk", [(2, 130, None), (2, 1000, None), (2, 1000, 8 * 500 * 2), (2, 777, 64),
                                               (3, 1000, 8 * 300), (3, 5000, 8 * 1000), (4, 3000, 64)])
def test_gather_shards_gloo(world, total, chunk):
    """The chunked point-to-point gather reassembles every array exactly, whatever the chunk size (64 B: one
    row per message); every receive buffer holds at most one chunk (one row when a row is larger than the chunk),
    at most two per source rank, and with several source ranks their receives are in flight together, posted as one
    batch_isend_irecv group per round (the RCCL N > 1 path itself is unmeasured until the driver's 8-GPU run)."""
    nk, d = 3, 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, nk, d, q, chunk)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = next(r for r in res if isinstance(r, dict))
    assert sum(r is None for r in res) == world - 1
    s, acc, words = _fake_shard(0, total, nk, d)
    assert np.array_equal(full["samples"], s)
    assert np.array_equal(full["final_lp"], s[-1, 0])
    assert np.array_equal(full["accept_bits"].view(np.uint64), words)
    st = full["_stats"]
    cnts = [shard(total, world, r)[1] for r in range(1, world)]
    assert st["bytes"] == sum(8 * c * (nk * d + 1) + 8 * nk * ((c + 63) // 64) for c in cnts)
    one = max(8 * c for c in cnts)                         # the largest row of any array
    if chunk is not None:
        assert st["max_recv_buffer_bytes"] <= max(chunk, one)
        assert st["max_buffer_bytes_per_source"] <= 2 * max(chunk, one)
    if sum(c > 0 for c in cnts) >= 2:
        assert st["max_sources_in_flight"] >= 2             # receives from several ranks outstanding together
    assert st["GB_per_s"] > 0
    # one batch_isend_irecv (one RCCL group call) per round on dst, the round's receives from every source in it
    assert st["group_calls"] == st["rounds"] >= 1
    assert st["max_chunks_in_flight"] <= 2 * sum(c > 0 for c in cnts)
