"""Chains sharded across GPUs: one process per GPU, one gather at the end.

The reference runs independent chains independently (runners.jl:21-26; `prun`
maps tasks to processes, runners.jl:40).  Here a run of `nchains` chains is
split into contiguous blocks, one per rank of a torch.distributed group (one
process per GPU, backend "nccl" = RCCL over xGMI).  Each rank steps its block
with the same kernels as a single-GPU run; the Philox stream is keyed by the
*global* chain id (chain_offset), so the union of the shards is bit-identical
to a one-GPU run of all chains.  Nothing crosses GPUs inside the step loop.
After the loop, one gather collects samples, gradients, accept bits and the
final state on the destination rank, which assembles the MCMCChain.

Shard blocks are multiples of 64 chains so that the packed accept-bit words of
each shard are exactly a slice of the global bit array (bit c%64 of word c/64).
"""
from __future__ import annotations

import ctypes as ct
import time
from typing import Optional

import numpy as np

from . import _lib
from .api import MCMCChain, MCMCTask, SerialMC, _unpack_bits

__all__ = ["shard", "gather_shards", "run_sharded"]



def shard(nchains: int, world: int, rank: int, align: int = 64):
    """(offset, count, block) of `rank`'s contiguous chain block; block = per-rank capacity (align multiple)."""
    if nchains <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("need nchains > 0 and 0 <= rank < world")
    per = -(-nchains // world)
    block = -(-per // align) * align
    off = min(rank * block, nchains)
    return off, min(block, nchains - off), block


DEFAULT_CHUNK_BYTES = 256 << 20


def _host_empty(shape, dtype, pin):
    """Destination host array (numpy view of a torch tensor, page-locked when the transfers come from a GPU)."""
    import torch
    if pin:
        try:
            return torch.empty(shape, dtype=dtype, pin_memory=True)
        except RuntimeError:            # page-locking refused (size, limits): pageable memory still works
            pass
    return torch.empty(shape, dtype=dtype)


class _Plan:
    """The chunks of one array that one source rank sends to dst: (row0, nrows) runs of whole leading rows."""

    def __init__(self, name, rows, width, woff, per):
        self.name, self.rows, self.width, self.woff = name, rows, width, woff
        self.chunks = [(r0, min(per, rows - r0)) for r0 in range(0, rows, per)]


def gather_shards(parts: dict, count: int, block: int, nchains: int, group=None, dst: int = 0,
                  chunk_bytes: int = DEFAULT_CHUNK_BYTES, stats: Optional[dict] = None, slots: int = 2):
    """Gather per-rank arrays whose LAST axis is the rank's chain block into host memory on `dst`.

    parts: name -> torch tensor [..., count] (accept bits: [..., ceil(count/64)] words), on the rank's GPU
    (NCCL) or on the host (gloo).  Rank r's columns are the global chains shard(nchains, world, r).  The
    transfer is point to point in chunks (runs of whole leading rows, e.g. kept steps, of at most `chunk_bytes`)
    and concurrent across sources, in rounds: round k moves chunk k of every source that has one, and its receives
    on dst (one per source) are posted together as ONE dist.batch_isend_irecv -- one NCCL group call on the process
    group's communicator, so no two p2p communicators of one device ever have operations outstanding at once; each
    source posts its send of round k the same way.  `slots` rounds are in flight at a time, each into its own buffer
    per source; as a round lands its chunks go on to host memory (NCCL: an asynchronous device -> page-locked host
    copy on a side stream, so the next round's receives overlap it) and are then placed into the destination
    arrays.  So `dst` holds at most `slots` chunks per source on its device (the world's outputs are never
    concatenated on one GPU: at the 8-GPU metric they would be 193 GB).  Returns name -> numpy array over all
    `nchains` chains (bits: ceil(nchains/64) words) on dst, None elsewhere.  `stats` (a dict, dst only) receives
    `bytes` (received from other ranks), `max_recv_buffer_bytes` (the largest one buffer),
    `max_buffer_bytes_per_source`, `max_sources_in_flight` (source ranks with a receive outstanding at one time),
    `max_chunks_in_flight`, `rounds` and `group_calls` (batch_isend_irecv calls on dst)."""
    import collections
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if chunk_bytes <= 0:
        raise ValueError("chunk_bytes must be > 0")
    if slots < 1:
        raise ValueError("slots must be >= 1")
    on_gpu = dist.get_backend(group) == "nccl"
    glob = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    names = list(parts)
    # per array: its host destination (dst) and each rank's plan
    lead = {n: tuple(parts[n].shape[:-1]) for n in names}
    rowsof = {n: int(np.prod(lead[n], dtype=np.int64)) if lead[n] else 1 for n in names}
    plans = {}                                            # source rank -> [_Plan] in send order
    for r in range(world):
        off, cnt, _ = shard(nchains, world, r)
        plans[r] = []
        if cnt <= 0:
            continue
        for n in names:
            is_bits = n == "accept_bits"
            width = (cnt + 63) // 64 if is_bits else cnt
            per = max(1, chunk_bytes // max(1, width * parts[n].element_size()))
            plans[r].append(_Plan(n, rowsof[n], width, off // 64 if is_bits else off, per))
    if rank != dst:
        # the source: chunk k is its send of round k, one batch_isend_irecv each, at most `slots` rounds outstanding
        pending = collections.deque()
        for pl in plans[rank]:
            mine = parts[pl.name].reshape(pl.rows, parts[pl.name].shape[-1])[:, :pl.width]
            for r0, n in pl.chunks:
                while len(pending) >= slots:
                    for w in pending.popleft()[0]:
                        w.wait()
                t = mine[r0:r0 + n].contiguous()
                pending.append((dist.batch_isend_irecv([dist.P2POp(dist.isend, t, glob(dst), group)]), t))
        while pending:
            for w in pending.popleft()[0]:
                w.wait()
        return None
    # dst: host arrays, its own columns copied directly
    host = {}
    for n in names:
        is_bits = n == "accept_bits"
        keep = (nchains + 63) // 64 if is_bits else nchains
        host[n] = _host_empty((rowsof[n], keep), parts[n].dtype, False).numpy()
    for pl in plans[dst]:
        mine = parts[pl.name].reshape(pl.rows, parts[pl.name].shape[-1])[:, :pl.width]
        host[pl.name][:, pl.woff:pl.woff + pl.width] = mine.cpu().numpy()
    chunks = {r: [(pl, r0, n) for pl in plans[r] for r0, n in pl.chunks] for r in range(world) if r != dst and plans[r]}
    rounds = max((len(v) for v in chunks.values()), default=0)
    dev = next(iter(parts.values())).device
    esz = {n: parts[n].element_size() for n in names}
    dtype = {n: parts[n].dtype for n in names}
    side = torch.cuda.Stream(device=dev) if on_gpu else None
    bufs = {}                                             # (source, slot) -> device (or host) buffer, reused
    stage = {}                                            # (source, slot) -> page-locked host staging (NCCL)
    inflight = collections.deque()                        # (round, [(source, slot, plan, row0, nrows, view)], works)
    copying = collections.deque()                         # (round, source, slot, plan, row0, nrows, event)
    max_buf = max_src_buf = moved = 0
    max_src = max_chunks = calls = 0
    src_buf_bytes = collections.Counter()

    def buffer(key, pl, n):
        need = n * pl.width * esz[pl.name]
        b = bufs.get(key)
        if b is None or b.numel() * b.element_size() < need:
            nonlocal max_buf, max_src_buf
            old = 0 if b is None else b.numel() * b.element_size()
            b = torch.empty(need, dtype=torch.uint8, device=dev)
            bufs[key] = b
            src_buf_bytes[key[0]] += need - old
            max_buf = max(max_buf, need)
            max_src_buf = max(max_src_buf, src_buf_bytes[key[0]])
            if on_gpu:
                stage[key] = _host_empty((need,), torch.uint8, True)
        return b[:need].view(dtype[pl.name]).view(n, pl.width)

    def place(pl, r0, n, arr):
        host[pl.name][r0:r0 + n, pl.woff:pl.woff + pl.width] = arr

    def finish_copies(upto):
        # copies of rounds <= upto to their place (their staging buffers are reused by round upto + slots)
        while copying and copying[0][0] <= upto:
            _, r, k, pl, r0, n, ev = copying.popleft()
            ev.synchronize()
            st = stage[(r, k)][:n * pl.width * esz[pl.name]].view(dtype[pl.name]).view(n, pl.width)
            place(pl, r0, n, st.numpy())

    def complete(rnd, entries, works):
        nonlocal moved
        for w in works:
            w.wait()
        finish_copies(rnd - slots)
        if on_gpu:
            side.wait_stream(torch.cuda.current_stream(dev))
        for r, k, pl, r0, n, view in entries:
            moved += n * pl.width * esz[pl.name]
            if on_gpu:
                with torch.cuda.stream(side):
                    st = stage[(r, k)][:n * pl.width * esz[pl.name]].view(dtype[pl.name]).view(n, pl.width)
                    st.copy_(view, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                # the next receive into this buffer runs on the NCCL stream after the current stream: make the
                # current stream wait for the copy out of it
                torch.cuda.current_stream(dev).wait_event(ev)
                copying.append((rnd, r, k, pl, r0, n, ev))
            else:
                place(pl, r0, n, view.numpy())

    t0 = time.perf_counter()
    for k in range(rounds):
        slot = k % slots
        while inflight and inflight[0][0] <= k - slots:        # slot's previous round landed before its reuse
            complete(*inflight.popleft())
        ops, entries = [], []
        for r, lst in chunks.items():
            if k < len(lst):
                pl, r0, n = lst[k]
                view = buffer((r, slot), pl, n)
                ops.append(dist.P2POp(dist.irecv, view, glob(r), group))
                entries.append((r, slot, pl, r0, n, view))
        inflight.append((k, entries, dist.batch_isend_irecv(ops)))
        calls += 1
        max_chunks = max(max_chunks, sum(len(e) for _, e, _ in inflight))
        max_src = max(max_src, len({e[0] for _, es, _ in inflight for e in es}))
    while inflight:
        complete(*inflight.popleft())
    finish_copies(rounds)
    out = {n: host[n].reshape(lead[n] + (host[n].shape[1],)) for n in names}
    if stats is not None:
        sec = time.perf_counter() - t0
        stats.update(bytes=moved, max_recv_buffer_bytes=max_buf, max_buffer_bytes_per_source=max_src_buf,
                     max_sources_in_flight=max_src, max_chunks_in_flight=max_chunks, slots=slots, seconds=sec,
                     rounds=rounds, group_calls=calls, GB_per_s=moved / sec / 1e9 if sec > 0 else None)
    return out


def run_sharded(model, sampler, runner: SerialMC, nchains: int, seed: int = 1, group=None, dst: int = 0,
                device: Optional[int] = None, chunk_bytes: int = DEFAULT_CHUNK_BYTES) -> Optional[MCMCChain]:
    """run(model * sampler * runner) over `nchains` chains split across the ranks of `group`.

    Call on every rank (torch.distributed initialised; one GPU per rank: `device` defaults to the rank's
    LOCAL_RANK).  Returns the assembled MCMCChain on `dst`, None elsewhere.  chain.runTime is the step loop's
    wall time (max over ranks); chain.gather_s the end-of-run gather (chunked point to point into host memory
    on `dst`, gather_shards), chain.gather_stats its bytes and largest receive buffer."""
    import os
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    off, cnt, block = shard(nchains, world, rank)
    d = model.size
    nk = len(runner.r)
    dev = torch.device("cuda", device)
    grad = sampler.uses_gradient
    parts = {
        "samples": torch.empty((nk, d, max(cnt, 1)), dtype=torch.float64, device=dev),
        "gradients": torch.empty((nk, d, max(cnt, 1)), dtype=torch.float64, device=dev) if grad else None,
        "accept_bits": torch.zeros((nk, max(1, (cnt + 63) // 64)), dtype=torch.int64, device=dev),
        "final_x": torch.empty((d, max(cnt, 1)), dtype=torch.float64, device=dev),
        "final_lp": torch.empty((max(cnt, 1),), dtype=torch.float64, device=dev),
    }
    runtime = 0.0
    task = None
    if cnt > 0:
        task = MCMCTask(model, sampler, runner, nchains=cnt, seed=seed, device=device, chain_offset=off)
        out = _lib.Outputs()
        for name in ("samples", "gradients", "accept_bits", "final_x", "final_lp"):
            t = parts[name]
            setattr(out, name, t.data_ptr() if t is not None else None)
        out.on_device = 1
        cfg = runner.cfg()
        _lib.check(_lib.load().mcmc_run_serialmc(task.handle(), ct.byref(cfg), ct.byref(out)))
        runtime = out.runtime_s
    parts = {k: (v[..., :cnt] if k != "accept_bits" else v) for k, v in parts.items() if v is not None}
    # the collective runs on the backend's device: NCCL on the GPU tensors, gloo on host copies
    if dist.get_backend(group) != "nccl":
        parts = {k: v.cpu() for k, v in parts.items()}
    rt = torch.tensor([runtime], dtype=torch.float64, device=dev if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(rt, op=dist.ReduceOp.MAX, group=group)
    t0 = time.perf_counter()
    gstats = {}
    full = gather_shards(parts, cnt, block, nchains, group=group, dst=dst, chunk_bytes=chunk_bytes, stats=gstats)
    gather_s = time.perf_counter() - t0
    if rank != dst:
        return None
    bits = full["accept_bits"].view(np.uint64)
    diags = {"step": list(runner.r), "accept": _unpack_bits(bits, nchains)}
    whole = MCMCTask(model, sampler, runner, nchains=nchains, seed=seed, device=device)
    ch = MCMCChain(runner.r, full["samples"], full.get("gradients"), diags, whole, float(rt[0]),
                   final_x=full["final_x"], final_lp=full["final_lp"])
    ch.gather_s = gather_s
    ch.gather_stats = gstats
    return ch
