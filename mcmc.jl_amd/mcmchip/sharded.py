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


def gather_shards(parts: dict, count: int, block: int, nchains: int, group=None, dst: int = 0,
                  chunk_bytes: int = DEFAULT_CHUNK_BYTES, stats: Optional[dict] = None):
    """Gather per-rank arrays whose LAST axis is the rank's chain block into host memory on `dst`.

    parts: name -> torch tensor [..., count] (accept bits: [..., ceil(count/64)] words), on the rank's GPU
    (NCCL) or on the host (gloo).  Rank r's columns are the global chains shard(nchains, world, r).  The
    transfer is point to point, rank by rank and chunk by chunk: a chunk is a run of whole leading rows
    (e.g. kept steps) of at most `chunk_bytes`, sent by its rank and received on `dst` into ONE reused
    buffer, then copied straight into the destination's host array.  So `dst` never holds more than one
    chunk of another rank's data on its device (the world's outputs are never concatenated on one GPU:
    at the 8-GPU metric they would be 193 GB).  Returns name -> numpy array over all `nchains` chains
    (bits: ceil(nchains/64) words) on dst, None elsewhere.  `stats` (a dict, dst only) receives
    `max_recv_buffer_bytes` and `bytes` (bytes received from other ranks)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if chunk_bytes <= 0:
        raise ValueError("chunk_bytes must be > 0")
    on_gpu = dist.get_backend(group) == "nccl"
    out = {} if rank == dst else None
    max_buf = 0
    moved = 0
    for name, t in parts.items():
        is_bits = name == "accept_bits"
        lead = tuple(t.shape[:-1])
        rows = 1
        for n in lead:
            rows *= n
        esize = t.element_size()
        keep = (nchains + 63) // 64 if is_bits else nchains
        host = None
        if rank == dst:
            host = _host_empty((rows, keep), t.dtype, on_gpu and torch.cuda.is_available())
        buf = None
        for r in range(world):
            off, cnt, _ = shard(nchains, world, r)
            if cnt <= 0:
                continue
            woff = off // 64 if is_bits else off
            width = (cnt + 63) // 64 if is_bits else cnt
            per = max(1, chunk_bytes // max(1, width * esize))
            if r == rank:
                mine = t.reshape(rows, t.shape[-1])[:, :width]
                if rank == dst:
                    host[:, woff:woff + width].copy_(mine)
                else:
                    for r0 in range(0, rows, per):
                        dist.send(mine[r0:r0 + per].contiguous(), dst=dist.get_global_rank(group, dst)
                                  if group is not None else dst, group=group)
            elif rank == dst:
                src = dist.get_global_rank(group, r) if group is not None else r
                for r0 in range(0, rows, per):
                    n = min(per, rows - r0)
                    need = n * width
                    if buf is None or buf.numel() < need:
                        buf = torch.empty(max(need, min(rows, per) * width), dtype=t.dtype, device=t.device)
                        max_buf = max(max_buf, buf.numel() * esize)
                    view = buf[:need].view(n, width)
                    dist.recv(view, src=src, group=group)
                    host[r0:r0 + n, woff:woff + width].copy_(view)
                    moved += need * esize
        buf = None
        if rank == dst:
            out[name] = host.numpy().reshape(lead + (keep,))
    if stats is not None and rank == dst:
        stats["max_recv_buffer_bytes"] = max_buf
        stats["bytes"] = moved
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
