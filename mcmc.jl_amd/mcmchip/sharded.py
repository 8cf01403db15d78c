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


def gather_shards(parts: dict, count: int, block: int, nchains: int, group=None, dst: int = 0):
    """Gather per-rank arrays whose LAST axis is the rank's chain block onto `dst`.

    parts: name -> torch tensor [..., count] (accept bits: [..., ceil(count/64)] words).  Every rank pads its
    block to `block` chains, one torch.distributed.gather per array; on dst returns name -> numpy array over
    all `nchains` chains (bits: ceil(nchains/64) words), elsewhere None."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    out = {} if rank == dst else None
    for name, t in parts.items():
        is_bits = name == "accept_bits"
        width = (block // 64) if is_bits else block
        have = t.shape[-1]
        padded = torch.zeros(t.shape[:-1] + (width,), dtype=t.dtype, device=t.device)
        padded[..., :have] = t
        bucket = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
        dist.gather(padded, bucket, dst=dst, group=group)
        if rank == dst:
            full = torch.cat(bucket, dim=-1)
            keep = (nchains + 63) // 64 if is_bits else nchains
            out[name] = full[..., :keep].cpu().numpy()
    return out


def run_sharded(model, sampler, runner: SerialMC, nchains: int, seed: int = 1, group=None, dst: int = 0,
                device: Optional[int] = None) -> Optional[MCMCChain]:
    """run(model * sampler * runner) over `nchains` chains split across the ranks of `group`.

    Call on every rank (torch.distributed initialised; one GPU per rank: `device` defaults to the rank's
    LOCAL_RANK).  Returns the assembled MCMCChain on `dst`, None elsewhere.  chain.runTime is the step loop's
    wall time (max over ranks); chain.gather_s the end-of-run gather."""
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
    full = gather_shards(parts, cnt, block, nchains, group=group, dst=dst)
    gather_s = time.perf_counter() - t0
    if rank != dst:
        return None
    bits = full["accept_bits"].view(np.uint64)
    diags = {"step": list(runner.r), "accept": _unpack_bits(bits, nchains)}
    whole = MCMCTask(model, sampler, runner, nchains=nchains, seed=seed, device=device)
    ch = MCMCChain(runner.r, full["samples"], full.get("gradients"), diags, whole, float(rt[0]),
                   final_x=full["final_x"], final_lp=full["final_lp"])
    ch.gather_s = gather_s
    return ch
