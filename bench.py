#!/usr/bin/env python3
"""Throughput benchmark of the many-chain MCMC inner loop (BASELINE.json metric).

Workload (BASELINE.json "metric" config): d = 32 iso-Normal target -dot(v,v),
RWM(0.1), init ones(32), SerialMC(steps=1000, burnin=100, thinning=10), 2^20
chains per GPU, seed 1, fp64.  A "step" is one MCMC step of every chain
(one pass of the hot path over the chain batch).  The timed region runs
`--steps` steps through run_serialmc with kept samples, gradients and accept
bits written to HBM (device-resident outputs); chain state is resident in HBM
before the clock starts.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, weak scaling:
                                                      every rank runs 2^20 chains)
Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mcmc.jl_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# BASELINE.json configs (per-GPU chain counts for the sharded ones)
CONFIGS = {
    "metric": dict(d=32, chains=1 << 20, sampler="rwm", thinning=10,
                   desc="d=32 iso-Normal, RWM(0.1), 2^20 chains/GPU (BASELINE metric)"),
    "readme": dict(d=3, chains=1, sampler="rwm", thinning=1,
                   desc="config 1: d=3 iso-Normal, RWM(0.1), SerialMC(1000,100), 1 chain"),
    "d3": dict(d=3, chains=1 << 20, sampler="rwm", thinning=10,
               desc="config 2: d=3 iso-Normal, RWM(0.1), 1,048,576 chains"),
    "hmc1024": dict(d=1024, chains=524288 // 8, sampler="hmc", thinning=100,
                    desc="config 4: d=1024 iso-Normal, HMC(10, 0.1), 524,288 chains over 8 GPUs (65,536/GPU)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="metric", choices=list(CONFIGS),
                   help="BASELINE.json workload (metric = 2^20 chains x d=32 RWM)")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--d", type=int, default=None)
    p.add_argument("--chains", type=int, default=None, help="chains per GPU")
    p.add_argument("--sampler", default=None, choices=["rwm", "mala", "hmc", "hmcda"])
    p.add_argument("--thinning", type=int, default=None)
    p.add_argument("--spl", type=int, default=-1, help="steps per launch (0: whole run in one launch; "
                                                       "-1: default of the library)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--strong", action="store_true", help="fixed total chains (--chains) split over ranks")
    return p.parse_args()


def algorithmic_bytes(d, C, steps, burnin, thinning, spl, grad_sampler):
    """state round trip 16d + 16 B per chain per launch-step of state traffic,
    8d B per kept chain-step (+8d for gradients), 1 bit per kept chain-step."""
    nkept = len(range(burnin + 1, steps + 1, thinning))
    launches = 1 if spl == 0 else -(-steps // spl)
    state = launches * C * (16 * d + 16)
    kept = nkept * C * (8 * d * (2 if grad_sampler else 1)) + nkept * ((C + 63) // 64) * 8
    return state + kept, launches


def cpu_baseline(args, model, sampler, seconds):
    """The oracle (scalar C port of SerialMC + sampler, OpenMP over chains) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as orc
    import mcmchip as mc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    C = 4096
    steps = 50
    t0 = time.perf_counter()
    oc = orc.OracleChains(model, sampler, nchains=C, seed=1)
    oc.run(mc.SerialMC(steps=steps, burnin=5, thinning=10), nthreads=threads)
    dt = time.perf_counter() - t0
    rate = C * steps / dt
    steps2 = max(steps, int(rate * seconds / C))
    oc = orc.OracleChains(model, sampler, nchains=C, seed=1)
    t0 = time.perf_counter()
    oc.run(mc.SerialMC(steps=steps2, burnin=max(1, steps2 // 10), thinning=10), nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": C * steps2 / dt, "unit": "chain-steps/s", "cores": threads, "kind": "port",
            "sample": f"{C} chains x {steps2} steps of the same workload on the host ({dt:.1f} s), "
                      f"oracle/oracle.c OpenMP over chains; the GPU run's chain count scales it linearly"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch            # first: libmcmc_hip.so then binds to the HIP runtime torch already loaded
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import mcmchip as mc
    from mcmchip import _lib

    cfg0 = CONFIGS[args.config]
    for k in ("d", "chains", "sampler", "thinning"):
        if getattr(args, k) is None:
            setattr(args, k, cfg0[k])
    d = args.d
    C = max(1, args.chains // world) if args.strong else args.chains
    model = mc.model(mc.IsoNormalDot(), init=np.ones(d), grad=True)
    sampler = {"rwm": lambda: mc.RWM(0.1), "mala": lambda: mc.MALA(0.1), "hmc": lambda: mc.HMC(10, 0.1),
               "hmcda": lambda: mc.HMCDA()}[args.sampler]()
    K, W = args.steps, args.warmup
    burnin = K // 10
    runner = mc.SerialMC(steps=K, burnin=burnin, thinning=args.thinning)
    task = mc.MCMCTask(model, sampler, runner, nchains=C, seed=1, device=local, chain_offset=rank * C,
                       steps_per_launch=max(args.spl, 0))
    h = task.handle()
    lib = _lib.load()

    # device-resident outputs (caller-owned, as the C ABI's on_device mode)
    dev = torch.device("cuda", local)
    nkept = len(runner.r)
    samples = torch.empty((nkept, d, C), dtype=torch.float64, device=dev)
    grad_sampler = args.sampler != "rwm"
    grads = torch.empty((nkept, d, C), dtype=torch.float64, device=dev) if grad_sampler else None
    bits = torch.empty((nkept, (C + 63) // 64), dtype=torch.int64, device=dev)
    out = _lib.Outputs()
    out.samples = samples.data_ptr()
    out.gradients = grads.data_ptr() if grads is not None else None
    out.accept_bits = bits.data_ptr()
    out.on_device = 1

    if W > 0:
        wr = mc.SerialMC(steps=W, burnin=0, thinning=1)
        wout = _lib.Outputs()
        cfg = wr.cfg()
        _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(wout)))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    cfg = runner.cfg()
    t0 = time.perf_counter()
    _lib.check(lib.mcmc_run_serialmc(h, ct.byref(cfg), ct.byref(out)))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    T = time.perf_counter() - t0
    kernel_ms = out.kernel_ms
    if dist is not None:
        t = torch.tensor([T, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        T, kernel_ms = float(t[0]), float(t[1])
    total_chains = C * world
    value = total_chains * K / T

    spl = args.spl if args.spl >= 0 else 0
    nbytes, launches = algorithmic_bytes(d, C, K, burnin, args.thinning, spl, grad_sampler)
    avg_launch_s = kernel_ms * 1e-3 / launches
    achieved = nbytes / launches / avg_launch_s / 1e9
    line = {
        "metric": "MCMC steps*chains/sec (1M chains, d=32)",
        "value": value,
        "unit": "chain-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": T * 1e3 / K,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (model init ones(d); Philox4x32-10 stream, seed 1)",
        "config": {
            "workload": f"{args.config}: iso-Normal -dot(v,v) d={d}, {type(sampler).__name__}, "
                        f"SerialMC(steps={K}, burnin={burnin}, thinning={args.thinning}), {C} chains/GPU",
            "d": d, "chains_per_gpu": C, "global_chains": total_chains, "sampler": args.sampler,
            "burnin": burnin, "thinning": args.thinning, "kept_per_chain": nkept,
            "steps_per_launch": spl, "parallelism": f"chains sharded over {world} GPU(s), no collective in loop",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": f"{'lpc' if d <= 32 else 'wpc'}_{args.sampler}", "launches": launches, "avg_launch_ms": avg_launch_s * 1e3,
            "algorithmic_bytes_per_launch": nbytes / launches,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, model, sampler, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
