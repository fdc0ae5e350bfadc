"""bench.py -- walker log-prob throughput of the MI355X RV engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

A "step" is one pass of the hot path over one batch: the per-walker
log-likelihood of a W-walker ensemble (config 2: 1 planet x 256 epochs x
4096 walkers per GPU, fp64) with theta already resident in HBM, i.e. one
rvk_loglike_device launch.  With N > 1 each rank evaluates its own 4096-walker
shard (weak scaling) and the per-walker log-probs are all-gathered over RCCL
(the exchange back to the stretch move); all-gathers are
pipelined one step behind the kernels on RCCL's stream.

Rank 0 prints ONE JSON line (metric/value = Kepler solves/s over all GPUs,
plus the roofline of the dominant kernel measured live with HIP events and a
bounded CPU baseline of the C oracle on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VALU_PEAK = 256 * 4 * 16 * 2.4e9   # lane-ops/s: 256 CU x 4 SIMD x 16 fp64 lanes/clk x 2.4 GHz
BYTES_PER_WALKER_EPOCH = 28    # t, v, sigma fp64 + int32 inst


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--walkers", type=int, default=None, help="walkers per GPU (default: config's, 4096 for cfg 2)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(ds, theta, budget_s):
    """Time the C oracle (oracle/rv_oracle.c, OpenMP over walkers) on a bounded sample."""
    from oracle import oracle
    threads = min(16, os.cpu_count() or 1)
    n_ep, n_pl = len(ds.time), len(ds.planet_letters)
    sample = theta[: min(len(theta), 4096)]
    oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                   ds.parameterisation.code, ds.t0, sample[:64], nthreads=threads)   # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        _, used = oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                                 ds.parameterisation.code, ds.t0, sample, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    solves = reps * len(sample) * n_ep * n_pl
    # single-core scalar leg (emcee's serial map), ~1/4 of the budget
    one = sample[:256]
    r1, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < budget_s / 4:
        oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                       ds.parameterisation.code, ds.t0, one, nthreads=1)
        r1 += 1
    el1 = time.perf_counter() - t1
    return {"value": solves / el, "unit": "Kepler solves/s", "cores": used, "kind": "port",
            "sample": f"{reps} x {len(sample)} walkers x {n_ep} epochs x {n_pl} planet(s) of the same "
                      f"config-{ds.cfg} ensemble, C oracle (oracle/rv_oracle.c, fp64, OpenMP), {el:.1f} s",
            "single_core_value": r1 * len(one) * n_ep * n_pl / el1}


def load_pmc(cfg):
    p = os.path.join(ROOT, "profiles", f"pmc_config{cfg}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import CONFIGS, make_dataset, make_walkers
    c = CONFIGS[args.config]
    W = args.walkers or (c["n_walkers"] if args.config != 4 else c["n_walkers"] // 8)
    ds = make_dataset(c["n_planets"], c["n_epochs"], c["n_inst"], seed=c["seed"])
    ds.cfg = args.config
    theta_all = make_walkers(ds, W * world, seed=c["seed"])
    theta = theta_all[rank * W:(rank + 1) * W]
    n_ep, n_pl, n_in = len(ds.time), len(ds.planet_letters), len(ds.unique_instruments)

    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, n_in, n_pl, ds.parameterisation, ds.t0,
                   device=dev.index)
    th_d = torch.from_numpy(theta).to(dev)
    nbuf = 2
    outs = [torch.empty(W, dtype=torch.float64, device=dev) for _ in range(nbuf)]
    gath = [torch.empty(W * world, dtype=torch.float64, device=dev) for _ in range(nbuf)] if world > 1 else None
    stream = torch.cuda.current_stream(dev)

    works = [None] * nbuf

    def step(k, ev=None):
        b = k % nbuf
        if works[b] is not None:       # buffer b's previous all-gather must have read it
            works[b].wait()
        if ev is not None:
            ev[0].record(stream)
        eng.loglike_device(th_d, outs[b], stream)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            works[b] = dist.all_gather_into_tensor(gath[b], outs[b], async_op=True)

    def drain():
        for i, w_ in enumerate(works):
            if w_ is not None:
                w_.wait()
                works[i] = None

    for k in range(args.warmup):
        step(k)
    drain()
    torch.cuda.synchronize(dev)

    # correctness guard on the bench inputs: finite count matches the built-in mask
    ll = outs[(args.warmup - 1) % nbuf].cpu().numpy() if args.warmup else None

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, ev[k])
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))   # per-launch duration on the kernel's stream
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])

    solves = W * n_ep * n_pl * args.steps * world
    value = solves / el
    if rank == 0:
        alg_bytes = W * (n_ep * BYTES_PER_WALKER_EPOCH + theta.shape[1] * 8 + 8)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        pmc = load_pmc(args.config)
        traffic = None
        valu = None
        if pmc:
            traffic = pmc.get("hbm_bytes_per_launch")
            if pmc.get("valu_insts_per_launch"):
                # wave64 fp64 VALU instruction = 64 lane-ops; FP64_VALU_PEAK in lane-ops/s
                ops = pmc["valu_insts_per_launch"] * 64
                valu = {"achieved_lane_ops_per_s": ops / (kern_ms * 1e-3), "peak_fp64_lane_ops_per_s": FP64_VALU_PEAK,
                        "frac": ops / (kern_ms * 1e-3) / FP64_VALU_PEAK, "source": pmc.get("source")}
        line = {
            "metric": "walker-log-prob evals/sec (= Kepler solves/sec) at 1/2/4/8 MI355X",
            "value": value, "unit": "Kepler solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"config {args.config}: {n_pl} planet(s), {n_ep} epochs, {W} walkers per GPU, "
                                   f"fp64, theta resident in HBM" + (", RCCL all-gather of log-probs" if world > 1 else ""),
                       "n_planets": n_pl, "n_epochs": n_ep, "walkers_per_gpu": W, "n_inst": n_in,
                       "parameterisation": ds.parameterisation.parameterisation,
                       "parallelism": f"walker-shard x{world}"},
            "walker_evals_per_s": W * world * args.steps / el,
            "kernel_ms": kern_ms,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "note": "algorithmic bytes = W*(28*N_epochs + 8*P_full + 8) per launch (SURVEY §8(d)); "
                                 "the kernel is fp64-VALU bound, see 'valu'"},
            "valu": valu,
        }
        if ll is not None:
            line["n_masked_walkers"] = int((~np.isfinite(ll)).sum())
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(ds, theta, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
