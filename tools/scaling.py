"""Kernel time vs (walkers, epochs) for the 1-planet loglike kernel: separates fixed cost from per-epoch cost."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_dataset, make_walkers
from tools.kbench import timeit
for N in (64, 256, 1024):
    ds = make_dataset(1, N, 1, seed=2)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    for W in (256, 1024, 4096, 8192, 16384, 65536):
        th = torch.from_numpy(make_walkers(ds, W, seed=2)).cuda()
        out = torch.empty(W, dtype=torch.float64, device="cuda")
        us = timeit(eng, th, out, reps=20, rounds=3)
        print(json.dumps({"N": N, "W": W, "us": round(us, 2), "solves_per_s": W * N / us * 1e6}), flush=True)
