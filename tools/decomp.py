"""Decompose loglike_kernel time: per-launch µs (50-launch HIP graph replays, as bench.py) over
sweeps of epochs N and walkers W, to separate the fixed per-launch floor, the per-wave
overhead (prep, barrier, reduction) and the per-solve cost.

usage: python tools/decomp.py [np=1]
"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_dataset, make_walkers


def graph_us(eng, th, W, G=50, reps=20):
    cap = torch.cuda.Stream()
    out = torch.empty(G, W, dtype=torch.float64, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for j in range(G):
            eng.loglike_device(th, out[j], cap)
    g.replay(); torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); g.replay(); b.record(s); ev.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3 / G


def main():
    NP = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    # graph-replay floor of a trivial kernel (fill of 4096 doubles)
    x = torch.empty(4096, dtype=torch.float64, device="cuda")
    cap = torch.cuda.Stream(); g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for _ in range(50):
            x.fill_(1.0)
    g.replay(); torch.cuda.synchronize()
    s = torch.cuda.current_stream(); ev = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); g.replay(); b.record(s); ev.append((a, b))
    torch.cuda.synchronize()
    print(json.dumps({"trivial_kernel_us": float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3 / 50}), flush=True)
    cases = [(n, 4096) for n in (1, 64, 128, 256, 512, 1024)] + [(256, w) for w in (256, 1024, 2048, 8192, 16384, 32768)]
    for n, W in cases:
        ds = make_dataset(NP, n, 1, seed=2)
        ds.theta = make_walkers(ds, W, seed=2)
        eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, NP, ds.parameterisation, ds.t0, device=0)
        th = torch.from_numpy(ds.theta).cuda()
        us = graph_us(eng, th, W)
        print(json.dumps({"NP": NP, "N": n, "W": W, "us": round(us, 3),
                          "ns_per_wave_solve_per_simd": round(us * 1e3 / max(1.0, W * NP * -(-n // 64) / 1024), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
