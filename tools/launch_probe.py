"""Timed-region overhead of K config-2 steps: one G=K-launch HIP graph replay (bench.py's way) vs
K eager launches from Python (ctypes) vs K eager launches with the ctypes call pre-bound.
Wall time per step (barrier-free: synchronize, perf_counter, launches, synchronize) and the
event time per launch."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from ravest_amd import _lib
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ds = make_config(2)
    W = len(ds.theta)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    th = torch.from_numpy(ds.theta).to(dev)
    out = torch.empty(W, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    L = _lib.load()
    res = {}
    for K in (20, 200):
        for _ in range(20):
            eng.loglike_device(th, out, st)
        torch.cuda.synchronize()
        # graph
        cap = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            for _ in range(K):
                eng.loglike_device(th, out, cap)
        g.replay()
        torch.cuda.synchronize()
        walls, evs = [], []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(st)
            g.replay()
            b.record(st)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            evs.append(a.elapsed_time(b))
        res[f"graph_K{K}"] = {"wall_us_per_step": 1e6 * np.median(walls) / K, "event_us_per_step": 1e3 * np.median(evs) / K}
        # eager via the engine wrapper
        walls, evs = [], []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(st)
            for _ in range(K):
                eng.loglike_device(th, out, st)
            b.record(st)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            evs.append(a.elapsed_time(b))
        res[f"eager_K{K}"] = {"wall_us_per_step": 1e6 * np.median(walls) / K, "event_us_per_step": 1e3 * np.median(evs) / K}
        # eager, pre-bound ctypes call
        f = L.rvk_loglike_device
        args = (eng._h, th.data_ptr(), W, th.stride(0), out.data_ptr(), st.cuda_stream)
        walls, evs = [], []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(st)
            for _ in range(K):
                f(*args)
            b.record(st)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            evs.append(a.elapsed_time(b))
        res[f"bound_K{K}"] = {"wall_us_per_step": 1e6 * np.median(walls) / K, "event_us_per_step": 1e3 * np.median(evs) / K}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
