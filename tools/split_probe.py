import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_dataset, make_walkers
def t(W, N):
    ds = make_dataset(1, N, 1, seed=2)
    th = make_walkers(ds, W, seed=2)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    eng.reserve(W)
    tt = torch.from_numpy(th).cuda(); out = torch.empty(W, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(20): eng.loglike_device(tt, out, s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(50): eng.loglike_device(tt, out, s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(5):
        a.record(); g.replay(); b.record(); torch.cuda.synchronize(); res.append(a.elapsed_time(b) / 50 * 1e3)
    return np.median(res)
for W, N in [(4096, 256), (8192, 128), (2048, 256), (4096, 128), (16384, 64)]:
    print(W, N, f"{t(W, N):.2f} us")
