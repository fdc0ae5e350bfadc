"""Dump the fp64 GP kernel's outputs on config 5 for a bitwise A/B between library builds:
the log-likelihood of 1024 walkers (GPLogLikelihood.device, precision fp64) and the GP-conditioned
mean of 64 of them at 300 times (GPLogLikelihood.condition).  The library is the one
RAVEST_AMD_LIB names (default: the in-tree build).

usage: python tools/gp_dump.py OUT.npz        compare: python tools/gp_dump.py --cmp A.npz B.npz
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    if sys.argv[1] == "--cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for k in a.files:
            x, y = a[k], b[k]
            same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
            fin = np.isfinite(x) & np.isfinite(y)
            rel = float(np.max(np.abs(x[fin] - y[fin]) / np.maximum(np.abs(x[fin]), 1e-300))) if fin.any() else 0.0
            print(f"{k}: bitwise {'identical' if same else 'DIFFERENT'}, max rel diff {rel:.3e}, "
                  f"masks {'same' if np.array_equal(np.isfinite(x), np.isfinite(y)) else 'DIFFER'}")
        return
    import torch
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    W = 1024
    ds, th, hy = make_gp_config(W, n_epochs=512)
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                         ds.parameterisation, GPKernel("Quasiperiodic"), device=0, precision="fp64")
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    gp.device(torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda(), out)
    torch.cuda.synchronize()
    times = np.linspace(ds.time.min(), ds.time.max(), 300)
    cond = gp.condition(th[:64], hy[:64], times)
    np.savez(sys.argv[1], loglike=out.cpu().numpy(), condition=np.asarray(cond))
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
