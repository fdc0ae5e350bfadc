"""WRITE_SIZE micro-probe for the posterior predictive's 1.51x write bytes (Weak 6).

Three kernels write the same [S, T] fp64 block (S = 98.7 k samples, T = 1000 times, 0.79 GB):
  * predict_kernel (rvk_predict_device, the bench's predictive line: one wave per sample, lanes
    over times, 512-byte row chunks);
  * torch's fill_ of the same tensor (a plain full-line streaming write);
  * torch's fill_ of a [S, 1024] tensor (rows a multiple of 128 bytes).
Run under `rocprofv3 --pmc WRITE_SIZE -- python tools/probe_write.py` (and a FETCH_SIZE pass):
each kernel's WRITE_SIZE (KB per dispatch) against its bytes says whether the predictive's
excess is its store pattern or the counter.  Prints the byte counts per kernel for the summary."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    ds = make_config(2)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    rng = np.random.default_rng(7)
    good = ds.theta[np.all(np.isfinite(ds.theta), axis=1)]
    samples = good[rng.integers(0, len(good), 100_000)]
    samples = samples[(samples[:, 2] >= 0) & (samples[:, 2] < 1) & (samples[:, 1] > 0)]
    S, T = len(samples), 1000
    th = torch.from_numpy(np.ascontiguousarray(samples)).cuda()
    tq = torch.linspace(0.0, 1000.0, T, dtype=torch.float64, device="cuda")
    out = torch.empty((S, T), dtype=torch.float64, device="cuda")
    out2 = torch.empty((S, 1024), dtype=torch.float64, device="cuda")
    out3 = torch.empty((S, 2048), dtype=torch.float64, device="cuda")
    tq2 = torch.linspace(0.0, 1000.0, 1024, dtype=torch.float64, device="cuda")
    cases = [  # label, bytes written, fn -- each run 3 times back to back, in this order
        ("predict T=1000 (rows 8000 B, 8 B/lane)", S * T * 8, lambda: eng.predict_device(th, tq, out)),
        ("predict T=1024 (rows 8192 B, 8 B/lane)", S * 1024 * 8, lambda: eng.predict_device(th, tq2, out2)),
        ("fill [S,1000] contiguous (vectorised)", S * T * 8, lambda: out.fill_(1.0)),
        ("fill [S,1024] contiguous (vectorised)", S * 1024 * 8, lambda: out2.fill_(2.0)),
        ("fill [S,:999] of [S,1000] (8 B/lane, rows 8000 B)", S * 999 * 8, lambda: out[:, :999].fill_(3.0)),
        ("fill [S,:1024] of [S,2048] (8 B/lane, rows aligned)", S * 1024 * 8, lambda: out3[:, :1024].fill_(4.0)),
    ]
    torch.cuda.synchronize()
    for _, _, fn in cases:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
    print(json.dumps({"S": S, "T": T, "reps": 3, "cases": [[c[0], c[1]] for c in cases]}))


if __name__ == "__main__":
    main()
