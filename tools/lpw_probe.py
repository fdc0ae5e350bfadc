"""Config-2 launches with a forced lanes-per-walker layout (PMC / timing probe).
usage: python tools/lpw_probe.py LPW [launches=50]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    lpw = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    ds = make_config(2)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    eng.set_lanes_per_walker(lpw)
    th = torch.from_numpy(ds.theta).cuda()
    out = torch.empty(len(ds.theta), dtype=torch.float64, device="cuda")
    for _ in range(n):
        eng.loglike_device(th, out)
    torch.cuda.synchronize()
    print(lpw, float(out[:8].sum()))


if __name__ == "__main__":
    main()
