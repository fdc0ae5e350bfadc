"""Device log-posterior kernel time (the DIRECT one-kernel form, rvk_logpost_device) for the
config-2 posterior at W = 4096 and H = 2048 walkers (theta resident in HBM; HIP events around
200 back-to-back launches, median of 5 groups), plus the uniform / Beta / VanEylen e priors:
the A/B probe for where the DIRECT kernels are compiled (rvk.hip or rvk_sample.hip).

usage: python tools/logpost_probe.py          (library: RAVEST_AMD_LIB or the in-tree build)
"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd.synth import make_posterior
    res = {}
    for eprior in ("uniform", "beta", "vaneylen"):
        lpost, x0 = make_posterior(2, 4096, device=0, e_prior=eprior)
        dpost = lpost.device_posterior()
        for W in (4096, 2048):
            x = torch.from_numpy(np.ascontiguousarray(x0[:W])).cuda()
            out = torch.empty(W, dtype=torch.float64, device="cuda")
            st = torch.cuda.current_stream()
            for _ in range(10):
                dpost.device(x, out, st)
            torch.cuda.synchronize()
            g = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(200):
                    dpost.device(x, out, st)
                b.record(st)
                torch.cuda.synchronize()
                g.append(a.elapsed_time(b) / 200 * 1e3)
            res[f"{eprior}_W{W}_us"] = round(float(np.median(g)), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
