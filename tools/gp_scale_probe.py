"""GP kernel time vs walkers per launch (fp32 / fp64): a bandwidth-bound kernel gets faster per
walker when fewer CUs run; a per-CU latency-bound one keeps its time per CU generation.
usage: python tools/gp_scale_probe.py"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(4096, n_epochs=512)
    res = {}
    for prec in os.environ.get("GPS_PREC", "fp64,fp32").split(","):
        gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments,
                             ds.planet_letters, ds.parameterisation, GPKernel("Quasiperiodic"), device=0, precision=prec)
        for W in [int(x) for x in os.environ.get('GPS_W', '32,64,128,256,512,1024,2048,4096').split(',')]:
            tt, ht = torch.from_numpy(th[:W]).cuda(), torch.from_numpy(hy[:W]).cuda()
            out = torch.empty(W, dtype=torch.float64, device="cuda")
            s = torch.cuda.current_stream()
            gp.device(tt, ht, out, s)
            torch.cuda.synchronize()
            reps = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                gp.device(tt, ht, out, s)
                b.record(s)
                torch.cuda.synchronize()
                reps.append(a.elapsed_time(b))
            res[f"{prec}_W{W}"] = round(float(np.median(reps)), 4)
        gp.close()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
