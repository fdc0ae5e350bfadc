"""Raw device stretch-move ms per step (rvk_stretch_run, chain in HBM) for the bench's posteriors:
config 2 with each eccentricity prior kind, config 3, config 4 (65536 walkers).  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from bench import _stretch_raw_ms
    from ravest_amd.synth import make_posterior
    torch.cuda.set_device(0)
    out = {}
    which = sys.argv[1:] or ["uniform", "beta", "rayleigh", "vaneylen", "cfg3", "cfg4"]
    for name in which:
        cfg, prior, W, steps = {"uniform": (2, "uniform", 4096, 256), "uniform_fixed": (2, "uniform", 4096, 256),
                                "beta": (2, "beta", 4096, 256),
                                "rayleigh": (2, "rayleigh", 4096, 256), "vaneylen": (2, "vaneylen", 4096, 256),
                                "cfg3": (3, "uniform", 16384, 64), "cfg4": (4, "uniform", 65536, 32)}[name]
        lp, x0 = make_posterior(cfg, W, device=0, e_prior=prior)
        reps = [_stretch_raw_ms(lp, x0, steps, flags=int(name.endswith("_fixed")))[0] for _ in range(3)]
        out[name] = {"ms_per_step": sorted(reps)[1], "reps": reps, "W": W, "D": x0.shape[1]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
