"""DeviceEnsembleSampler.run_mcmc wall-clock (chain + log-probs in host memory) against the raw
kernel step, config-2 posterior, 4096 walkers, for several chunk sizes.  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from bench import _stretch_raw_ms
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    torch.cuda.set_device(0)
    if os.environ.get("E2E_HP"):                         # the run on a high-priority stream
        torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    lpost, x0 = make_posterior(2, 4096, device=0)
    if os.environ.get("RVK_GRAPH"):
        lpost.log_likelihood.engine.set_graph(True)
    raw = sorted(_stretch_raw_ms(lpost, x0, 256)[0] for _ in range(3))[1]
    out = {"kernel_ms_per_step": raw}
    if "quick" not in sys.argv:
        out["kernel_ms_per_step_2048"] = sorted(_stretch_raw_ms(lpost, x0, 2048)[0] for _ in range(3))[1]
        out["kernel_ms_per_step_4096"] = sorted(_stretch_raw_ms(lpost, x0, 4096)[0] for _ in range(3))[1]
    quick = "quick" in sys.argv
    for spc in [int(a) for a in (sys.argv[1:] or ["128", "256", "512"]) if a != "quick"]:
        for steps in ((2048,) if quick else (1024, 2048, 4096)):
            s = DeviceEnsembleSampler(lpost, 4096, seed=1234, steps_per_call=spc)
            s.run_mcmc(x0, 2 * spc)
            ts = []
            for _ in range(3):
                s.reset()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                s.run_mcmc(x0, steps)
                ts.append(time.perf_counter() - t0)
            ms = sorted(ts)[1] / steps * 1e3
            out[f"spc{spc}_steps{steps}"] = {"e2e_ms_per_step": ms, "over_kernel": ms / raw}
    os.environ["RVK_SAMPLER_TRACE"] = "1"
    s = DeviceEnsembleSampler(lpost, 4096, seed=1234, steps_per_call=256)
    s.run_mcmc(x0, 512)
    s.reset()
    s._trace.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run_mcmc(x0, 2048)
    out["trace_ms"] = [(k, round(1e3 * (t - t0), 3)) for k, t in s._trace]
    g = s._gpu_trace[-8:]
    out["gpu_chunks_ms"] = [(round(a.elapsed_time(b), 3), round(b.elapsed_time(c), 3),
                             round(c.elapsed_time(g[i + 1][0]), 3) if i + 1 < len(g) else None)
                            for i, (a, b, c) in enumerate(g)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
