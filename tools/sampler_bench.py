"""Stretch-move steps/s on BASELINE config 2 (1 planet, 256 epochs, W walkers):
host sampler (numpy stretch move + LogPosterior.log_probability_batch, likelihood on the GPU)
vs the device-resident sampler (rvk_stretch_run) with device (Philox) and host (emcee) draws.

usage: python tools/sampler_bench.py [W=4096] [steps=200]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def build(W):
    from ravest_amd.synth import make_posterior
    return make_posterior(2, W, device=0)


def main():
    import torch
    from ravest_amd.sampler import DeviceEnsembleSampler, EnsembleSampler
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["host", "philox", "emcee"]
    lpost, x0 = build(W)
    D = x0.shape[1]
    out = {"config": f"config 2 posterior: 1 planet, 256 epochs, {W} walkers, {D} free parameters", "steps": steps}

    if "host" in modes:
        s = EnsembleSampler(W, D, lpost.log_probability_batch, seed=1)
        s.run_mcmc(x0, 5)
        t = time.perf_counter()
        s.run_mcmc(x0, steps)
        out["host_sampler_ms_per_step"] = (time.perf_counter() - t) / steps * 1e3
        out["host_sampler_acceptance"] = float(s.acceptance_fraction.mean())

    from ravest_amd import _lib
    graph = int(os.environ.get("SB_GRAPH", "0"))
    _lib.check(_lib.load().rvk_set_option(lpost.log_likelihood.engine._h, _lib.OPT_GRAPH, graph))
    out["graph"] = graph
    for rng in [m for m in modes if m in ("philox", "emcee")]:
        d = DeviceEnsembleSampler(lpost, W, seed=1 if rng == "philox" else np.random.RandomState(1), rng=rng,
                                  steps_per_call=min(steps, 256))
        d.run_mcmc(x0, 16)   # includes the one-time graph capture
        torch.cuda.synchronize()
        t = time.perf_counter()
        d.run_mcmc(x0, steps)
        torch.cuda.synchronize()
        out[f"device_{rng}_ms_per_step"] = (time.perf_counter() - t) / steps * 1e3
        out[f"device_{rng}_acceptance"] = float(d.acceptance_fraction.mean())
    if "raw" in modes:   # rvk_stretch_run alone (HIP events; state and chain stay in HBM, no host copies)
        from ravest_amd.posterior import DevicePosterior
        dp = DevicePosterior(lpost)
        dev = torch.device("cuda", 0)
        x = torch.from_numpy(x0).to(dev)
        lp = torch.empty(W, dtype=torch.float64, device=dev)
        dp.device(x, lp)
        chain = torch.empty((steps, W, D), dtype=torch.float64, device=dev)
        lnpc = torch.empty((steps, W), dtype=torch.float64, device=dev)
        nacc = torch.zeros(W, dtype=torch.int64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        L = _lib.load()
        st = torch.cuda.current_stream(dev)

        def run(n, step0, with_chain):
            _lib.check(L.rvk_stretch_run(dp._p, x.data_ptr(), lp.data_ptr(), W, n, 2.0, 7, step0, 0, 0, 0, 0, 0,
                                         chain.data_ptr() if with_chain else 0, lnpc.data_ptr() if with_chain else 0,
                                         nacc.data_ptr(), status.data_ptr(), st.cuda_stream))
        run(16, 0, True)
        for with_chain in (True, False):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            run(steps, 100, with_chain)
            b.record(st)
            torch.cuda.synchronize()
            out[f"raw_ms_per_step{'_chain' if with_chain else '_nochain'}"] = a.elapsed_time(b) / steps
    if "host_sampler_ms_per_step" in out and "device_philox_ms_per_step" in out:
        out["speedup_device_philox_vs_host"] = out["host_sampler_ms_per_step"] / out["device_philox_ms_per_step"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
