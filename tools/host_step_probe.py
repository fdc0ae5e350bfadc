"""Per-phase cost of the host stretch move driving LogPosterior.log_probability_batch
(the north-star drop-in path, fit.py:1068-1075): emcee's numpy step alone, the host-side
posterior work (template scatter, jitter mask, priors), and -- on a GPU -- the engine call
through each route.  Usage: python tools/host_step_probe.py [--cpu] [--walkers 4096]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def tmin(fn, reps=50, inner=1):
    best = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(inner):
            fn()
        best.append((time.perf_counter() - t0) / inner)
    return float(np.median(best)) * 1e6, float(np.min(best)) * 1e6


class _ZeroEngine:
    def loglike(self, theta):
        return np.zeros(theta.shape[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true", help="mock the engine (no GPU)")
    ap.add_argument("--walkers", type=int, default=4096)
    a = ap.parse_args()
    from ravest_amd.sampler import EnsembleSampler
    from ravest_amd.synth import make_posterior
    W = a.walkers
    lpost, x0 = make_posterior(2, W, device=-1 if a.cpu else 0)
    H = W // 2
    q = np.ascontiguousarray(x0[:H])
    res = {"walkers": W, "half": H, "free": x0.shape[1]}
    # emcee step with a free log-prob (the sampler's own numpy work)
    hs = EnsembleSampler(W, x0.shape[1], lambda x: np.zeros(len(x)), seed=1)
    hs.run_mcmc(x0, 2)
    res["emcee_step_only_us"] = tmin(lambda: hs.run_mcmc(None, 1), reps=30)
    # host posterior work with a zero likelihood
    real = lpost.log_likelihood._engine
    lpost.log_likelihood._engine = _ZeroEngine()
    res["host_posterior_work_us"] = tmin(lambda: lpost.log_probability_batch(q), reps=30)
    full = lpost._full(q)
    res["full_scatter_us"] = tmin(lambda: lpost._full(q), reps=30)
    res["priors_us"] = tmin(lambda: lpost._log_prior_batch(q, full), reps=30)
    lpost.log_likelihood._engine = real
    if not a.cpu:
        eng = lpost.log_likelihood.engine
        fl = np.ascontiguousarray(full)
        eng.loglike(fl)
        res["engine_loglike_H_us"] = tmin(lambda: eng.loglike(fl), reps=50)
        res["engine_loglike_1_us"] = tmin(lambda: eng.loglike(fl[:1]), reps=200)
        res["log_probability_batch_H_us"] = tmin(lambda: lpost.log_probability_batch(q), reps=50)
        d = dict(zip(lpost.free_params_names, q[0]))
        res["log_probability_dict_us"] = tmin(lambda: lpost.log_probability(d), reps=200)
        dp = lpost.device_posterior()
        dp(q)
        res["device_posterior_H_us"] = tmin(lambda: dp(q), reps=50)
        res["device_posterior_1_us"] = tmin(lambda: dp(q[:1]), reps=200)
        hs = EnsembleSampler(W, x0.shape[1], lpost.log_probability_batch, seed=1)
        hs.run_mcmc(x0, 2)
        res["host_stretch_step_us"] = tmin(lambda: hs.run_mcmc(None, 1), reps=20)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
