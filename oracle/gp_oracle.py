"""CPU restatement of ravest's GP log-likelihood (TEST INFRASTRUCTURE ONLY).

Parity is UNPINNED at the tinygp boundary: ravest computes
``tinygp.GaussianProcess(kernel, X=time, diag=velerr^2 + jit^2).log_probability(
vel - mean)`` (src/ravest/fit.py:8053-8067, 8087-8105) and tinygp (pinned
``tinygp>=0.3.0,<0.4.0``, pyproject.toml:31) is not installed here, nor are any
numeric GP fixtures in the reference's tests (tests/test_fit.py:1549-1575
checks finiteness only).  This module restates tinygp 0.3's published
algorithm -- DirectSolver: L = cholesky(K + diag(d)), alpha = L^-1 r,
log_probability = -1/2 alpha.alpha - sum(log diag L) - N/2 log(2 pi) -- in
fp64 with numpy/scipy, with the kernel of ravest's GPKernel.build_kernel
(src/ravest/gp.py:126-156) and the mean model of GPLogLikelihood
(_calculate_mean_model, fit.py:7995-8047) taken from the pinned C oracle
(oracle/rv_oracle.c, planet RVs) plus trend and gamma.

``gp_condition`` restates tinygp 0.3's ``GaussianProcess.condition(y, X_test).mean``
with the zero mean function (alpha = (K + diag)^-1 r by Cholesky, mean =
K(X_test, X) alpha), as GPFitter.calculate_rv_gp_custom calls it
(fit.py:7494-7554): residuals = (vel - gamma[inst]) - (trend + planets).
Same "parity unpinned" status as the likelihood.
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cho_factor, cho_solve, solve_triangular

from . import oracle


def qp_kernel(t, amp, lam_e, lam_p, period):
    """gp.py:126-156: amp^2 ExpSineSquared(P, gamma=1/(2 lam_p^2)) ExpSquared(lam_e)."""
    tau = np.subtract.outer(t, t)
    gamma = 1.0 / (2.0 * lam_p ** 2)
    return amp ** 2 * np.exp(-gamma * np.sin(np.pi * np.abs(tau) / period) ** 2) * np.exp(-0.5 * (tau / lam_e) ** 2)


def mean_model(time, inst_idx, n_inst, n_planets, par_code, t0, row):
    rv = np.zeros(len(time))
    for p in range(n_planets):
        r = oracle.planet_rv(par_code, row[5 * p: 5 * p + 5], time)
        if r is None:
            return None                                        # Planet() raised: -inf
        rv += r
    g = row[5 * n_planets: 5 * n_planets + n_inst]
    gd, gdd = row[5 * n_planets + 2 * n_inst], row[5 * n_planets + 2 * n_inst + 1]
    rv += gd * (time - t0) + gdd * (time - t0) ** 2
    return rv + g[inst_idx]


def gp_loglike(time, vel, velerr, inst_idx, n_inst, n_planets, par_code, t0, theta, hyper):
    """Per-walker GP log-likelihood, fp64.  theta [W, P_full] (include/rvk.h order), hyper [W, 4]."""
    theta = np.atleast_2d(theta)
    hyper = np.atleast_2d(hyper)
    out = np.empty(len(theta))
    n = len(time)
    for w, (row, hp) in enumerate(zip(theta, hyper)):
        mu = mean_model(time, inst_idx, n_inst, n_planets, par_code, t0, row)
        if mu is None:
            out[w] = -np.inf
            continue
        jit = row[5 * n_planets + n_inst: 5 * n_planets + 2 * n_inst]
        K = qp_kernel(time, *hp)
        K[np.diag_indices(n)] += velerr ** 2 + jit[inst_idx] ** 2
        try:
            L, _ = cho_factor(K, lower=True, check_finite=False)
        except np.linalg.LinAlgError:
            out[w] = np.nan
            continue
        alpha = solve_triangular(L, vel - mu, lower=True, check_finite=False)
        out[w] = -0.5 * alpha @ alpha - np.sum(np.log(np.diag(L))) - 0.5 * n * np.log(2 * np.pi)
    return out


def qp_kernel_cross(tq, t, amp, lam_e, lam_p, period):
    """K(X_test, X): gp.py:126-156 between query and data times (no diagonal term)."""
    tau = np.subtract.outer(tq, t)
    gamma = 1.0 / (2.0 * lam_p ** 2)
    return amp ** 2 * np.exp(-gamma * np.sin(np.pi * np.abs(tau) / period) ** 2) * np.exp(-0.5 * (tau / lam_e) ** 2)


def gp_condition(time, vel, velerr, inst_idx, n_inst, n_planets, par_code, t0, theta, hyper, tq):
    """[S, T] fp64 conditional GP mean at tq per sample (NaN row: invalid planet)."""
    theta = np.atleast_2d(theta)
    hyper = np.atleast_2d(hyper)
    tq = np.asarray(tq, np.float64)
    out = np.empty((len(theta), len(tq)))
    n = len(time)
    for s, (row, hp) in enumerate(zip(theta, hyper)):
        mu = mean_model(time, inst_idx, n_inst, n_planets, par_code, t0, row)
        if mu is None:
            out[s] = np.nan
            continue
        jit = row[5 * n_planets + n_inst: 5 * n_planets + 2 * n_inst]
        K = qp_kernel(time, *hp)
        K[np.diag_indices(n)] += velerr ** 2 + jit[inst_idx] ** 2
        alpha = cho_solve(cho_factor(K, lower=True, check_finite=False), vel - mu, check_finite=False)
        out[s] = qp_kernel_cross(tq, time, *hp) @ alpha
    return out
