"""Vectorised NumPy restatement of ravest's RV log-likelihood (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

SURVEY.md §8(d)(iii): the reference's per-walker arithmetic, evaluated for a whole walker block
at once with NumPy arrays [W, N] -- the CPU path a ravest user gets by vectorising over walkers
(emcee's ``vectorize=True``) without numba.  Imported by tests/ (checked against the pinned C
oracle, oracle/rv_oracle.c) and by bench.py's cpu_baseline leg; never by the product path.

Follows, element-wise:
  _solve_kepler        src/ravest/model.py:23-70   Halley from E0 = M, |dE| < 1.48e-8, <= 50 iterations;
                                                   sin/cos re-evaluated at E_new on convergence, else the
                                                   last iterate's
  _true_anomaly        model.py:73-122
  _radial_velocity_from_f  model.py:125-170
  _compute_rv          model.py:216-243            e == 0: K (cos(M + w) + e cos w)
  Planet               model.py:259-354            validation (param.py:88-105), n = 2 pi / P, M = n (t - Tp)
  Trend                model.py:483-509
  LogLikelihood.__call__  fit.py:3600-3660          -1/2 sum((rv - v)^2 / s^2 + (log 2 pi + log s^2))
Parameterisation: default ("P K e w Tp") only -- the timing baseline's configuration.
"""
from __future__ import annotations

import numpy as np

LOG_2PI = np.log(2.0 * np.pi)


def solve_kepler(M: np.ndarray, e: np.ndarray, tol: float = 1.48e-08, maxiter: int = 50):
    """(cos E, sin E) for arrays M and e (broadcastable), per element as model.py:23-70."""
    M, e = np.broadcast_arrays(np.asarray(M, np.float64), np.asarray(e, np.float64))
    E = M.copy()
    cos_E = np.zeros_like(M)
    sin_E = np.zeros_like(M)
    active = np.ones(M.shape, dtype=bool)
    for _ in range(maxiter):
        if not active.any():
            break
        Ea, Ma, ea = E[active], M[active], e[active]
        s, c = np.sin(Ea), np.cos(Ea)
        f = Ea - ea * s - Ma
        fp = 1.0 - ea * c
        fpp = ea * s
        E_new = Ea - f / (fp - (f * fpp) / (2.0 * fp))
        done = np.abs(E_new - Ea) < tol
        idx = np.flatnonzero(active)
        # not converged: keep this iterate's sin/cos (returned if maxiter runs out) and step on
        sin_E.flat[idx] = s
        cos_E.flat[idx] = c
        fin = idx[done]
        sin_E.flat[fin] = np.sin(E_new[done])
        cos_E.flat[fin] = np.cos(E_new[done])
        E.flat[idx[~done]] = E_new[~done]
        active.flat[fin] = False
    return cos_E, sin_E


def planet_rv(P, K, e, w, Tp, t) -> np.ndarray:
    """[W, N] RV of one planet for walker arrays P..Tp [W] at times t [N] (valid parameters)."""
    P, K, e, w, Tp = (np.asarray(x, np.float64)[:, None] for x in (P, K, e, w, Tp))
    n = 2.0 * np.pi / P
    M = n * (t[None, :] - Tp)
    cos_E, sin_E = solve_kepler(M, e)
    sqrt_1me2 = np.sqrt(1.0 - e * e)
    cos_w, sin_w = np.cos(w), np.sin(w)
    e_cos_w = e * cos_w
    denom = 1.0 - e * cos_E
    cos_f = (cos_E - e) / denom
    sin_f = sqrt_1me2 * sin_E / denom
    rv = K * (cos_f * cos_w - sin_f * sin_w + e_cos_w)
    circ = (e[:, 0] == 0.0)
    if circ.any():                                           # model.py:236-241
        rv[circ] = (K[circ] * (np.cos(M[circ] + w[circ]) + e[circ] * np.cos(w[circ])))
    return rv


def valid_default(P, K, e, w) -> np.ndarray:
    """param.py:88-105 (ValueError -> False)."""
    return (P > 0) & (K > 0) & (e >= 0) & (e < 1) & (w >= -np.pi) & (w < np.pi)


def loglike(time, vel, velerr, inst_idx, n_inst: int, n_planets: int, t0: float, theta) -> np.ndarray:
    """Per-walker log-likelihood of theta [W, P_full] (include/rvk.h order, "P K e w Tp")."""
    theta = np.atleast_2d(np.asarray(theta, np.float64))
    t = np.asarray(time, np.float64)
    W = theta.shape[0]
    ok = np.ones(W, dtype=bool)
    rv = np.zeros((W, t.size))
    for p in range(n_planets):
        P, K, e, w, Tp = (theta[:, 5 * p + k] for k in range(5))
        good = valid_default(P, K, e, w)
        ok &= good
        if good.any():
            rv[good] += planet_rv(P[good], K[good], e[good], w[good], Tp[good], t)
    g = theta[:, 5 * n_planets: 5 * n_planets + n_inst]
    jit = theta[:, 5 * n_planets + n_inst: 5 * n_planets + 2 * n_inst]
    gd = theta[:, 5 * n_planets + 2 * n_inst][:, None]
    gdd = theta[:, 5 * n_planets + 2 * n_inst + 1][:, None]
    dt = (t - t0)[None, :]
    rv = rv + gd * dt + gdd * dt ** 2 + g[:, inst_idx]
    s2 = np.asarray(velerr, np.float64)[None, :] ** 2 + jit[:, inst_idx] ** 2
    ll = -0.5 * np.sum((rv - np.asarray(vel, np.float64)[None, :]) ** 2 / s2 + (LOG_2PI + np.log(s2)), axis=1)
    ll[~ok] = -np.inf
    return ll
