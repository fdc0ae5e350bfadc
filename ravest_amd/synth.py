"""Seeded synthetic RV datasets and walker ensembles for the BASELINE configs.

SURVEY.md §8(d) fixes the generator: seed ``c`` for config ``c``; epochs
``t = sort(U(0, 1000))``; ``velerr = U(1, 3)``; velocities from a Keplerian
truth (``P=U(2,50) K=U(5,50) e=U(0,0.9) w=U(-pi,pi) Tp=U(0,P)``) plus per-
instrument offsets plus Gaussian noise of variance ``velerr^2 + jit^2``.
Walkers are a 5 % Gaussian ball around the truth with ~2 % deliberately
invalid rows (``e >= 1``, ``K <= 0``, ``jit < 0``) so every mask is exercised.

Nothing here is on the measured path: it only produces inputs.  The truth
velocities use a small vectorised Kepler solve (Newton on ``E - e sin E = M``);
they are data, not a reference result.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .param import Parameterisation, full_param_names

# config id -> shape (BASELINE.json "configs")
CONFIGS = {
    2: dict(seed=2, n_planets=1, n_epochs=256, n_walkers=4096, n_inst=1),
    3: dict(seed=3, n_planets=3, n_epochs=1024, n_walkers=16384, n_inst=2),
    4: dict(seed=4, n_planets=2, n_epochs=512, n_walkers=65536, n_inst=1),
    5: dict(seed=5, n_planets=1, n_epochs=512, n_walkers=4096, n_inst=1),   # + quasi-periodic GP
}

LETTERS = [c for c in "bcdefghijklmnopqrstuvwxyz"] + [f"z{k}" for k in range(8)]   # 33 planet names
INSTRUMENTS = ["HARPS", "HIRES", "ESPRESSO", "CORALIE"] + [f"INST{k:02d}" for k in range(60)]


@dataclass
class Dataset:
    time: np.ndarray
    vel: np.ndarray
    velerr: np.ndarray
    instrument: np.ndarray          # per-epoch instrument name (str)
    unique_instruments: list
    inst_idx: np.ndarray            # int32, index into unique_instruments
    t0: float
    planet_letters: list
    parameterisation: Parameterisation
    truth: dict                     # full parameter dict at the truth
    names: list = field(default_factory=list)   # full parameter order
    theta: np.ndarray | None = None  # [W, P_full] walker block in `names` order


def _kepler_E(M, e):
    E = M + e * np.sin(M)
    for _ in range(60):
        E = E - (E - e * np.sin(E) - M) / (1.0 - e * np.cos(E))
    return E


def _planet_rv(t, P, K, e, w, Tp):
    M = (2 * np.pi / P) * (t - Tp)
    E = _kepler_E(np.mod(M, 2 * np.pi), e)
    f = 2 * np.arctan2(np.sqrt(1 + e) * np.sin(E / 2), np.sqrt(1 - e) * np.cos(E / 2))
    return K * (np.cos(f + w) + e * np.cos(w))


def make_dataset(n_planets: int, n_epochs: int, n_inst: int = 1, seed: int = 2,
                 parameterisation: str = "P K e w Tp", trend: bool = False,
                 t_offset: float = 0.0) -> Dataset:
    rng = np.random.default_rng(seed)
    t = np.sort(rng.uniform(0.0, 1000.0, n_epochs)) + t_offset
    velerr = rng.uniform(1.0, 3.0, n_epochs)
    insts = INSTRUMENTS[:n_inst]
    uniq = sorted(insts)                       # np.unique order (fit.py:113)
    if n_inst == 1:
        inst_names = np.array([insts[0]] * n_epochs)
    else:
        inst_names = np.array(insts)[rng.integers(0, n_inst, n_epochs)]
    inst_idx = np.array([uniq.index(s) for s in inst_names], dtype=np.int32)
    letters = list(LETTERS[:n_planets])
    par = Parameterisation(parameterisation)
    truth = {}
    rv = np.zeros(n_epochs)
    for L in letters:
        P = rng.uniform(2, 50); K = rng.uniform(5, 50); e = rng.uniform(0, 0.9)
        w = rng.uniform(-np.pi, np.pi); Tp = rng.uniform(0, P) + t_offset
        rv += _planet_rv(t, P, K, e, w, Tp)
        default = {"P": P, "K": K, "e": e, "w": w, "Tp": Tp}
        conv = par.convert_pars_from_default_parameterisation(default)
        for k, v in conv.items():
            truth[f"{k}_{L}"] = float(v)
    t0 = float(np.mean(t))
    gd = rng.uniform(-0.02, 0.02) if trend else 0.0
    gdd = rng.uniform(-1e-4, 1e-4) if trend else 0.0
    rv += gd * (t - t0) + gdd * (t - t0) ** 2
    jits = {}
    for i, s in enumerate(uniq):
        g = rng.uniform(-20, 20); jit = rng.uniform(0.5, 2.0)
        truth[f"g_{s}"] = float(g); jits[s] = jit
        rv += np.where(inst_idx == i, g, 0.0)
    for s in uniq:
        truth[f"jit_{s}"] = float(jits[s])
    truth["gd"] = float(gd); truth["gdd"] = float(gdd)
    jit_obs = np.array([jits[uniq[i]] for i in inst_idx])
    vel = rv + rng.normal(0.0, np.sqrt(velerr ** 2 + jit_obs ** 2))
    names = full_param_names(letters, par, uniq)
    return Dataset(time=t, vel=vel, velerr=velerr, instrument=inst_names,
                   unique_instruments=uniq, inst_idx=inst_idx, t0=t0,
                   planet_letters=letters, parameterisation=par, truth=truth,
                   names=names)


def make_walkers(ds: Dataset, n_walkers: int, seed: int = 0, frac_invalid: float = 0.02,
                 scale: float = 0.05) -> np.ndarray:
    """5 % Gaussian ball around ``ds.truth`` with ``frac_invalid`` broken rows."""
    rng = np.random.default_rng(seed + 1000)
    x0 = np.array([ds.truth[n] for n in ds.names])
    theta = x0[None, :] + scale * np.abs(x0)[None, :] * rng.standard_normal((n_walkers, x0.size))
    # trend terms stay at the truth when they are zero (fixed in the configs)
    for j, n in enumerate(ds.names):
        if n in ("gd", "gdd") and x0[j] == 0.0:
            theta[:, j] = 0.0
    # keep the ball inside the domain, so only the deliberate rows are invalid
    for j, n in enumerate(ds.names):
        base = n.split("_")[0]
        if base == "w":
            theta[:, j] = np.mod(theta[:, j] + np.pi, 2 * np.pi) - np.pi
        elif base == "e":
            theta[:, j] = np.clip(theta[:, j], 0.0, 0.98)
        elif base in ("P", "K", "jit"):
            theta[:, j] = np.abs(theta[:, j])
    n_bad = int(round(frac_invalid * n_walkers))
    if n_bad:
        rows = rng.choice(n_walkers, n_bad, replace=False)
        for k, r in enumerate(rows):
            kind = k % 3
            if kind == 0:
                cols = [j for j, n in enumerate(ds.names) if n.split("_")[0] in ("e", "secosw")]
                if cols:
                    j = cols[k % len(cols)]
                    theta[r, j] = 1.0 + rng.uniform(0, 0.2) if ds.names[j].startswith("e") else 1.2
                    continue
                kind = 1
            if kind == 1:
                cols = [j for j, n in enumerate(ds.names) if n.startswith("K_")]
                theta[r, cols[k % len(cols)]] = -rng.uniform(0, 5) if k % 2 else 0.0
            else:
                cols = [j for j, n in enumerate(ds.names) if n.startswith("jit_")]
                theta[r, cols[k % len(cols)]] = -rng.uniform(0.01, 1.0)
    return np.ascontiguousarray(theta)


def make_config(cfg: int, n_walkers: int | None = None) -> Dataset:
    c = CONFIGS[cfg]
    ds = make_dataset(c["n_planets"], c["n_epochs"], c["n_inst"], seed=c["seed"])
    ds.theta = make_walkers(ds, n_walkers or c["n_walkers"], seed=c["seed"])
    return ds


def make_posterior(config: int = 2, n_walkers: int | None = None, device: int = -1, seed: int = 0,
                   e_prior: str = "uniform"):
    """A LogPosterior over the config's synthetic dataset with built-in priors on every
    free parameter (trend fixed at 0), and a tight starting ball around the truth.
    ``e_prior``: the eccentricity prior -- "uniform" (EccentricityUniform(0.99)), or one of
    ravest's eccentricity priors "beta" (Kipping 2013's Beta(0.867, 3.03)), "rayleigh"
    (Rayleigh(0.2)), "vaneylen" (VanEylen19Mixture(0.049, 0.26, 0.08)) (prior.py:252-511).
    Used by the sampler benchmarks (bench.py "sampler", tools/sampler_bench.py)."""
    from . import prior as P
    from .posterior import LogPosterior
    ds = make_config(config, n_walkers=n_walkers or 8)
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    fixed = {"gd": 0.0, "gdd": 0.0}
    priors = {}
    for n in free:
        v = ds.truth[n]
        base = n.split("_")[0]
        if base == "e":
            priors[n] = {"uniform": lambda: P.EccentricityUniform(0.99), "beta": lambda: P.Beta(0.867, 3.03),
                         "rayleigh": lambda: P.Rayleigh(0.2),
                         "vaneylen": lambda: P.VanEylen19Mixture(0.049, 0.26, 0.08)}[e_prior]()
        elif base == "w":
            priors[n] = P.Uniform(-np.pi, np.pi)
        elif base == "jit":
            priors[n] = P.HalfNormal(5.0)
        else:
            priors[n] = P.Uniform(v - 0.5 * abs(v) - 1.0, v + 0.5 * abs(v) + 1.0)
    lpost = LogPosterior(ds.planet_letters, ds.parameterisation, priors, fixed, free, ds.time, ds.vel, ds.velerr,
                         ds.instrument, ds.unique_instruments, ds.t0, device=device)
    W = n_walkers or CONFIGS[config]["n_walkers"]
    rng = np.random.default_rng(seed)
    x0 = np.array([ds.truth[n] for n in free])[None, :] * (1 + 1e-4 * rng.standard_normal((W, len(free))))
    return lpost, x0


def make_gp_config(n_walkers: int | None = None, n_epochs: int = 512, seed: int = 5, n_planets: int = 1,
                   n_inst: int = 1):
    """BASELINE config 5: one planet + quasi-periodic GP residuals.  Returns (dataset,
    theta [W, P_full], hyper [W, 4] (gp_amp, gp_lambda_e, gp_lambda_p, gp_period)).
    The data are a Keplerian plus one draw of the GP (fp64 Cholesky of the truth's
    covariance) plus white noise; walkers are a 5 % ball around the truth (2 % with a
    broken planet, as in make_walkers)."""
    rng = np.random.default_rng(seed + 77)
    ds = make_dataset(n_planets, n_epochs, n_inst, seed=seed)
    hyper0 = np.array([rng.uniform(3, 6), rng.uniform(40, 90), rng.uniform(0.4, 0.8), rng.uniform(15, 30)])
    amp, lam_e, lam_p, per = hyper0
    tau = np.subtract.outer(ds.time, ds.time)
    K = amp ** 2 * np.exp(-np.sin(np.pi * np.abs(tau) / per) ** 2 / (2 * lam_p ** 2)) * np.exp(-0.5 * (tau / lam_e) ** 2)
    Lc = np.linalg.cholesky(K + 1e-8 * amp ** 2 * np.eye(n_epochs))
    ds.vel = ds.vel + Lc @ rng.standard_normal(n_epochs)
    W = n_walkers or CONFIGS[5]["n_walkers"]
    theta = make_walkers(ds, W, seed=seed)
    hyper = hyper0[None, :] * (1 + 0.05 * rng.standard_normal((W, 4)))
    hyper = np.abs(hyper)
    ds.truth.update(dict(zip(["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"], hyper0)))
    return ds, theta, hyper
