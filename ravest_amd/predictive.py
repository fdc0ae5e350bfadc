"""Posterior-predictive RVs on the GPU.

Batched mirror of ravest's per-sample loops
``Fitter.calculate_rv_{planet,trend,total}_from_samples`` (fit.py:2690-2824) and
``calculate_rv_{planet,trend,total}_custom`` (fit.py:2826-2939): the reference
builds a params dict and a ``Planet`` per sample and calls
``Planet.radial_velocity(times)`` (model.py:329-354) -- (samples x times)
Kepler solves with no reduction.  Here one ``rvk_predict`` launch evaluates the
whole [S, T] grid (one wave per sample, lanes over times, same conversion and
solver as the log-likelihood kernel).

As in the reference, an invalid planet in any sample raises ``ValueError``
(Planet() would), and the total is trend + sum of planets.  ``freeze_params``
overrides planet parameters in every sample (fit.py:2586-2749; ``None`` values
resolve to the posterior median over the given samples).

``GPPosteriorPredictive`` adds the GP half of GPFitter's predictive
(fit.py:7241-7594): the GP conditioned on each sample's residuals at the data,
evaluated at the requested times (rvk_gp_predict, fp64), and the total
trend + planets + GP.
"""
from __future__ import annotations

import warnings

import numpy as np

from .engine import RVEngine
from .param import Parameterisation, as_parameterisation, full_param_names


class PosteriorPredictive:
    def __init__(self, planet_letters, parameterisation: Parameterisation, fixed_params: dict,
                 free_params_names: list, unique_instruments, t0: float, device: int = -1) -> None:
        parameterisation = as_parameterisation(parameterisation)   # str, ours or ravest's own object
        self.planet_letters = list(planet_letters)
        self.parameterisation = parameterisation
        self.fixed_params = dict(fixed_params)
        self.free_params_names = list(free_params_names)
        self.unique_instruments = list(unique_instruments)
        self.t0 = float(t0)
        self.names = full_param_names(self.planet_letters, parameterisation, self.unique_instruments)
        self._template = np.array([float(self.fixed_params.get(n, np.nan)) for n in self.names])
        self._free_idx = np.array([self.names.index(n) for n in self.free_params_names], dtype=np.int64)
        self.engine = RVEngine(None, None, None, None, len(self.unique_instruments), len(self.planet_letters),
                               parameterisation, self.t0, device=device)

    # fit.py:1390-1430 build_params_dict, for a whole block of samples
    def full(self, samples_free) -> np.ndarray:
        samples_free = np.atleast_2d(np.asarray(samples_free, dtype=np.float64))
        full = np.repeat(self._template[None, :], samples_free.shape[0], axis=0)
        full[:, self._free_idx] = samples_free
        return full

    def _run(self, samples_free, times, planets, trend):
        return self._run_full(self.full(samples_free), times, planets, trend)

    def _run_full(self, full, times, planets, trend):
        out = self.engine.predict(full, np.asarray(times, np.float64), planets=planets, trend=trend)
        if planets and np.isnan(out).all(axis=1).any():
            bad = int(np.nonzero(np.isnan(out).all(axis=1))[0][0])
            raise ValueError(f"sample {bad}: invalid planet parameters (ravest Planet() raises ValueError)")
        return out

    def resolve_freeze_params(self, freeze_params, samples_free, planet_letter=None):
        """fit.py:2586-2688 (GPFitter: 7137-7239): validate ``freeze_params`` (keys are planet
        parameters of the active parameterisation), warn on a key for another planet or on an
        already-fixed parameter, and resolve ``None`` values to the median over the samples
        (a fixed parameter resolves to its fixed value)."""
        if freeze_params is None:
            return None
        valid_names = {f"{par}_{letter}" for par in self.parameterisation.pars for letter in self.planet_letters}
        unknown = set(freeze_params) - valid_names
        if unknown:
            raise ValueError(f"Unknown freeze_params key(s): {sorted(unknown)}. Keys must be planet parameters of "
                             f"the active parameterisation, i.e. one of {sorted(valid_names)}.")
        if planet_letter is not None:
            wrong_planet = [key for key in freeze_params if key.rsplit("_", 1)[-1] != planet_letter]
            if wrong_planet:
                warnings.warn(f"freeze_params names parameter(s) for a different planet than '{planet_letter}': "
                              f"{sorted(wrong_planet)}. Freezing is intended for the target planet's parameters "
                              "(typically P and Tc); check the planet letter.", UserWarning, stacklevel=2)
        fixed_frozen = [key for key in freeze_params if key not in self.free_params_names]
        if fixed_frozen:
            warnings.warn(f"freeze_params names parameter(s) that are already fixed, not free: {sorted(fixed_frozen)}. "
                          "Freezing only affects parameters that vary across posterior samples, so this has no "
                          "de-smearing effect (a None value just resolves to the fixed value). Did you mean a free "
                          "parameter, or pass the wrong name?", UserWarning, stacklevel=2)
        samples_free = np.atleast_2d(np.asarray(samples_free, dtype=np.float64))
        resolved = {}
        for key, value in freeze_params.items():
            if value is None:
                if key in self.free_params_names:
                    resolved[key] = float(np.median(samples_free[:, self.free_params_names.index(key)]))
                else:
                    resolved[key] = float(self.fixed_params[key])
            else:
                resolved[key] = float(value)
        return resolved

    def _frozen(self, samples_free, resolved):
        full = self.full(samples_free)
        for key, v in (resolved or {}).items():
            full[:, self.names.index(key)] = v
        return full

    def rv_planet_from_samples(self, planet_letter: str, times, samples_free, freeze_params=None) -> np.ndarray:
        """[S, T]: fit.py:2690-2749 for flat samples (free parameters, free_params_names order)."""
        resolved = self.resolve_freeze_params(freeze_params, samples_free, planet_letter=planet_letter)
        if not resolved:
            return self._run(samples_free, times, [self.planet_letters.index(planet_letter)], False)
        return self._run_full(self._frozen(samples_free, resolved), times, [self.planet_letters.index(planet_letter)],
                              False)

    def rv_trend_from_samples(self, times, samples_free) -> np.ndarray:
        """[S, T]: fit.py:2751-2789 (gd (t - t0) + gdd (t - t0)^2)."""
        return self._run(samples_free, times, [], True)

    def rv_total_from_samples(self, times, samples_free) -> np.ndarray:
        """[S, T]: fit.py:2791-2824 (trend + every planet)."""
        return self._run(samples_free, times, list(range(len(self.planet_letters))), True)

    # fit.py:2826-2939 *_custom: one complete params dict
    def _row(self, params: dict) -> np.ndarray:
        return np.array([[params[n] for n in self.names]], dtype=np.float64)

    def rv_planet_custom(self, planet_letter: str, times, params: dict) -> np.ndarray:
        out = self.engine.predict(self._row(params), np.asarray(times, np.float64),
                                  planets=[self.planet_letters.index(planet_letter)], trend=False)[0]
        if np.isnan(out).all():
            raise ValueError("invalid planet parameters (ravest Planet() raises ValueError)")
        return out

    def rv_trend_custom(self, times, params: dict) -> np.ndarray:
        return self.engine.predict(self._row(params), np.asarray(times, np.float64), planets=[], trend=True)[0]

    def rv_total_custom(self, times, params: dict) -> np.ndarray:
        out = self.engine.predict(self._row(params), np.asarray(times, np.float64), trend=True)[0]
        if np.isnan(out).all():
            raise ValueError("invalid planet parameters (ravest Planet() raises ValueError)")
        return out


class GPPosteriorPredictive(PosteriorPredictive):
    """GPFitter's per-sample predictive (fit.py:7241-7594), batched: samples are emcee's combined
    coordinates [S, len(free_params_names) + len(free_hyperparams_names)]."""

    def __init__(self, planet_letters, parameterisation, fixed_params: dict, free_params_names: list,
                 fixed_hyperparams: dict, free_hyperparams_names: list, time, vel, velerr, instrument,
                 unique_instruments, t0: float, gp_kernel, device: int = -1) -> None:
        from .gp import HYPERPARAMS, GPLogLikelihood
        super().__init__(planet_letters, parameterisation, fixed_params, free_params_names, unique_instruments, t0,
                         device=device)
        self.fixed_hyperparams = dict(fixed_hyperparams)
        self.free_hyperparams_names = list(free_hyperparams_names)
        self._hyper = list(HYPERPARAMS)
        self._htemplate = np.array([float(self.fixed_hyperparams.get(k, np.nan)) for k in HYPERPARAMS])
        self._hfree_idx = np.array([HYPERPARAMS.index(k) for k in self.free_hyperparams_names], dtype=np.int64)
        self.gp = GPLogLikelihood(time, vel, velerr, t0, instrument, unique_instruments, self.planet_letters,
                                  self.parameterisation, gp_kernel, device=device, precision="fp64")
        if self.gp.names != self.names:
            raise RuntimeError("parameter layout mismatch between the predictive and the GP likelihood")

    def _split(self, samples):
        samples = np.atleast_2d(np.asarray(samples, dtype=np.float64))
        nf = len(self.free_params_names)
        hyper = np.repeat(self._htemplate[None, :], samples.shape[0], axis=0)
        hyper[:, self._hfree_idx] = samples[:, nf:]
        return samples[:, :nf], hyper

    def _gp(self, full, hyper, times):
        out = self.gp.condition(full, hyper, times)
        if np.isnan(out).all(axis=1).any():
            bad = int(np.nonzero(np.isnan(out).all(axis=1))[0][0])
            raise ValueError(f"sample {bad}: invalid planet parameters (ravest Planet() raises ValueError)")
        return out

    def rv_planet_from_samples(self, planet_letter: str, times, samples, freeze_params=None) -> np.ndarray:
        """fit.py:7241-7302."""
        return super().rv_planet_from_samples(planet_letter, times, self._split(samples)[0], freeze_params)

    def rv_trend_from_samples(self, times, samples) -> np.ndarray:
        """fit.py:7304-7340."""
        return super().rv_trend_from_samples(times, self._split(samples)[0])

    def rv_gp_from_samples(self, times, samples) -> np.ndarray:
        """[S, T]: fit.py:7342-7386 -- the GP component of every sample, conditioned on that
        sample's residuals (vel - gamma - trend - planets) at the data times."""
        xp, hyper = self._split(samples)
        return self._gp(self.full(xp), hyper, times)

    def rv_total_from_samples(self, times, samples) -> np.ndarray:
        """[S, T]: fit.py:7388-7425 (trend + planets at ``times``, + the GP component)."""
        xp, hyper = self._split(samples)
        total = self._run(xp, times, list(range(len(self.planet_letters))), True)
        return total + self._gp(self.full(xp), hyper, times)

    # fit.py:7494-7594 *_custom: one complete params + hyperparams dict
    def _hrow(self, params: dict) -> np.ndarray:
        return np.array([[params[k] for k in self._hyper]], dtype=np.float64)

    def rv_gp_custom(self, times, params: dict) -> np.ndarray:
        return self._gp(self._row(params), self._hrow(params), times)[0]

    def rv_total_custom(self, times, params: dict) -> np.ndarray:
        return super().rv_total_custom(times, params) + self.rv_gp_custom(times, params)
