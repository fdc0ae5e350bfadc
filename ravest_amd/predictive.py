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
(Planet() would), and the total is trend + sum of planets.
"""
from __future__ import annotations

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
        out = self.engine.predict(self.full(samples_free), np.asarray(times, np.float64), planets=planets,
                                  trend=trend)
        if planets and np.isnan(out).all(axis=1).any():
            bad = int(np.nonzero(np.isnan(out).all(axis=1))[0][0])
            raise ValueError(f"sample {bad}: invalid planet parameters (ravest Planet() raises ValueError)")
        return out

    def rv_planet_from_samples(self, planet_letter: str, times, samples_free) -> np.ndarray:
        """[S, T]: fit.py:2690-2749 for flat samples (free parameters, free_params_names order)."""
        return self._run(samples_free, times, [self.planet_letters.index(planet_letter)], False)

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
