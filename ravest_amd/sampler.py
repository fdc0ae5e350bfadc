"""Vectorised affine-invariant ensemble sampler (emcee's StretchMove semantics).

ravest's Fitter.run_mcmc drives emcee.EnsembleSampler with one Python call per
walker (fit.py:1068-1111).  The batched log-probability takes the whole
half-ensemble at once; with emcee installed, use

    emcee.EnsembleSampler(nwalkers, ndim, lpost.log_probability_batch, vectorize=True)

emcee is not available in this image, so this module provides the same move
(Goodman & Weare stretch, a = 2, red-blue halves with a random split each step,
as emcee 3.1's StretchMove/RedBlueMove) with emcee's chain layout
(steps, walkers, dim), so samples can be consumed like ``sampler.get_chain``.
It is the host-side stretch move that the multi-GPU all-gather feeds
(SURVEY.md §5, §8(e)).
"""
from __future__ import annotations

import numpy as np


class EnsembleSampler:
    def __init__(self, nwalkers: int, ndim: int, log_prob_batch, a: float = 2.0, seed=None) -> None:
        if nwalkers < 2 * ndim:
            raise ValueError(f"nwalkers ({nwalkers}) must be at least 2 * ndim ({2 * ndim})")
        if nwalkers % 2:
            raise ValueError("nwalkers must be even for the red-blue stretch move")
        self.nwalkers, self.ndim, self.a = nwalkers, ndim, float(a)
        self.log_prob_batch = log_prob_batch
        self.rng = np.random.default_rng(seed)
        self.reset()

    def reset(self) -> None:
        self._chain, self._lnp = [], []
        self.naccepted = np.zeros(self.nwalkers, dtype=np.int64)
        self.iteration = 0

    def _propose(self, s, c):
        ns, nc = len(s), len(c)
        zz = ((self.a - 1.0) * self.rng.random(ns) + 1.0) ** 2.0 / self.a
        factors = (self.ndim - 1.0) * np.log(zz)
        rint = self.rng.integers(nc, size=ns)
        return c[rint] - (c[rint] - s) * zz[:, None], factors

    def sample(self, initial_state, iterations: int):
        x = np.array(initial_state, dtype=np.float64, copy=True)
        if x.shape != (self.nwalkers, self.ndim):
            raise ValueError(f"initial_state must have shape ({self.nwalkers}, {self.ndim})")
        lnp = np.asarray(self.log_prob_batch(x), dtype=np.float64)
        if np.any(np.isnan(lnp)):
            raise ValueError("The initial log_prob was NaN")
        if not np.all(np.isfinite(lnp)):
            raise ValueError("Initial state has walkers with -inf log-probability")
        for _ in range(iterations):
            idx = self.rng.permutation(self.nwalkers)        # randomize_split (emcee RedBlueMove)
            halves = (idx[: self.nwalkers // 2], idx[self.nwalkers // 2:])
            for k in (0, 1):
                S, Cc = halves[k], halves[1 - k]
                q, factors = self._propose(x[S], x[Cc])
                new = np.asarray(self.log_prob_batch(q), dtype=np.float64)
                if np.any(np.isnan(new)):
                    raise ValueError("The log_prob was NaN")      # emcee's behaviour: -inf rejects, NaN raises
                lnpdiff = factors + new - lnp[S]
                acc = lnpdiff > np.log(self.rng.random(len(S)))
                x[S[acc]] = q[acc]
                lnp[S[acc]] = new[acc]
                self.naccepted[S[acc]] += 1
            self.iteration += 1
            self._chain.append(x.copy())
            self._lnp.append(lnp.copy())
            yield x, lnp

    def run_mcmc(self, initial_state, nsteps: int):
        state = None
        for state in self.sample(initial_state, nsteps):
            pass
        return state

    @property
    def acceptance_fraction(self) -> np.ndarray:
        return self.naccepted / max(1, self.iteration)

    def get_chain(self, discard: int = 0, thin: int = 1, flat: bool = False) -> np.ndarray:
        ch = np.array(self._chain)[discard::thin]
        return ch.reshape(-1, self.ndim) if flat else ch

    def get_log_prob(self, discard: int = 0, thin: int = 1, flat: bool = False) -> np.ndarray:
        lp = np.array(self._lnp)[discard::thin]
        return lp.reshape(-1) if flat else lp
