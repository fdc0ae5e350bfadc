"""Affine-invariant ensemble samplers with emcee's StretchMove semantics.

ravest's Fitter.run_mcmc drives ``emcee.EnsembleSampler`` (fit.py:1068-1111)
with the default move, ``StretchMove(a=2)`` = ``RedBlueMove(nsplits=2,
randomize_split=True)``: each step shuffles ``arange(W) % 2`` into two halves
and updates each half against the other (proposal ``c - (c - s) z``,
``z = ((a-1) u + 1)^2 / a``, acceptance ``(ndim-1) log z + lp(q) - lp(s) >
log u'``).  emcee is not installed in this image, so two samplers provide that
move here, with emcee's chain layout (steps, walkers, ndim) and accessors:

* ``EnsembleSampler`` -- host loop around a batched log-probability (e.g.
  ``LogPosterior.log_probability_batch``, whose likelihood runs on the GPU);
  random numbers from ``numpy.random.RandomState`` in emcee's exact call order
  (``emcee_step_draws``), so for the same RandomState state it makes emcee's
  chain.
* ``DeviceEnsembleSampler`` -- the whole step on the GPU (rvk_stretch_run,
  include/rvk_post.h): proposals, priors, likelihood, acceptance and the chain
  stay in HBM.  ``rng="emcee"`` feeds it the same host-drawn stream (same chain
  as ``EnsembleSampler``); ``rng="philox"`` (default) draws on the device
  (counter-based Philox; halves [0, W/2) / [W/2, W), emcee 2's split), with no
  host work per step.
"""
from __future__ import annotations

import os

import numpy as np


def emcee_step_draws(random: np.random.RandomState, nwalkers: int):
    """One emcee step's random numbers, drawn in emcee 3.1's call order
    (RedBlueMove.propose + StretchMove.get_proposal):

        inds = arange(W) % 2; random.shuffle(inds)
        for split in (0, 1):  zz-u = random.rand(H); rint = random.randint(H, size=H);
                              acceptance u = random.rand() once per walker of the half

    Returns set[2, H] (walker indices of each half, ascending), zu[2, H],
    rint[2, H], au[2, H]."""
    W, H = nwalkers, nwalkers // 2
    all_inds = np.arange(W)
    inds = all_inds % 2
    random.shuffle(inds)
    sets = np.empty((2, H), np.int32)
    zu = np.empty((2, H))
    rint = np.empty((2, H), np.int32)
    au = np.empty((2, H))
    for split in (0, 1):
        sets[split] = all_inds[inds == split]
        zu[split] = random.rand(H)
        rint[split] = random.randint(H, size=(H,))
        au[split] = random.rand(H)            # == H successive random.rand() calls
    return sets, zu, rint, au


def _random_state(seed):
    if isinstance(seed, np.random.RandomState):
        return seed
    return np.random.RandomState(seed)


class _ChainMixin:
    def reset(self) -> None:
        self._chain, self._lnp = [], []
        self.naccepted = np.zeros(self.nwalkers, dtype=np.int64)
        self.iteration = 0

    @property
    def acceptance_fraction(self) -> np.ndarray:
        return self.naccepted / max(1, self.iteration)

    def get_chain(self, discard: int = 0, thin: int = 1, flat: bool = False) -> np.ndarray:
        ch = (np.concatenate(self._chain) if self._chain else np.zeros((0, self.nwalkers, self.ndim)))[discard::thin]
        return ch.reshape(-1, self.ndim) if flat else ch

    def get_log_prob(self, discard: int = 0, thin: int = 1, flat: bool = False) -> np.ndarray:
        lp = (np.concatenate(self._lnp) if self._lnp else np.zeros((0, self.nwalkers)))[discard::thin]
        return lp.reshape(-1) if flat else lp

    def _check_init(self, x, nwalkers, ndim):
        if x.shape != (nwalkers, ndim):
            raise ValueError(f"initial_state must have shape ({nwalkers}, {ndim})")

    @staticmethod
    def _check_init_lnp(lnp):
        if np.any(np.isnan(lnp)):
            raise ValueError("The initial log_prob was NaN")
        if not np.all(np.isfinite(lnp)):
            raise ValueError("Initial state has walkers with -inf log-probability")


class EnsembleSampler(_ChainMixin):
    def __init__(self, nwalkers: int, ndim: int, log_prob_batch, a: float = 2.0, seed=None) -> None:
        if nwalkers < 2 * ndim:
            raise ValueError(f"nwalkers ({nwalkers}) must be at least 2 * ndim ({2 * ndim})")
        if nwalkers % 2:
            raise ValueError("nwalkers must be even for the red-blue stretch move")
        self.nwalkers, self.ndim, self.a = nwalkers, ndim, float(a)
        self.log_prob_batch = log_prob_batch
        self.random = _random_state(seed)
        self.reset()

    def sample(self, initial_state, iterations: int):
        x = np.array(initial_state, dtype=np.float64, copy=True)
        self._check_init(x, self.nwalkers, self.ndim)
        lnp = np.asarray(self.log_prob_batch(x), dtype=np.float64)
        self._check_init_lnp(lnp)
        for _ in range(iterations):
            sets, zu, rint, au = emcee_step_draws(self.random, self.nwalkers)
            for split in (0, 1):
                S, Cc = sets[split], sets[1 - split]
                s, c = x[S], x[Cc]
                zz = ((self.a - 1.0) * zu[split] + 1) ** 2.0 / self.a
                factors = (self.ndim - 1.0) * np.log(zz)
                q = c[rint[split]] - (c[rint[split]] - s) * zz[:, None]
                new = np.asarray(self.log_prob_batch(q), dtype=np.float64)
                if np.any(np.isnan(new)):
                    raise ValueError("The log_prob was NaN")   # emcee: -inf rejects, NaN raises
                lnpdiff = factors + new - lnp[S]
                acc = lnpdiff > np.log(au[split])
                x[S[acc]] = q[acc]
                lnp[S[acc]] = new[acc]
                self.naccepted[S[acc]] += 1
            self.iteration += 1
            self._chain.append(x[None].copy())
            self._lnp.append(lnp[None].copy())
            yield x, lnp

    def run_mcmc(self, initial_state, nsteps: int):
        state = None
        for state in self.sample(initial_state, nsteps):
            pass
        return state


class DeviceEnsembleSampler(_ChainMixin):
    """The stretch move with every sub-step on the GPU (include/rvk_post.h rvk_stretch_run).

    ``log_posterior`` is a ``posterior.LogPosterior`` (or its ``DevicePosterior``), or a
    ``gp.GPLogPosterior`` (or its ``DeviceGPPosterior``: GPFitter.run_mcmc's sampler,
    rvk_gp_stretch_run); its priors must be built-in prior classes.  The walker state,
    the chain and the log-probabilities live in HBM; ``get_chain`` copies them to the host."""

    def __init__(self, log_posterior, nwalkers: int, a: float = 2.0, seed=None, rng: str = "philox",
                 steps_per_call: int = 256) -> None:
        import torch
        from .gp import DeviceGPPosterior, GPLogPosterior
        from .posterior import DevicePosterior
        if isinstance(log_posterior, (DevicePosterior, DeviceGPPosterior)):
            self.post = log_posterior
        elif isinstance(log_posterior, GPLogPosterior):
            self.post = DeviceGPPosterior(log_posterior)
        else:
            self.post = DevicePosterior(log_posterior)
        self._run_fn = "rvk_gp_stretch_run" if isinstance(self.post, DeviceGPPosterior) else "rvk_stretch_run"
        ndim = self.post.n_free
        if nwalkers < 2 * ndim:
            raise ValueError(f"nwalkers ({nwalkers}) must be at least 2 * ndim ({2 * ndim})")
        if nwalkers % 2 or nwalkers < 4:
            raise ValueError("nwalkers must be even (and >= 4) for the red-blue stretch move")
        if rng not in ("philox", "emcee"):
            raise ValueError("rng must be 'philox' (device) or 'emcee' (host RandomState stream)")
        self.nwalkers, self.ndim, self.a, self.rng = nwalkers, ndim, float(a), rng
        self.steps_per_call = int(steps_per_call)
        self.device = torch.device("cuda", torch.cuda.current_device())
        if rng == "emcee":
            self.random = _random_state(seed)
        else:
            self.seed = int(seed) if seed is not None else int.from_bytes(os.urandom(8), "little")
        self.post.reserve(nwalkers)
        self.reset()

    def run_mcmc(self, initial_state, nsteps: int):
        import torch
        from . import _lib
        W, D = self.nwalkers, self.ndim
        x0 = np.array(initial_state, dtype=np.float64, copy=True)
        self._check_init(x0, W, D)
        dev = self.device
        x = torch.from_numpy(x0).to(dev)
        lp = torch.empty(W, dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        self.post.device(x, lp, stream)
        self._check_init_lnp(lp.cpu().numpy())
        nacc = torch.zeros(W, dtype=torch.int64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        L = _lib.load()
        done = 0
        while done < nsteps:
            n = min(self.steps_per_call, nsteps - done)
            chain = torch.empty((n, W, D), dtype=torch.float64, device=dev)
            lnpc = torch.empty((n, W), dtype=torch.float64, device=dev)
            draws = None
            if self.rng == "emcee":
                steps = [emcee_step_draws(self.random, W) for _ in range(n)]
                draws = [torch.from_numpy(np.ascontiguousarray(np.stack([s[k] for s in steps]))).to(dev)
                         for k in range(4)]
            ptr = (lambda t: t.data_ptr()) if draws else (lambda t: 0)
            _lib.check(getattr(L, self._run_fn)(self.post._p, x.data_ptr(), lp.data_ptr(), W, n, self.a,
                                         getattr(self, "seed", 0), self.iteration + done,
                                         ptr(draws[0]) if draws else 0, ptr(draws[1]) if draws else 0,
                                         ptr(draws[2]) if draws else 0, ptr(draws[3]) if draws else 0,
                                         chain.data_ptr(), lnpc.data_ptr(), nacc.data_ptr(), status.data_ptr(),
                                         stream.cuda_stream))
            if int(status.item()):
                raise ValueError("The log_prob was NaN")
            self._chain.append(chain.cpu().numpy())
            self._lnp.append(lnpc.cpu().numpy())
            done += n
        self.iteration += nsteps
        self.naccepted += nacc.cpu().numpy()
        self.state = (x.cpu().numpy(), lp.cpu().numpy())
        return self.state
