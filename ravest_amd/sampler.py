"""Affine-invariant ensemble samplers with emcee 3.1's EnsembleSampler interface.

ravest's Fitter.run_mcmc / GPFitter.run_mcmc drive ``emcee.EnsembleSampler``
(fit.py:1068-1160, 4982-5075) with the default move, ``StretchMove(a=2)`` =
``RedBlueMove(nsplits=2, randomize_split=True)``: each step shuffles
``arange(W) % 2`` into two halves and updates each half against the other
(proposal ``c - (c - s) z``, ``z = ((a-1) u + 1)^2 / a``, acceptance
``(ndim-1) log z + lp(q) - lp(s) > log u'``).  ravest uses ``run_mcmc``,
``sample`` (its convergence loop), ``iteration``, ``get_autocorr_time(tol=0)``,
``get_chain`` and ``get_log_prob``; emcee is not installed in this image, so
two samplers provide that interface here:

* ``EnsembleSampler`` -- host loop around a batched log-probability (e.g.
  ``LogPosterior.log_probability_batch``, whose likelihood runs on the GPU);
  random numbers from ``numpy.random.RandomState`` in emcee's exact call order
  (``emcee_step_draws``), so for the same RandomState state it makes emcee's
  chain.
* ``DeviceEnsembleSampler`` -- the whole step on the GPU (rvk_stretch_run,
  include/rvk_post.h): proposals, priors, likelihood, acceptance and the chain
  stay in HBM; chunks of steps are copied to the host on a copy stream while
  the next chunk runs.  ``rng="emcee"`` feeds it the same host-drawn stream
  (same chain as ``EnsembleSampler``); ``rng="philox"`` (default) draws on the
  device (counter-based Philox, emcee 3's randomised balanced split per step),
  with no host work per step.

The chain accessors follow emcee 3.1's backend (``get_value``: rows
``[discard + thin - 1 : iteration : thin]``) and its integrated
autocorrelation time (``emcee.autocorr.integrated_time``: FFT autocovariance
per walker, averaged over walkers, Sokal's window with c = 5) is restated in
``integrated_time`` below.
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np

logger = logging.getLogger(__name__)


# ---- emcee 3.1 pieces restated (emcee/state.py, emcee/autocorr.py, emcee/ensemble.py) ------------

class State:
    """emcee.State: the walkers' coordinates and log-probabilities after a step.  Unpacks as
    ``coords, log_prob, random_state`` (emcee 3's iteration protocol, no blobs)."""
    __slots__ = ("coords", "log_prob", "blobs", "random_state")

    def __init__(self, coords, log_prob=None, blobs=None, random_state=None, copy=False) -> None:
        if isinstance(coords, State):
            coords, log_prob, blobs, random_state = coords.coords, coords.log_prob, coords.blobs, coords.random_state
        self.coords = np.array(coords, copy=True) if copy else np.atleast_2d(coords)
        self.log_prob = None if log_prob is None else (np.array(log_prob, copy=True) if copy else log_prob)
        self.blobs = blobs
        self.random_state = random_state

    def __len__(self) -> int:
        return 3 if self.blobs is None else 4

    def __iter__(self):
        if self.blobs is None:
            return iter((self.coords, self.log_prob, self.random_state))
        return iter((self.coords, self.log_prob, self.random_state, self.blobs))

    def __repr__(self) -> str:
        return f"State({self.coords}, log_prob={self.log_prob}, blobs={self.blobs}, random_state={self.random_state})"


class AutocorrError(Exception):
    """emcee.autocorr.AutocorrError: the chain is too short to estimate tau reliably."""

    def __init__(self, tau, *args, **kwargs):
        self.tau = tau
        super().__init__(*args, **kwargs)


def next_pow_two(n: int) -> int:
    i = 1
    while i < n:
        i = i << 1
    return i


def function_1d(x) -> np.ndarray:
    """Normalised autocorrelation function of a 1-D series (emcee.autocorr.function_1d)."""
    x = np.atleast_1d(x)
    if len(x.shape) != 1:
        raise ValueError("invalid dimensions for 1D autocorrelation function")
    n = next_pow_two(len(x))
    f = np.fft.fft(x - np.mean(x), n=2 * n)
    acf = np.fft.ifft(f * np.conjugate(f))[: len(x)].real
    acf /= acf[0]
    return acf


def _acf_walker_mean(x: np.ndarray, block: int = 256) -> np.ndarray:
    """Mean over walkers of function_1d of each walker's series: x [n_t, n_w] -> [n_t].  Batched
    FFTs over blocks of walkers (same arithmetic per walker as function_1d)."""
    n_t, n_w = x.shape
    n = next_pow_two(n_t)
    f = np.zeros(n_t)
    for k0 in range(0, n_w, block):
        xb = x[:, k0:k0 + block]
        F = np.fft.fft(xb - np.mean(xb, axis=0), n=2 * n, axis=0)
        acf = np.fft.ifft(F * np.conjugate(F), axis=0)[:n_t].real
        acf /= acf[0]
        for k in range(acf.shape[1]):        # emcee's order: f += acf of walker k
            f += acf[:, k]
    return f / n_w


def auto_window(taus, c) -> int:
    m = np.arange(len(taus)) < c * taus
    if np.any(m):
        return int(np.argmin(m))
    return len(taus) - 1


def integrated_time(x, c=5, tol=50, quiet=False) -> np.ndarray:
    """emcee.autocorr.integrated_time: x [n_steps, n_walkers, n_dim] (or 1-D / 2-D) -> tau [n_dim].
    Raises AutocorrError when tol * tau > n_steps unless quiet (then logs a warning); tol=0
    (ravest's call, fit.py:1131) never raises."""
    x = np.atleast_1d(x)
    if len(x.shape) == 1:
        x = x[:, np.newaxis, np.newaxis]
    if len(x.shape) == 2:
        x = x[:, :, np.newaxis]
    if len(x.shape) != 3:
        raise ValueError("invalid dimensions")
    n_t, n_w, n_d = x.shape
    tau_est = np.empty(n_d)
    windows = np.empty(n_d, dtype=int)
    for d in range(n_d):
        f = _acf_walker_mean(np.asarray(x[:, :, d], dtype=np.float64))
        taus = 2.0 * np.cumsum(f) - 1.0
        windows[d] = auto_window(taus, c)
        tau_est[d] = taus[windows[d]]
    flag = tol * tau_est > n_t
    if np.any(flag):
        msg = ("The chain is shorter than {0} times the integrated autocorrelation time for {1} parameter(s). "
               "Use this estimate with caution and run a longer chain!\n").format(tol, np.sum(flag))
        msg += "N/{0} = {1:.0f};\ntau: {2}".format(tol, n_t / tol, tau_est)
        if not quiet:
            raise AutocorrError(tau_est, msg)
        logger.warning(msg)
    return tau_est


def walkers_independent(coords) -> bool:
    """emcee.ensemble.walkers_independent: finite, no constant coordinate, and the centred,
    scaled walker matrix has condition number <= 1e8."""
    coords = np.asarray(coords, dtype=np.float64)
    if not np.all(np.isfinite(coords)):
        return False
    C = coords - np.mean(coords, axis=0)[None, :]
    C_colmax = np.amax(np.abs(C), axis=0)
    if np.any(C_colmax == 0):
        return False
    C /= C_colmax
    C_colsum = np.sqrt(np.sum(C ** 2, axis=0))
    C /= C_colsum
    return bool(np.linalg.cond(C.astype(float)) <= 1e8)


def emcee_step_draws(random: np.random.RandomState, nwalkers: int):
    """One emcee step's random numbers, drawn in emcee 3.1's call order
    (RedBlueMove.propose + StretchMove.get_proposal):

        inds = arange(W) % 2; random.shuffle(inds)
        for split in (0, 1):  zz-u = random.rand(H); rint = random.randint(H, size=H);
                              acceptance u = random.rand() once per walker of the half

    Returns set[2, H] (walker indices of each half, ascending), zu[2, H],
    rint[2, H], au[2, H] (indices as np.intp)."""
    W, H = nwalkers, nwalkers // 2
    inds = np.arange(W) % 2
    random.shuffle(inds)
    sets = np.empty((2, H), np.intp)
    zu = np.empty((2, H))
    rint = np.empty((2, H), np.intp)
    au = np.empty((2, H))
    for split in (0, 1):
        sets[split] = np.flatnonzero(inds == split)        # all_inds[inds == split]
        zu[split] = random.rand(H)
        rint[split] = random.randint(H, size=(H,))
        au[split] = random.rand(H)            # == H successive random.rand() calls
    return sets, zu, rint, au


def _host_array(shape) -> np.ndarray:
    """An fp64 host array for a chain: large ones on an anonymous mapping advised for transparent
    huge pages, so the first touch (the chunk copy-out) faults 2 MB pages, not 4 KB ones (a 58 MB
    chunk lands in ~0.5 ms instead of ~4 ms on the GPU box)."""
    n = int(np.prod(shape))
    if n * 8 < (2 << 20):
        return np.empty(shape)
    import mmap
    m = mmap.mmap(-1, n * 8, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m.madvise(mmap.MADV_HUGEPAGE)
    except (AttributeError, OSError):
        pass
    return np.frombuffer(m, dtype=np.float64, count=n).reshape(shape)


def _copy(dst: np.ndarray, src) -> None:
    """dst[...] = src with torch's multi-threaded copy (src: a host tensor or array)."""
    import torch
    if os.environ.get("RVK_HOST_COPY") == "numpy":          # experiment hook: one thread
        np.copyto(dst, src.numpy() if isinstance(src, torch.Tensor) else src)
        return
    torch.from_numpy(dst).copy_(src if isinstance(src, torch.Tensor) else torch.from_numpy(np.asarray(src)))


def _random_state(seed):
    if isinstance(seed, np.random.RandomState):
        return seed
    return np.random.RandomState(seed)


class _Backend:
    """emcee.backends.Backend (in memory): chain [n, W, D], log_prob [n, W], accepted [W] and the
    iteration count; grown ahead of a run, read through get_value's slicing."""

    def __init__(self, nwalkers: int, ndim: int) -> None:
        self.nwalkers, self.ndim = nwalkers, ndim
        self.reset()

    def reset(self) -> None:
        self.iteration = 0
        self.accepted = np.zeros(self.nwalkers, dtype=np.int64)
        self.chain = np.empty((0, self.nwalkers, self.ndim))
        self.log_prob = np.empty((0, self.nwalkers))

    def grow(self, ngrow: int) -> None:
        need = self.iteration + ngrow
        if need <= len(self.chain):
            return
        chain = _host_array((need, self.nwalkers, self.ndim))    # untouched pages cost nothing
        lnp = _host_array((need, self.nwalkers))
        if self.iteration:
            _copy(chain[:self.iteration], self.chain[:self.iteration])
            _copy(lnp[:self.iteration], self.log_prob[:self.iteration])
        self.chain, self.log_prob = chain, lnp

    def get_value(self, name: str, flat=False, thin=1, discard=0):
        if self.iteration <= 0:
            raise AttributeError("you must run the sampler with 'store == True' before accessing the results")
        v = getattr(self, name)[discard + thin - 1:self.iteration:thin]
        if flat:
            return v.reshape((-1,) + v.shape[2:])
        return v


class _DeviceBackend(_Backend):
    """The same backend with the chain and log-probabilities in device memory (HBM): the step
    kernels write each chunk straight into its rows, nothing is copied during the run, and
    ``get_value`` copies only the slice asked for.  288 GB per MI355X holds e.g. 10^5 steps of
    4096 walkers x 14 parameters (46 GB).  Grown ahead of a run (device-to-device copy)."""

    def __init__(self, nwalkers: int, ndim: int, device) -> None:
        self.device = device
        super().__init__(nwalkers, ndim)

    def reset(self) -> None:
        import torch
        self.iteration = 0
        self.accepted = np.zeros(self.nwalkers, dtype=np.int64)
        self.chain = torch.empty((0, self.nwalkers, self.ndim), dtype=torch.float64, device=self.device)
        self.log_prob = torch.empty((0, self.nwalkers), dtype=torch.float64, device=self.device)

    def grow(self, ngrow: int) -> None:
        import torch
        need = self.iteration + ngrow
        if need <= len(self.chain):
            return
        chain = torch.empty((need, self.nwalkers, self.ndim), dtype=torch.float64, device=self.device)
        lnp = torch.empty((need, self.nwalkers), dtype=torch.float64, device=self.device)
        if self.iteration:
            chain[:self.iteration].copy_(self.chain[:self.iteration])
            lnp[:self.iteration].copy_(self.log_prob[:self.iteration])
        self.chain, self.log_prob = chain, lnp

    def view(self, name: str, thin=1, discard=0):
        """The device tensor of get_value's rows (no copy)."""
        if self.iteration <= 0:
            raise AttributeError("you must run the sampler with 'store == True' before accessing the results")
        return getattr(self, name)[discard + thin - 1:self.iteration:thin]

    def get_value(self, name: str, flat=False, thin=1, discard=0):
        v = self.view(name, thin=thin, discard=discard).cpu().numpy()
        if flat:
            return v.reshape((-1,) + v.shape[2:])
        return v


class _DeviceState(State):
    """A State whose coordinates and log-probabilities stay in device memory until first read
    (the device-chain backend's rows: sample() yields one per step without a copy each)."""
    __slots__ = ("_c", "_l")

    def __init__(self, coords, log_prob, random_state=None) -> None:
        self._c, self._l = coords, log_prob
        self.blobs = None
        self.random_state = random_state

    @property
    def coords(self):
        if not isinstance(self._c, np.ndarray):
            self._c = self._c.cpu().numpy()
        return self._c

    @coords.setter
    def coords(self, v) -> None:
        self._c = v

    @property
    def log_prob(self):
        if self._l is not None and not isinstance(self._l, np.ndarray):
            self._l = self._l.cpu().numpy()
        return self._l

    @log_prob.setter
    def log_prob(self, v) -> None:
        self._l = v


def integrated_time_device(x, c=5, tol=50, quiet=False) -> np.ndarray:
    """integrated_time on a device tensor x [n_steps, n_walkers, n_dim] (the device-chain
    backend's rows): the same estimator -- per-walker autocovariance by zero-padded FFT
    (torch.fft, fp64; real transforms), averaged over walkers, Sokal's window -- without copying
    the chain to the host.  Agrees with the host restatement to rounding (tests/test_sampler.py)."""
    import torch
    if x.dim() != 3:
        raise ValueError("invalid dimensions")
    n_t, n_w, n_d = x.shape
    n = next_pow_two(n_t)
    f = torch.zeros((n_t, n_d), dtype=torch.float64, device=x.device)
    per = max(1, (1 << 30) // (2 * n * n_d * 16))      # walkers per batch: ~1 GB of spectrum
    for k0 in range(0, n_w, per):
        xb = x[:, k0:k0 + per, :]
        F = torch.fft.rfft(xb - xb.mean(dim=0, keepdim=True), n=2 * n, dim=0)
        acf = torch.fft.irfft(F.real * F.real + F.imag * F.imag, n=2 * n, dim=0)[:n_t]
        f += (acf / acf[0:1]).sum(dim=1)
    taus = (2.0 * torch.cumsum(f / n_w, dim=0) - 1.0).cpu().numpy()
    tau_est = np.empty(n_d)
    for d in range(n_d):
        tau_est[d] = taus[auto_window(taus[:, d], c), d]
    flag = tol * tau_est > n_t
    if np.any(flag):
        msg = ("The chain is shorter than {0} times the integrated autocorrelation time for {1} parameter(s). "
               "Use this estimate with caution and run a longer chain!\n").format(tol, np.sum(flag))
        msg += "N/{0} = {1:.0f};\ntau: {2}".format(tol, n_t / tol, tau_est)
        if not quiet:
            raise AutocorrError(tau_est, msg)
        logger.warning(msg)
    return tau_est


class _SamplerBase:
    """emcee.EnsembleSampler's accessors over a _Backend."""

    def reset(self) -> None:
        self.backend.reset()

    @property
    def iteration(self) -> int:
        return self.backend.iteration

    @property
    def naccepted(self) -> np.ndarray:
        return self.backend.accepted

    @property
    def acceptance_fraction(self) -> np.ndarray:
        return self.naccepted / float(self.iteration)

    def get_chain(self, flat=False, thin=1, discard=0) -> np.ndarray:
        return self.backend.get_value("chain", flat=flat, thin=thin, discard=discard)

    def get_log_prob(self, flat=False, thin=1, discard=0) -> np.ndarray:
        return self.backend.get_value("log_prob", flat=flat, thin=thin, discard=discard)

    def get_blobs(self, **kwargs):
        return None

    @property
    def chain(self) -> np.ndarray:
        return np.swapaxes(self.get_chain(), 0, 1)

    @property
    def flatchain(self) -> np.ndarray:
        return self.get_chain(flat=True)

    @property
    def lnprobability(self) -> np.ndarray:
        return np.swapaxes(self.get_log_prob(), 0, 1)

    def get_autocorr_time(self, discard=0, thin=1, **kwargs) -> np.ndarray:
        """emcee: thin * integrated_time(get_chain(discard, thin), **kwargs) (on the device for a
        device-chain backend)."""
        if isinstance(self.backend, _DeviceBackend):
            return thin * integrated_time_device(self.backend.view("chain", thin=thin, discard=discard), **kwargs)
        return thin * integrated_time(self.get_chain(discard=discard, thin=thin), **kwargs)

    def get_last_sample(self) -> State:
        it = self.iteration
        if it <= 0:
            raise AttributeError("you must run the sampler with 'store == True' before accessing the results")
        return State(self.get_chain(discard=it - 1)[0], log_prob=self.get_log_prob(discard=it - 1)[0],
                     random_state=getattr(self, "_last_random_state", None))

    def _initial(self, initial_state, log_prob0, skip_initial_state_check):
        """emcee's checks of the initial state (EnsembleSampler.sample)."""
        if initial_state is None:
            prev = getattr(self, "_previous_state", None)
            if prev is None:
                raise ValueError("Cannot have `initial_state=None` if run_mcmc has never been called.")
            return prev
        st = State(initial_state, copy=True)
        if log_prob0 is not None:
            st.log_prob = np.array(log_prob0, dtype=np.float64, copy=True)
        st.coords = np.asarray(st.coords, dtype=np.float64)
        if np.shape(st.coords) != (self.nwalkers, self.ndim):
            raise ValueError(f"incompatible input dimensions: initial_state must have shape "
                             f"({self.nwalkers}, {self.ndim})")
        if not skip_initial_state_check and not walkers_independent(st.coords):
            raise ValueError("Initial state has a large condition number. Make sure that your walkers are linearly "
                             "independent for the best performance")
        return st

    @staticmethod
    def _check_initial_log_prob(lnp) -> None:
        if np.any(np.isnan(lnp)):
            raise ValueError("The initial log_prob was NaN")

    @staticmethod
    def _unsupported(blobs0) -> None:
        if blobs0 is not None:
            raise NotImplementedError("blobs are not supported (ravest's log-probabilities have none)")

    @staticmethod
    def _thinning(iterations, thin_by, thin):
        """emcee 3.1's thinning arguments -> (raw steps per yielded step, raw steps per stored step,
        rows stored): ``thin_by=k`` runs k steps per yielded step and stores every k-th; the
        deprecated ``thin=k`` yields every step and stores every k-th (iterations // k rows)."""
        if thin is not None:
            import warnings
            warnings.warn("The 'thin' argument is deprecated. Use 'thin_by' instead.", DeprecationWarning)
            thin = int(thin)
            if thin <= 0:
                raise ValueError("Invalid thinning argument")
            return 1, thin, int(iterations) // thin
        thin_by = int(thin_by)
        if thin_by <= 0:
            raise ValueError("Invalid thinning argument")
        return thin_by, thin_by, int(iterations)

    def run_mcmc(self, initial_state, nsteps: int, **kwargs):
        """emcee: iterate sample() for nsteps steps; returns the last State."""
        results = None
        for results in self.sample(initial_state, iterations=nsteps, **kwargs):
            pass
        return results


def _progress_bar(progress, total):
    if not progress:
        return None
    try:
        import tqdm
    except ImportError:
        return None
    return tqdm.tqdm(total=total, **(progress if isinstance(progress, dict) else {}))


class EnsembleSampler(_SamplerBase):
    """emcee's stretch move on the host over a batched log-probability (``vectorize=True`` form:
    ``log_prob_batch([W/2, D]) -> [W/2]``), emcee's RandomState call order."""

    def __init__(self, nwalkers: int, ndim: int, log_prob_batch, a: float = 2.0, seed=None) -> None:
        if nwalkers < 2 * ndim:
            raise ValueError(f"nwalkers ({nwalkers}) must be at least 2 * ndim ({2 * ndim})")
        if nwalkers % 2:
            raise ValueError("nwalkers must be even for the red-blue stretch move")
        self.nwalkers, self.ndim, self.a = nwalkers, ndim, float(a)
        self.log_prob_batch = log_prob_batch
        self.random = _random_state(seed)
        self.backend = _Backend(nwalkers, ndim)
        self._previous_state = None

    @property
    def random_state(self):
        return self.random.get_state()

    def sample(self, initial_state=None, log_prob0=None, rstate0=None, blobs0=None, iterations=1, tune=False,
               skip_initial_state_check=False, thin_by=1, thin=None, store=True, progress=False, progress_kwargs=None):
        """emcee 3.1's EnsembleSampler.sample, including its thinning: ``thin_by=k`` runs k steps per
        yielded step and stores every k-th; the deprecated ``thin=k`` runs ``iterations`` steps,
        yields each and stores every k-th (iterations // k rows).  As in emcee, only the stored
        steps' acceptances are counted (backend.save_step)."""
        if blobs0 is not None:
            raise NotImplementedError("blobs are not supported (ravest's log-probabilities have none)")
        if thin is not None:
            import warnings
            warnings.warn("The 'thin' argument is deprecated. Use 'thin_by' instead.", DeprecationWarning)
            thin = int(thin)
            if thin <= 0:
                raise ValueError("Invalid thinning argument")
            yield_step, checkpoint, nsaves = 1, thin, int(iterations) // thin
        else:
            thin_by = int(thin_by)
            if thin_by <= 0:
                raise ValueError("Invalid thinning argument")
            yield_step, checkpoint, nsaves = thin_by, thin_by, int(iterations)
        iterations = int(iterations)
        st = self._initial(initial_state, log_prob0, skip_initial_state_check)
        if rstate0 is not None:
            self.random.set_state(rstate0)
        x = np.array(st.coords, dtype=np.float64, copy=True)
        lnp = (np.asarray(self.log_prob_batch(x), dtype=np.float64) if st.log_prob is None
               else np.array(st.log_prob, dtype=np.float64, copy=True))
        self._check_initial_log_prob(lnp)
        if store:
            self.backend.grow(nsaves)
        bar = _progress_bar(progress, iterations * yield_step)
        a, nd1, b = self.a, self.ndim - 1.0, self.backend
        # emcee keeps ONE State, updates its coordinates and log-probabilities in place and yields
        # it every step (EnsembleSampler.sample); so do we (no per-step copies of the ensemble)
        state = State(x, log_prob=lnp)
        for i in range(iterations * yield_step):
            sets, zu, rint, au = emcee_step_draws(self.random, self.nwalkers)
            accepted = np.zeros(self.nwalkers, dtype=bool)
            for split in (0, 1):                               # np.take / np.compress: the same
                S = sets[split]                                # rows as fancy indexing, ~3x faster
                s = np.take(x, S, axis=0)
                cr = np.take(x, np.take(sets[1 - split], rint[split]), axis=0)   # c[rint] (get_proposal)
                zz = ((a - 1.0) * zu[split] + 1) ** 2.0 / a
                factors = nd1 * np.log(zz)
                q = cr - (cr - s) * zz[:, None]
                new = np.asarray(self.log_prob_batch(q), dtype=np.float64)
                if np.isnan(new).any():
                    raise ValueError("Probability function returned NaN")   # emcee: -inf rejects, NaN raises
                acc = factors + new - np.take(lnp, S) > np.log(au[split])
                Sa = np.compress(acc, S)
                x[Sa] = np.compress(acc, q, axis=0)
                lnp[Sa] = np.compress(acc, new)
                accepted[Sa] = True
            if store and (i + 1) % checkpoint == 0:           # emcee's backend.save_step
                b.chain[b.iteration] = x
                b.log_prob[b.iteration] = lnp
                b.accepted += accepted
                b.iteration += 1
            state.random_state = self.random.get_state()
            self._previous_state = state
            if bar is not None:
                bar.update(1)
            if (i + 1) % yield_step == 0:
                yield state
        if bar is not None:
            bar.close()


class _Chunk:
    """One chunk of device steps in flight: where it starts, its copy-out slot and events, and what
    its sampler needs to resume exactly at any step inside it."""
    __slots__ = ("start", "n", "slot", "copied", "bufs", "x0", "lp0", "nacc0", "draws", "rstate0", "row0", "store")


class _DevicePipeline(_SamplerBase):
    """emcee's EnsembleSampler.sample over chunks of device steps.  The walker state, the draws and
    each chunk's chain stay in device memory.  Chain storage "device" (the default on a GPU): the
    chunk's kernels write into the device backend's rows and nothing is copied during the run
    (get_chain copies what it returns; get_autocorr_time runs on the device).  "host": a finished
    chunk is copied to pinned host memory on a copy stream while the next chunk runs, then into
    the backend's host arrays.  Either way the chunk's steps are yielded one by one.  Subclasses
    provide the steps (_run_chunk), what a chunk must record to be resumed inside (_begin_chunk)
    and the rewind to a step inside the last chunks (_settle, naccepted)."""

    def _pipeline_init(self, device, keep_host: bool = True, chain_storage: str = "auto") -> None:
        import torch
        if chain_storage not in ("auto", "device", "host"):
            raise ValueError("chain_storage must be 'auto', 'device' or 'host'")
        self.device = device
        self.chain_storage_requested = chain_storage
        self._dev_chain = chain_storage == "device" or (chain_storage == "auto" and device.type == "cuda")
        self.chain_storage = "device" if self._dev_chain else "host"
        self.backend = _DeviceBackend(self.nwalkers, self.ndim, device) if self._dev_chain else \
            _Backend(self.nwalkers, self.ndim)
        self._keep_host = keep_host          # copy the chain to this process's host memory
        self._token = 0
        self._x = self._lp = None            # device state, at step self._dev_iter
        self._nacc = torch.zeros(self.nwalkers, dtype=torch.int64, device=device)
        self._nacc_tmp = None                # acceptance counts of unstored steps (discarded, as emcee does)
        self._status = torch.zeros(1, dtype=torch.int32, device=device)
        # Step positions: _pos = steps the consumer has taken (stored or not), _dev_iter = steps the
        # device state has taken (up to one chunk ahead).  The draws of a step are keyed by its
        # position, which reset() does not rewind (emcee's RandomState goes on after reset too);
        # backend.iteration counts STORED steps only (emcee's save_step).
        self._pos = 0
        self._dev_iter = 0
        self._chunks = []                    # the last chunks (the committed step lies in them)
        self._dbuf = [None, None]            # device chain / log-prob buffers, per slot
        self._stage = [None, None]           # pinned host staging, per slot
        self._stage_status = [None, None]    # pinned status word, per slot
        self._copy_stream = None
        self._nslot = 0
        self._accepted_pos = 0               # backend.accepted is exact at this position
        self._trace = [] if os.environ.get("RVK_SAMPLER_TRACE") else None   # (phase, perf_counter) timing probe

    @property
    def _cuda(self) -> bool:
        return self.device.type == "cuda"

    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.device) if self._cuda else None

    def _device_chain_fits(self, iterations: int) -> bool:
        """Whether growing the device chain by `iterations` steps leaves headroom in device memory
        (chain_storage="auto" only: an explicit "device" is honoured and may raise out of memory)."""
        import torch
        if self.chain_storage_requested != "auto" or not self._cuda:
            return True
        b = self.backend
        need = max(0, b.iteration + iterations - len(b.chain)) * self.nwalkers * (self.ndim + 1) * 8
        if need == 0:
            return True
        free, _ = torch.cuda.mem_get_info(self.device)
        return need + b.iteration * self.nwalkers * (self.ndim + 1) * 8 <= 0.8 * free

    def _chain_to_host(self) -> None:
        """Move the chain to a host backend (the run goes on with chunked copy-out)."""
        old = self.backend
        logger.warning("the chain no longer fits in device memory: keeping it in host memory from step %d",
                       old.iteration)
        new = _Backend(self.nwalkers, self.ndim)
        new.grow(old.iteration)
        if old.iteration:
            _copy(new.chain[:old.iteration], old.chain[:old.iteration].cpu())
            _copy(new.log_prob[:old.iteration], old.log_prob[:old.iteration].cpu())
        new.iteration, new.accepted = old.iteration, old.accepted
        self.backend = new
        self._dev_chain = False
        self.chain_storage = "host"

    def _ensure_buffers(self, slot: int, chunk_bufs: bool = True) -> None:
        """The slot's status word; chunk_bufs: also its device chunk buffers and pinned staging."""
        import torch
        if self._stage_status[slot] is None:
            self._stage_status[slot] = (torch.empty(1, dtype=torch.int32, pin_memory=True) if self._cuda
                                        else self._status.clone())
        if self._cuda and self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device, priority=int(os.environ.get("RVK_COPY_PRIO", "0")))
        if self._dbuf[slot] is not None or not chunk_bufs:
            return
        n, W, D = self.steps_per_call, self.nwalkers, self.ndim
        self._dbuf[slot] = (torch.empty((n, W, D), dtype=torch.float64, device=self.device),
                            torch.empty((n, W), dtype=torch.float64, device=self.device))
        if self._cuda:
            pin = dict(pin_memory=True)
            self._stage[slot] = (torch.empty((n, W, D), dtype=torch.float64, **pin) if self._keep_host else None,
                                 torch.empty((n, W), dtype=torch.float64, **pin) if self._keep_host else None,
                                 None)
        else:                                 # host tensors: the device buffers are the staging
            self._stage[slot] = (self._dbuf[slot][0], self._dbuf[slot][1], None)

    def reset(self) -> None:
        self.backend.reset()
        self._x = self._lp = None
        self._nacc.zero_()
        self._dev_iter = self._pos
        self._chunks = []
        self._accepted_pos = self._pos
        self._token += 1

    def _set_state(self, st: State) -> None:
        import torch
        self._x = torch.from_numpy(np.ascontiguousarray(st.coords, dtype=np.float64)).to(self.device)
        self._lp = torch.empty(self.nwalkers, dtype=torch.float64, device=self.device)
        if st.log_prob is None:
            self._initial_log_prob(self._x, self._lp)
        else:
            self._lp.copy_(torch.from_numpy(np.ascontiguousarray(st.log_prob, dtype=np.float64)))
        self._check_initial_log_prob(self._lp.cpu().numpy())
        self._dev_iter = self._pos
        self._x_init = (self._dev_iter, self._x.clone(), self._lp.clone(), self._nacc.clone())
        self._chunks = []

    def _enqueue(self, n: int, dev_store: bool = False, store: bool = True) -> _Chunk:
        """Launch the next n steps.  dev_store: into the device backend's rows (no copy-out);
        store: emcee's flag -- the steps count (iteration, acceptance counts; backend rows on the
        ranks that keep the chain)."""
        import torch
        stream = self._stream()
        slot = self._nslot % 2
        self._nslot += 1
        self._ensure_buffers(slot, chunk_bufs=not dev_store)
        prev = next((c for c in reversed(self._chunks) if c.slot == slot), None)
        if prev is not None and prev.copied is not None:
            stream.wait_event(prev.copied)    # the slot's device buffers were being copied out
        ch = _Chunk()
        ch.start, ch.n, ch.slot, ch.copied = self._dev_iter, n, slot, None
        ch.store = store
        # backend row of the chunk's first step: rows follow the committed position
        ch.row0 = self.backend.iteration + (self._dev_iter - self._pos) if store else None
        if self._trace is not None:
            self._trace.append(("enqueue", time.perf_counter()))
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        self._begin_chunk(ch)
        if dev_store:
            b = self.backend
            chain_d, lnp_d = b.chain[ch.row0:ch.row0 + n], b.log_prob[ch.row0:ch.row0 + n]
        else:
            chain_d, lnp_d = self._dbuf[slot]
        ch.bufs = (chain_d, lnp_d)
        if self._trace is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(stream)
        self._run_chunk(ch, chain_d, lnp_d, stream)
        if self._trace is not None:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record(stream)
            self._trace.append(("launched", time.perf_counter()))
            self._gpu_trace = getattr(self, "_gpu_trace", []) + [(e0, e1, e2)]
        self._dev_iter += n
        if self._cuda:
            computed = torch.cuda.Event()
            computed.record(stream)
            cs = self._copy_stream
            cs.wait_event(computed)
            sc, sl, _ = self._stage[slot] if not dev_store else (None,) * 3
            wg = int(os.environ.get("RVK_EGRESS_WG", "0"))   # experiment hook: copy with a few workgroups
            if self._keep_host and wg and sc is not None:
                from . import _lib
                L = _lib.load()
                _lib.check(L.rvk_copy_to_host(chain_d.data_ptr(), sc.data_ptr(), n * chain_d[0].numel() * 8, wg,
                                              cs.cuda_stream))
                _lib.check(L.rvk_copy_to_host(lnp_d.data_ptr(), sl.data_ptr(), n * lnp_d[0].numel() * 8, wg,
                                              cs.cuda_stream))
            if os.environ.get("RVK_NO_EGRESS"):   # experiment hook: no chain copy-out (timing only)
                sc = None
            ss = self._stage_status[slot]
            with torch.cuda.stream(cs):
                if self._keep_host and not wg and sc is not None:
                    sc[:n].copy_(chain_d[:n], non_blocking=True)
                    sl[:n].copy_(lnp_d[:n], non_blocking=True)
                ss.copy_(self._status, non_blocking=True)
            ch.copied = torch.cuda.Event()
            ch.copied.record(cs)
        else:                                 # host tensors: the chunk's status as it ended
            if not dev_store:
                self._stage[slot] = (chain_d, lnp_d, None)
            self._stage_status[slot] = self._status.clone()
        self._chunks = (self._chunks + [ch])[-3:]
        return ch

    def run_mcmc(self, initial_state, nsteps: int, **kwargs):
        """emcee's run_mcmc (iterates sample, returns the last State), without a Python object per step."""
        results = None
        for results in self.sample(initial_state, iterations=nsteps, _per_step=False, **kwargs):
            pass
        return results

    def sample(self, initial_state=None, log_prob0=None, rstate0=None, blobs0=None, iterations=1, tune=False,
               skip_initial_state_check=False, thin_by=1, thin=None, store=True, progress=False, progress_kwargs=None,
               _per_step=True):
        """emcee's EnsembleSampler.sample: yields a State per step (``iteration`` counts the stored
        ones).  Thinning as emcee 3.1 (``thin_by=k``: k steps per yielded step, every k-th stored;
        the deprecated ``thin=k``: every step yielded, every k-th stored), with emcee's accounting:
        only the stored steps' acceptances count (backend.save_step).  The steps between two stored
        ones run as unstored device steps (their acceptances go to a scratch counter); a stored step
        is one device step into the backend's next row.  The draws are keyed by the global step, so
        a thinned run is the unthinned chain's every k-th row, bit for bit."""
        self._unsupported(blobs0)
        if thin is None and int(thin_by) == 1:
            yield from self._sample_steps(initial_state, log_prob0, rstate0, iterations, skip_initial_state_check,
                                          store, progress, _per_step)
            return
        yield_step, checkpoint, nsaves = self._thinning(iterations, thin_by, thin)
        total = int(iterations) * yield_step
        if store and self._keep_host:                # the rows of the whole run at once (not one per save)
            self._settle()
            if self._dev_chain and not self._device_chain_fits(nsaves):
                self._chain_to_host()
            self.backend.grow(nsaves)
        start = dict(initial_state=initial_state, log_prob0=log_prob0, rstate0=rstate0,
                     skip_initial_state_check=skip_initial_state_check)
        bar = _progress_bar(progress, total)
        i, last = 0, None
        while i < total:
            # raw steps up to the next stored step (checkpoint) or the run's end
            ck = min((i // checkpoint + 1) * checkpoint, total)
            stored = store and ck % checkpoint == 0
            n_plain = ck - i - (1 if stored else 0)
            for part_store, n in ((False, n_plain), (store, 1 if stored else 0)):
                if n <= 0:
                    continue
                per = _per_step and yield_step == 1          # thin=k yields every raw step
                for st in self._sample_steps(iterations=n, store=part_store, _per_step=per, **start):
                    start = {}
                    last = st
                    if per:
                        yield st
                i += n
                if bar is not None:
                    bar.update(n)
                if not per and _per_step and i % yield_step == 0:
                    yield last
        if bar is not None:
            bar.close()
        if not _per_step and last is not None:
            yield last

    def _sample_steps(self, initial_state=None, log_prob0=None, rstate0=None, iterations=1,
                      skip_initial_state_check=False, store=True, progress=False, _per_step=True):
        """sample() without thinning: every device step is yielded (and stored when `store`)."""
        self._settle()
        self._token += 1
        tok = self._token
        if initial_state is None:
            if self._x is None:
                raise ValueError("Cannot have `initial_state=None` if run_mcmc has never been called.")
        else:
            st = self._initial(initial_state, log_prob0, skip_initial_state_check)
            if rstate0 is not None and getattr(self, "rng", None) == "emcee":
                self.random.set_state(rstate0)
            self._set_state(st)
        # store (emcee's flag) decides what COUNTS -- iteration and the acceptance counts advance on
        # every rank alike, so ravest's convergence loop (fit.py:1123-1131) runs the same collective
        # calls everywhere; keep decides whether this process also writes the chain rows
        # (keep_chain of the sharded sampler: the other ranks count steps but hold no rows).
        keep = store and self._keep_host
        if keep and self._dev_chain and not self._device_chain_fits(iterations):
            self._chain_to_host()
        dev_store = keep and self._dev_chain
        if keep:
            self.backend.grow(iterations)
        bar = _progress_bar(progress, iterations)
        done, pending = 0, None
        while True:
            nxt = None
            if done < iterations:
                nxt = self._enqueue(min(self.steps_per_call, iterations - done), dev_store, store)
                done += nxt.n
            if pending is not None:
                if pending.copied is not None:
                    pending.copied.synchronize()
                if self._trace is not None:
                    self._trace.append(("copied", time.perf_counter()))
                sc, sl = (None, None) if dev_store else self._stage[pending.slot][:2]
                ss = self._stage_status[pending.slot]
                if int(ss[0]):
                    self._status.zero_()
                    raise ValueError("Probability function returned NaN")
                b = self.backend
                a, e = pending.row0, (pending.row0 or 0) + pending.n     # backend rows (store only)
                if keep and not dev_store:    # multi-threaded copy out of the pinned staging
                    _copy(b.chain[a:e], sc[:pending.n])
                    _copy(b.log_prob[a:e], sl[:pending.n])
                if self._trace is not None:
                    self._trace.append(("stored", time.perf_counter()))
                if not _per_step:             # run_mcmc: the chunk's last state only
                    if tok != self._token:
                        raise RuntimeError("this run was superseded by a later sample()/run_mcmc()/reset() call")
                    self._pos = pending.start + pending.n
                    if store:
                        b.iteration = e
                    if bar is not None:
                        bar.update(pending.n)
                    yield (_DeviceState(b.chain[e - 1], b.log_prob[e - 1]) if dev_store else
                           State(b.chain[e - 1], log_prob=b.log_prob[e - 1]) if keep else
                           State(sc[pending.n - 1].numpy(), log_prob=sl[pending.n - 1].numpy(), copy=True)
                           if sc is not None else State(np.empty((0, self.ndim))))
                    if nxt is None:
                        break
                    pending = nxt
                    continue
                for i in range(pending.n):
                    if tok != self._token:
                        raise RuntimeError("this sample() generator was superseded by a later sample()/run_mcmc()/"
                                           "reset() call")
                    t = (a or 0) + i
                    self._pos = pending.start + i + 1
                    if store:
                        b.iteration = t + 1
                    if dev_store:
                        state = _DeviceState(b.chain[t], b.log_prob[t])
                    elif keep:
                        state = State(b.chain[t], log_prob=b.log_prob[t])
                    elif sc is not None:
                        state = State(sc[i].numpy(), log_prob=sl[i].numpy(), copy=True)
                    else:
                        state = State(np.empty((0, self.ndim)))   # this rank keeps no chain
                    if bar is not None:
                        bar.update(1)
                    yield state
            if nxt is None:
                break
            pending = nxt
        if bar is not None:
            bar.close()


class DeviceEnsembleSampler(_DevicePipeline):
    """The stretch move with every sub-step on the GPU (include/rvk_post.h rvk_stretch_run).

    ``log_posterior`` is a ``posterior.LogPosterior`` (or its ``DevicePosterior``), or a
    ``gp.GPLogPosterior`` (or its ``DeviceGPPosterior``: GPFitter.run_mcmc's sampler,
    rvk_gp_stretch_run); its priors must be built-in prior classes.  emcee 3.1's interface
    (``sample``, ``run_mcmc``, ``iteration``, ``get_chain``, ``get_log_prob``,
    ``get_autocorr_time``, ``acceptance_fraction``, ``get_last_sample``).

    Steps run in chunks of ``steps_per_call`` on the device (state and draws in HBM).
    ``chain_storage="auto"``/``"device"``: the chain is kept in HBM, written there by the step
    kernels with no copy during the run (``get_chain`` copies what it returns,
    ``get_autocorr_time`` runs on the device); ``"host"``: each finished chunk is copied to pinned
    host memory on a copy stream while the next chunk runs.  ``sample`` yields the steps one by
    one.  A consumer that stops early (ravest's
    convergence break) leaves the device up to one chunk ahead: the next call (and
    ``naccepted``) replays the chunk from its start up to ``iteration`` -- the draws depend only
    on (seed, global step), so the replay is exact and a run split over several calls is the
    same chain as one call.  A NaN log-probability raises ValueError at the chunk it occurs in,
    before any of that chunk's steps is yielded (emcee raises at the step)."""

    def __init__(self, log_posterior, nwalkers: int, a: float = 2.0, seed=None, rng: str = "philox",
                 steps_per_call: int = 256, randomize_split: bool = True, chain_storage: str = "auto") -> None:
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
        self.randomize_split = bool(randomize_split)
        self.steps_per_call = max(1, int(steps_per_call))
        if rng == "emcee":
            self.random = _random_state(seed)
            if not self.randomize_split:
                raise ValueError("rng='emcee' draws emcee's randomised split; randomize_split=False needs rng='philox'")
        else:
            self.seed = int(seed) if seed is not None else int.from_bytes(os.urandom(8), "little")
        self.post.reserve(nwalkers)
        self._pipeline_init(torch.device("cuda", torch.cuda.current_device()), chain_storage=chain_storage)

    def _flags(self) -> int:
        from . import _lib
        return 0 if self.randomize_split else _lib.STRETCH_FIXED_SPLIT

    def _initial_log_prob(self, x, lp) -> None:
        self.post.device(x, lp, self._stream())

    def _host_draws(self, n: int):
        import torch
        steps = [emcee_step_draws(self.random, self.nwalkers) for _ in range(n)]
        dt = (np.int32, np.float64, np.int32, np.float64)     # include/rvk_post.h d_set, d_zu, d_rint, d_au
        return [torch.from_numpy(np.ascontiguousarray(np.stack([s[k] for s in steps]), dtype=dt[k])).to(self.device)
                for k in range(4)]

    def _launch(self, x, lp, nacc, n, step0, draws, chain_d, lnp_d, stream) -> None:
        from . import _lib
        L = _lib.load()
        d = [t.data_ptr() for t in draws] if draws else [0, 0, 0, 0]
        _lib.check(getattr(L, self._run_fn)(self.post._p, x.data_ptr(), lp.data_ptr(), self.nwalkers, n, self.a,
                                            getattr(self, "seed", 0), step0, self._flags(), d[0], d[1], d[2], d[3],
                                            0 if chain_d is None else chain_d.data_ptr(),
                                            0 if lnp_d is None else lnp_d.data_ptr(), nacc.data_ptr(),
                                            self._status.data_ptr(), stream.cuda_stream))

    def _begin_chunk(self, ch: _Chunk) -> None:
        ch.x0, ch.lp0, ch.nacc0 = self._x.clone(), self._lp.clone(), self._nacc.clone()
        ch.rstate0 = self.random.get_state() if self.rng == "emcee" else None
        ch.draws = self._host_draws(ch.n) if self.rng == "emcee" else None

    def _run_chunk(self, ch: _Chunk, chain_d, lnp_d, stream) -> None:
        nacc = self._nacc
        if not ch.store:                      # emcee counts the acceptances of stored steps only
            if self._nacc_tmp is None:
                self._nacc_tmp = self._nacc.clone()
            nacc = self._nacc_tmp
        self._launch(self._x, self._lp, nacc, ch.n, ch.start, ch.draws, chain_d, lnp_d, stream)

    def _replay_to(self, target: int, x, lp, nacc) -> None:
        """Device state of step `target` into (x, lp, nacc): from the start of the chunk that
        holds it, replay the chunk's first target - start steps (same draws)."""
        ch = next((c for c in self._chunks if c.start <= target <= c.start + c.n), None)
        if ch is None:
            raise RuntimeError("internal: no chunk record covers the requested step")
        x.copy_(ch.x0)
        lp.copy_(ch.lp0)
        nacc.copy_(ch.nacc0)
        k = target - ch.start
        if k:
            draws = [t[:k] for t in ch.draws] if ch.draws else None
            self._launch(x, lp, nacc, k, ch.start, draws, None, None, self._stream())
            if not ch.store:
                nacc.copy_(ch.nacc0)

    def _settle(self) -> None:
        """Bring the device state back to the consumer's position after a generator stopped early."""
        if self._x is None or self._dev_iter == self._pos:
            return
        self._replay_to(self._pos, self._x, self._lp, self._nacc)
        if self.rng == "emcee":
            ch = next(c for c in self._chunks if c.start <= self._pos <= c.start + c.n)
            self.random.set_state(ch.rstate0)
            for _ in range(self._pos - ch.start):
                emcee_step_draws(self.random, self.nwalkers)
        self._dev_iter = self._pos
        self._chunks = []
        self.backend.accepted = self._nacc.cpu().numpy()
        self._accepted_pos = self._pos

    @property
    def naccepted(self) -> np.ndarray:
        if self._accepted_pos != self._pos:
            if self._dev_iter == self._pos:
                self.backend.accepted = self._nacc.cpu().numpy()
            else:                             # a generator is suspended inside a chunk: replay on scratch
                import torch
                x, lp, nacc = torch.empty_like(self._x), torch.empty_like(self._lp), torch.empty_like(self._nacc)
                self._replay_to(self._pos, x, lp, nacc)
                self.backend.accepted = nacc.cpu().numpy()
            self._accepted_pos = self._pos
        return self.backend.accepted
