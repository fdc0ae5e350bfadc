"""LogPosterior / LogLikelihood / LogPrior: drop-in mirrors of ravest.fit's.

Same constructor arguments, same per-walker semantics and error behaviour as
src/ravest/fit.py:3228-3691, so emcee, MAP and ravest's Fitter can use them
unchanged.  The difference is the engine underneath: the likelihood of every
walker is computed by the HIP kernel behind include/rvk.h (RVEngine), and the
host-side work (free -> full parameter scatter, jitter check, priors, prior
conversion, corrections) is vectorised over a whole walker block.

Entry points:
  * ``log_probability(free_params_dict) -> float``  -- the reference's scalar
    log_prob_fn (emcee with ``parameter_names``; MAP; single-point callers);
  * ``log_probability_batch(theta_free[W, D]) -> ndarray[W]`` -- the
    vectorised drop-in (emcee ``vectorize=True``); ``__call__`` is the same.
Both route through the device log-posterior (``DevicePosterior``: the scatter,
jitter check, conversion, priors, likelihood and corrections in one kernel,
one host round trip) whenever every prior is one of ravest's built-in classes;
a custom callable prior keeps the host-side prior path (``route="host"``).
Mask semantics follow fit.py:3461-3495 exactly: jitter < 0, a prior-side
conversion ValueError, a non-finite log-prior, or an invalid planet give -inf.
"""
from __future__ import annotations

import ctypes as C
import logging
import weakref
from typing import Callable, Dict

import numpy as np

from . import _lib
from .param import Parameterisation, as_parameterisation, full_param_names
from .prior import Uniform, is_builtin, as_priors, device_params, logpdf_vec


class LogLikelihood:
    """fit.py:3529-3660.  ``__call__(params: dict) -> float`` over ALL parameters."""

    def __init__(self, time, vel, velerr, instrument, unique_instruments, t0, planet_letters,
                 parameterisation: Parameterisation, engine=None, device: int = -1) -> None:
        self.time = time
        self.vel = vel
        self.velerr = velerr
        self.instrument = instrument
        self.unique_instruments = unique_instruments
        self.t0 = t0
        self.planet_letters = planet_letters
        self.parameterisation = as_parameterisation(parameterisation)
        # fit.py:3585-3598
        _inst_to_idx = {inst: i for i, inst in enumerate(self.unique_instruments)}
        self._instrument_indices = np.array([_inst_to_idx[inst] for inst in self.instrument], dtype=np.int32)
        self._gamma_keys = [f"g_{inst}" for inst in self.unique_instruments]
        self._jitter_keys = [f"jit_{inst}" for inst in self.unique_instruments]
        self._log_2pi = np.log(2 * np.pi)
        self._velerr_sq = np.asarray(self.velerr) ** 2
        self.names = full_param_names(planet_letters, parameterisation, list(unique_instruments))
        self._engine = engine
        self._device = device

    @property
    def engine(self):
        if self._engine is None:
            from .engine import RVEngine
            self._engine = RVEngine(self.time, self.vel, self.velerr, self._instrument_indices,
                                    len(self.unique_instruments), len(self.planet_letters),
                                    self.parameterisation, self.t0, device=self._device)
        return self._engine

    def __getstate__(self):           # picklable (multiprocessing pools), engine rebuilt lazily
        d = dict(self.__dict__)
        d["_engine"] = None
        return d

    def batch(self, theta_full: np.ndarray) -> np.ndarray:
        """[W, P_full] in ``self.names`` order -> [W] log-likelihoods."""
        return self.engine.loglike(theta_full)

    def __call__(self, params: Dict[str, float]) -> float:
        row = np.array([[params[n] for n in self.names]], dtype=np.float64)
        return float(self.batch(row)[0])


class LogPrior:
    """fit.py:3663-3691."""

    def __init__(self, priors: dict) -> None:
        self.priors = priors                  # the caller's objects: the scalar path calls them
        self._vec = as_priors(priors)         # ravest's built-ins re-expressed for the batch path

    def __call__(self, params: Dict[str, float]) -> float:
        log_prior_probability = 0
        for param in params:
            log_prior_probability += self.priors[param](params[param])
        return log_prior_probability

    def batch(self, cols: Dict[str, np.ndarray]) -> np.ndarray:
        """Same sum, same key order, vectorised over walkers."""
        lp = 0
        for param, col in cols.items():
            lp = lp + logpdf_vec(self._vec[param], col)
        return lp


class LogPosterior:
    """fit.py:3228-3526."""

    def __init__(self, planet_letters: list, parameterisation: Parameterisation, priors: dict,
                 fixed_params: dict, free_params_names: list, time, vel, velerr, instrument,
                 unique_instruments, t0: float, engine=None, device: int = -1, route: str = "auto") -> None:
        self.planet_letters = planet_letters
        self.parameterisation = as_parameterisation(parameterisation)   # ravest's own object accepted
        self.priors = priors
        self._priors = as_priors(priors)      # ravest's prior objects accepted (prior.as_prior)
        self.fixed_params = fixed_params
        self.free_params_names = free_params_names
        self.time = time
        self.vel = vel
        self.velerr = velerr
        self.instrument = instrument
        self.unique_instruments = unique_instruments
        self.t0 = t0
        self.log_likelihood = LogLikelihood(time=time, vel=vel, velerr=velerr, instrument=instrument,
                                            unique_instruments=unique_instruments, t0=t0,
                                            planet_letters=planet_letters, parameterisation=self.parameterisation,
                                            engine=engine, device=device)
        self.log_prior = LogPrior(self.priors)
        (self._logprob_jacobian_correction, self._logprob_prior_renorm_correction,
         self._logprob_correction_breakdown) = self._compute_logprob_corrections()
        self._build_plan()
        if route not in ("auto", "device", "host"):
            raise ValueError("route must be 'auto', 'device' or 'host'")
        # "auto": the device log-posterior when every prior has a device form and the likelihood
        # engine is this package's (not a caller-supplied stand-in); "host": priors on the host
        self._route = route
        self._dpost = None

    # ---- constant corrections: fit.py:3306-3397 ------------------------------------------
    def _classify_planet_case(self, letter: str) -> str:
        if self.parameterisation.log_jacobian_determinant() == 0.0:
            return "CASE_1"
        if f"secosw_{letter}" not in self.free_params_names:
            return "CASE_1"
        secosw_key, sesinw_key = f"secosw_{letter}", f"sesinw_{letter}"
        e_key, w_key = f"e_{letter}", f"w_{letter}"
        if secosw_key in self.priors and sesinw_key in self.priors:
            sp, vp = self._priors[secosw_key], self._priors[sesinw_key]
            if (isinstance(sp, Uniform) and isinstance(vp, Uniform) and sp.lower == -1 and sp.upper == 1
                    and vp.lower == -1 and vp.upper == 1):
                return "CASE_2"
            raise NotImplementedError(
                f"Unsupported priors on (secosw_{letter}, sesinw_{letter}): {sp!r}, {vp!r}. Only Uniform(-1, 1) "
                "priors on (secosw, sesinw) are supported for evidence-correct log-posterior corrections. A "
                "separable, rotationally-symmetric belief about eccentricity can always be re-expressed as a "
                f"prior on e instead - place priors on (e_{letter}, w_{letter}) using one of Ravest's "
                "eccentricity priors (HalfNormal, Rayleigh, VanEylen19Mixture, Beta, EccentricityUniform, "
                "TruncatedNormal).")
        elif e_key in self.priors and w_key in self.priors:
            return "CASE_3"
        raise RuntimeError(f"Could not classify log-posterior correction case for planet '{letter}': no priors "
                           "found on either (secosw, sesinw) or (e, w).")

    def _compute_logprob_corrections(self):
        log_jac = self.parameterisation.log_jacobian_determinant()
        total_jacobian, total_renorm, breakdown = 0.0, 0.0, {}
        for letter in self.planet_letters:
            case = self._classify_planet_case(letter)
            jacobian = log_jac if case == "CASE_3" else 0.0
            renorm = np.log(4.0 / np.pi) if case == "CASE_2" else 0.0
            total_jacobian += jacobian
            total_renorm += renorm
            breakdown[letter] = {"case": case, "jacobian": jacobian, "renorm": renorm}
            logging.info(f"Planet {letter}: log-posterior correction case {case} "
                         f"(jacobian={jacobian}, renorm={renorm})")
        return total_jacobian, total_renorm, breakdown

    # ---- vectorisation plan (built once) --------------------------------------------------
    def _build_plan(self) -> None:
        names = self.log_likelihood.names
        self._names = names
        self._template = np.array([float(self.fixed_params[n]) if n in self.fixed_params else np.nan
                                   for n in names])
        self._free_idx = np.array([names.index(n) for n in self.free_params_names], dtype=np.int64)
        missing = [n for n in names if n not in self.fixed_params and n not in self.free_params_names]
        if missing:
            raise KeyError(f"parameters neither fixed nor free: {missing}")
        self._jit_idx = np.array([names.index(f"jit_{inst}") for inst in self.unique_instruments])
        prior_keys = set(self.priors.keys())
        self._case3 = prior_keys != set(self.free_params_names)     # fit.py:3418-3423
        pars = self.parameterisation.pars
        # prior-evaluation key order, exactly the dict order of fit.py:3426-3444
        order = [k for k in self.free_params_names if k in prior_keys]
        if self._case3:
            for L in self.planet_letters:
                for dp in ("P", "K", "e", "w", "Tp"):
                    key = f"{dp}_{L}"
                    if key in prior_keys and key not in order:
                        order.append(key)
        self._prior_order = order
        self._planet_cols = {L: {par: names.index(f"{par}_{L}") for par in pars} for L in self.planet_letters}

    def _full(self, theta_free: np.ndarray) -> np.ndarray:
        full = np.repeat(self._template[None, :], theta_free.shape[0], axis=0)
        full[:, self._free_idx] = theta_free
        return full

    def _log_prior_batch(self, theta_free: np.ndarray, full: np.ndarray):
        """Vectorised fit.py:3475-3482: returns (lp, conversion_ok)."""
        free_col = {n: theta_free[:, i] for i, n in enumerate(self.free_params_names)}
        ok = np.ones(theta_free.shape[0], bool)
        if not self._case3:
            cols = {k: free_col[k] for k in self._prior_order}
        else:
            conv = {}
            for L, cmap in self._planet_cols.items():
                d, okL = self.parameterisation.to_default_vec({par: full[:, j] for par, j in cmap.items()})
                ok &= okL
                for dp, v in d.items():
                    conv[f"{dp}_{L}"] = v
            cols = {}
            for k in self._prior_order:
                # planet default keys take the converted value (fit.py:3441-3444 overwrite in place)
                cols[k] = conv[k] if k in conv else free_col[k]
        with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
            lp = self.log_prior.batch(cols)
        lp = np.broadcast_to(np.asarray(lp, dtype=np.float64), (theta_free.shape[0],))
        return lp, ok

    # ---- public API -----------------------------------------------------------------------
    @property
    def route(self) -> str:
        """Where the priors of log_probability[_batch] are evaluated: "device" or "host"."""
        if self._route == "auto":
            from .engine import RVEngine
            eng = self.log_likelihood._engine
            ok = all(is_builtin(self._priors[k]) for k in self._prior_order) and \
                (eng is None or isinstance(eng, RVEngine))
            self._route = "device" if ok else "host"
        return self._route

    def _device(self) -> "DevicePosterior":
        if self._dpost is None:
            self._dpost = DevicePosterior(self)
        return self._dpost

    def log_probability_batch(self, theta_free) -> np.ndarray:
        theta_free = np.ascontiguousarray(np.atleast_2d(np.asarray(theta_free, dtype=np.float64)))
        if theta_free.shape[1] != len(self.free_params_names):
            raise ValueError(f"expected {len(self.free_params_names)} free parameters, got {theta_free.shape[1]}")
        if self.route == "device":
            return self._device()._eval(theta_free)
        return self._host_batch(theta_free)

    def _host_batch(self, theta_free: np.ndarray) -> np.ndarray:
        """The host-prior form of log_probability_batch (custom priors; route="host")."""
        full = self._full(theta_free)
        dead = np.any(full[:, self._jit_idx] < 0, axis=1)                 # fit.py:3465-3468
        lp, conv_ok = self._log_prior_batch(theta_free, full)             # fit.py:3475-3480
        dead |= ~conv_ok
        dead |= ~np.isfinite(lp)                                          # fit.py:3481-3482
        out = np.full(theta_free.shape[0], -np.inf)
        live = ~dead
        if live.any():
            ll = self.log_likelihood.batch(full[live])                    # fit.py:3485
            logprob = ll + lp[live]                                       # fit.py:3492-3494
            logprob = logprob + self._logprob_jacobian_correction
            logprob = logprob + self._logprob_prior_renorm_correction
            out[live] = logprob
        return out

    __call__ = log_probability_batch

    def log_probability(self, free_params_dict: Dict[str, float]) -> float:
        """fit.py:3448-3495: the log-posterior of one walker given as {name: value} (emcee with
        ``parameter_names``, MAP).  A dict of equal-length arrays -- what emcee passes with
        ``parameter_names`` AND ``vectorize=True`` -- gives the array of the walkers' values in one
        device call."""
        vals = [free_params_dict[n] for n in self.free_params_names]
        if np.ndim(vals[0]) > 0:                                        # emcee vectorize=True
            return self.log_probability_batch(np.stack([np.asarray(v, np.float64) for v in vals], axis=1))
        row = np.array([vals], dtype=np.float64)
        if self.route == "device":
            return float(self._device()._eval(row)[0])
        return float(self._host_batch(row)[0])

    def __getstate__(self):           # picklable (multiprocessing pools): device objects rebuilt lazily
        d = dict(self.__dict__)
        d["_dpost"] = None
        return d

    def _convert_params_for_prior_evaluation(self, free_params_dict: Dict[str, float]) -> Dict[str, float]:
        """fit.py:3399-3446 (scalar form, kept for API parity)."""
        prior_keys = set(self.priors.keys())
        if prior_keys == set(self.free_params_names):
            return free_params_dict
        params_for_prior = {k: v for k, v in free_params_dict.items() if k in prior_keys}
        all_params = self.fixed_params | free_params_dict
        for L in self.planet_letters:
            planet_params = {par: all_params[f"{par}_{L}"] for par in self.parameterisation.pars}
            default_params = self.parameterisation.convert_pars_to_default_parameterisation(planet_params)
            for dp, value in default_params.items():
                key = f"{dp}_{L}"
                if key in prior_keys:
                    params_for_prior[key] = value
        return params_for_prior

    def device_posterior(self) -> "DevicePosterior":
        """The same log-posterior evaluated wholly on the GPU (priors included)."""
        return DevicePosterior(self)

    def _negative_log_probability_for_MAP(self, free_params_vals) -> float:
        """fit.py:3497-3526."""
        logprob = self.log_probability(dict(zip(self.free_params_names, free_params_vals)))
        neg = -logprob
        if not np.isfinite(neg):
            return 1e30
        return neg


class DevicePosterior:
    """``LogPosterior`` evaluated wholly on the GPU (include/rvk_post.h).

    The host builds, once, what ``LogPosterior.log_probability`` recomputes per
    call: the fixed/free layout, the prior slots in the reference's key order
    (fit.py:3426-3444 dict order) with each prior's constants, and the two
    correction constants.  ``__call__`` (host arrays) and ``device`` (torch
    tensors, stream-ordered) then run the jitter check, the prior-side conversion,
    the priors, the log-likelihood and the corrections in ONE kernel (the likelihood
    kernel's DIRECT mode: each wave builds its walker's row, checks and priors, then runs
    its epoch loop) when the posterior fits the fused limits (<= 64 free parameters, full
    columns and priors; <= 4 planets), else in two (the log-prior kernel, then the
    likelihood with the posterior epilogue; same bits).  Only the
    built-in priors have a device form; a custom callable prior raises
    NotImplementedError (use ``LogPosterior.log_probability_batch``)."""

    def __init__(self, lpost: "LogPosterior") -> None:
        self._lpost = weakref.ref(lpost)       # no cycle with LogPosterior._dpost (GC order)
        eng = lpost.log_likelihood.engine
        self.engine = eng
        names = lpost._names
        self.n_free = len(lpost.free_params_names)
        kinds, srcs, pars = [], [], []
        conv_keys = {f"{dp}_{L}": (i, j) for i, L in enumerate(lpost.planet_letters)
                     for j, dp in enumerate(("P", "K", "e", "w", "Tp"))}
        for k in lpost._prior_order:
            kind, p = device_params(lpost._priors[k])
            kinds.append(kind)
            pars.append(p)
            if lpost._case3 and k in conv_keys:
                srcs.append(_lib.prior_src_default(*conv_keys[k]))
            else:
                srcs.append(names.index(k))
        self._kinds = np.ascontiguousarray(kinds, np.int32)
        self._srcs = np.ascontiguousarray(srcs, np.int32)
        self._pars = np.ascontiguousarray(np.reshape(pars, (-1, _lib.PRIOR_NPAR)), np.float64)
        self._free_idx = np.ascontiguousarray(lpost._free_idx, np.int32)
        tmpl = np.nan_to_num(lpost._template, nan=0.0)            # free columns are overwritten per walker
        self._tmpl = np.ascontiguousarray(tmpl, np.float64)
        flags = _lib.POST_CONVERT if lpost._case3 else 0
        L = _lib.load()
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        self._p = L.rvk_post_create(eng._h, self.n_free, self._free_idx.ctypes.data_as(ip),
                                    self._tmpl.ctypes.data_as(dp), len(kinds), self._kinds.ctypes.data_as(ip),
                                    self._srcs.ctypes.data_as(ip), self._pars.ctypes.data_as(dp),
                                    float(lpost._logprob_jacobian_correction),
                                    float(lpost._logprob_prior_renorm_correction), flags)
        if not self._p:
            raise _lib.RVKError(f"rvk_post_create failed: {_lib.last_error()}")
        self._fn = _lib.fast().rvk_logpost

    def __call__(self, theta_free) -> np.ndarray:
        theta_free = np.ascontiguousarray(np.atleast_2d(np.asarray(theta_free, dtype=np.float64)))
        if theta_free.shape[1] != self.n_free:
            raise ValueError(f"expected {self.n_free} free parameters, got {theta_free.shape[1]}")
        return self._eval(theta_free)

    def _eval(self, x: np.ndarray) -> np.ndarray:
        """rvk_logpost on a C-contiguous float64 [W, n_free] block (checked by the caller)."""
        out = np.empty(x.shape[0])
        if self._fn(self._p, _lib.addr(x), x.shape[0], x.shape[1], _lib.addr(out)):
            _lib.check(-1)
        return out

    def device(self, theta_free, out, stream=None) -> None:
        """theta_free: float64 cuda tensor [W, >= n_free] (unit column stride); out: float64 [W]."""
        import torch
        assert theta_free.dtype == torch.float64 and out.dtype == torch.float64
        assert theta_free.is_cuda and theta_free.stride(1) == 1 and out.is_contiguous()
        if stream is None:
            stream = torch.cuda.current_stream(theta_free.device)
        _lib.check(_lib.load().rvk_logpost_device(self._p, theta_free.data_ptr(), theta_free.shape[0],
                                                  theta_free.stride(0), out.data_ptr(), stream.cuda_stream))

    def reserve(self, max_walkers: int) -> None:
        _lib.check(_lib.load().rvk_post_reserve(self._p, int(max_walkers)))

    def close(self) -> None:
        if getattr(self, "_p", None):
            _lib.load().rvk_post_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
