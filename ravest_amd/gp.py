"""Quasi-periodic GP likelihood: host mirror of ``ravest.gp.GPKernel`` and
``ravest.fit.GPLogLikelihood``, evaluated by the batched HIP kernel of
include/rvk_gp.h (BASELINE config 5).

``GPKernel`` keeps the reference's kernel-type handling and hyperparameter
validation (src/ravest/gp.py:13-127); ``build_kernel`` returns a small kernel
description (tinygp is not installed here) whose ``__call__`` evaluates the
same covariance, A^2 exp(-gamma sin^2(pi tau / P)) exp(-tau^2 / (2 lambda_e^2))
with gamma = 1 / (2 lambda_p^2) (gp.py:126-156).

``GPLogLikelihood`` has the reference's constructor and ``__call__(params,
hyperparams) -> float`` (fit.py:7942-8105), plus ``batch(theta_full, hyper)``
over a walker block.  The factorisation precision is a constructor option
(include/rvk_gp.h): "fp64" (default: the reference's own precision,
jax_enable_x64, fit.py:39), "fp32+fp64" (opt-in: fp32 MFMA Cholesky -- BASELINE
config 5 is fp32 -- with the walkers it rejects as not positive definite
re-evaluated in fp64) or "fp32".  An invalid planet gives -inf like the reference's mean-model
fail-fast.

``GPLogPosterior`` mirrors fit.py:7596-7939 (jitter check, hyperparameter
validity, priors with the Case-3 conversion, hyperpriors, the GP likelihood and
the evidence corrections), with ``log_probability(dict)`` for emcee's
``parameter_names`` form, ``log_probability_batch`` for ``vectorize=True`` and
``device_posterior()`` for the all-device form (rvk_gp_logpost).
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Dict, List

import numpy as np

from . import _lib
from .param import Parameterisation, as_parameterisation, full_param_names
from .prior import as_priors, is_builtin, device_params, logpdf_vec

SUPPORTED_KERNELS = ["Quasiperiodic"]
HYPERPARAMS = ["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"]   # gp.py:37, the C-ABI hyper row order
PRECISION = {"fp32": _lib.GP_FP32, "fp32+fp64": _lib.GP_FP32_FP64_FALLBACK, "fp64": _lib.GP_FP64}


class QuasiperiodicKernel:
    """A^2 * ExpSineSquared(scale=P, gamma=1/(2 lambda_p^2)) * ExpSquared(scale=lambda_e)."""

    def __init__(self, gp_amp, gp_lambda_e, gp_lambda_p, gp_period) -> None:
        self.gp_amp, self.gp_lambda_e = float(gp_amp), float(gp_lambda_e)
        self.gp_lambda_p, self.gp_period = float(gp_lambda_p), float(gp_period)
        self.gamma = 1 / (2 * np.square(self.gp_lambda_p))

    def __call__(self, x1, x2) -> np.ndarray:
        tau = np.subtract.outer(np.asarray(x1, float), np.asarray(x2, float))
        ess = np.exp(-self.gamma * np.square(np.sin(np.pi * np.abs(tau) / self.gp_period)))
        es = np.exp(-0.5 * np.square(tau / self.gp_lambda_e))
        return np.square(self.gp_amp) * ess * es

    def __repr__(self) -> str:
        return (f"QuasiperiodicKernel(gp_amp={self.gp_amp}, gp_lambda_e={self.gp_lambda_e}, "
                f"gp_lambda_p={self.gp_lambda_p}, gp_period={self.gp_period})")


class GPKernel:
    """gp.py:13-156."""

    def __init__(self, kernel_type: str) -> None:
        self.kernel_type = kernel_type
        if self.kernel_type == "Quasiperiodic":
            self.expected_hyperparams = list(HYPERPARAMS)
        else:
            raise ValueError(f"Unsupported kernel type: {kernel_type}. "
                             f"Supported kernels: {SUPPORTED_KERNELS}")

    def get_expected_hyperparams(self) -> List[str]:
        return self.expected_hyperparams.copy()

    def validate_hyperparams(self, hyperparams: dict) -> None:
        provided, expected = set(hyperparams.keys()), set(self.expected_hyperparams)
        missing = expected - provided
        if missing:
            raise ValueError(f"Missing required hyperparameters: {missing}")
        unexpected = provided - expected
        if unexpected:
            raise ValueError(f"Unexpected hyperparameters: {unexpected}")
        self._validate_hyperparams_values({name: p.value for name, p in hyperparams.items()})

    def _validate_hyperparams_values(self, hyperparams_values: Dict[str, float]) -> None:
        for key in self.expected_hyperparams:
            if not np.isfinite(hyperparams_values[key]):
                raise ValueError(f"Non-finite hyperparameter found in: {hyperparams_values}")
        if self.kernel_type == "Quasiperiodic":
            for key in self.expected_hyperparams:
                if hyperparams_values[key] <= 0:
                    raise ValueError(f"{key} must be positive, got {hyperparams_values[key]}")

    def valid_hyperparams_vec(self, hyper: np.ndarray) -> np.ndarray:
        """Vector form of _validate_hyperparams_values over [W, 4] rows (mask instead of raise)."""
        hyper = np.atleast_2d(hyper)
        return np.all(np.isfinite(hyper), axis=1) & np.all(hyper > 0, axis=1)

    def build_kernel(self, hyperparams: Dict[str, float]) -> QuasiperiodicKernel:
        return QuasiperiodicKernel(*(hyperparams[k] for k in self.expected_hyperparams))


class GPLogLikelihood:
    """fit.py:7942-8105 on the GPU (rvk_gp_loglike)."""

    def __init__(self, time, vel, velerr, t0, instrument, unique_instruments, planet_letters,
                 parameterisation: Parameterisation, gp_kernel: GPKernel, device: int = -1,
                 precision: str = "fp64") -> None:
        parameterisation = as_parameterisation(parameterisation)   # str, ours or ravest's own object
        if precision not in PRECISION:
            raise ValueError(f"precision must be one of {list(PRECISION)}, got {precision!r}")
        if gp_kernel.kernel_type != "Quasiperiodic":
            raise ValueError(f"no device form for GP kernel {gp_kernel.kernel_type}")
        self.time, self.vel, self.velerr, self.t0 = time, vel, velerr, t0
        self.instrument, self.unique_instruments = instrument, unique_instruments
        self.planet_letters, self.parameterisation, self.gp_kernel = planet_letters, parameterisation, gp_kernel
        _inst_to_idx = {inst: i for i, inst in enumerate(self.unique_instruments)}
        self._instrument_indices = np.array([_inst_to_idx[inst] for inst in self.instrument], dtype=np.int32)
        self.names = full_param_names(planet_letters, parameterisation, list(unique_instruments))
        from .engine import RVEngine
        self.engine = RVEngine(time, vel, velerr, self._instrument_indices, len(unique_instruments),
                               len(planet_letters), parameterisation, t0, device=device)
        self._g = _lib.load().rvk_gp_create(self.engine._h, _lib.GP_QUASIPERIODIC)
        if not self._g:
            raise _lib.RVKError(f"rvk_gp_create failed: {_lib.last_error()}")
        self.precision = precision
        _lib.check(_lib.load().rvk_gp_set_precision(self._g, PRECISION[precision]))

    def batch(self, theta_full: np.ndarray, hyper: np.ndarray) -> np.ndarray:
        """[W, P_full] (``self.names`` order) and [W, 4] (gp_amp, gp_lambda_e, gp_lambda_p, gp_period)."""
        theta_full = np.ascontiguousarray(np.atleast_2d(theta_full), np.float64)
        hyper = np.ascontiguousarray(np.atleast_2d(hyper), np.float64)
        if hyper.shape[0] != theta_full.shape[0] or hyper.shape[1] < _lib.GP_NHYPER:
            raise ValueError("hyper must be [W, 4] alongside theta [W, P_full]")
        out = np.empty(theta_full.shape[0])
        dp = C.POINTER(C.c_double)
        _lib.check(_lib.load().rvk_gp_loglike(self._g, theta_full.ctypes.data_as(dp), hyper.ctypes.data_as(dp),
                                              theta_full.shape[0], theta_full.shape[1], hyper.shape[1],
                                              out.ctypes.data_as(dp)))
        return out

    def device(self, theta, hyper, out, stream=None) -> None:
        """Stream-ordered form on float64 cuda tensors theta [W, >=P_full], hyper [W, >=4], out [W]."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(theta.device)
        _lib.check(_lib.load().rvk_gp_loglike_device(self._g, theta.data_ptr(), hyper.data_ptr(), theta.shape[0],
                                                     theta.stride(0), hyper.stride(0), out.data_ptr(),
                                                     stream.cuda_stream))

    def __call__(self, params: Dict[str, float], hyperparams: Dict[str, float]) -> float:
        row = np.array([[params[n] for n in self.names]], dtype=np.float64)
        hyp = np.array([[hyperparams[k] for k in HYPERPARAMS]], dtype=np.float64)
        return float(self.batch(row, hyp)[0])

    def condition(self, theta_full: np.ndarray, hyper: np.ndarray, times) -> np.ndarray:
        """[S, T] fp64: the GP conditioned on each sample's residuals at the data (diagonal
        velerr^2 + jit^2), its mean at ``times`` -- tinygp ``GaussianProcess(kernel, X=time,
        diag=...).condition(y=residuals, X_test=times).mean`` per sample (fit.py:7494-7554).
        A row of NaN marks a sample with an invalid planet."""
        theta_full = np.ascontiguousarray(np.atleast_2d(theta_full), np.float64)
        hyper = np.ascontiguousarray(np.atleast_2d(hyper), np.float64)
        times = np.ascontiguousarray(np.atleast_1d(np.asarray(times, np.float64)))
        if hyper.shape[0] != theta_full.shape[0] or hyper.shape[1] < _lib.GP_NHYPER:
            raise ValueError("hyper must be [S, 4] alongside theta [S, P_full]")
        out = np.empty((theta_full.shape[0], times.size))
        dp = C.POINTER(C.c_double)
        _lib.check(_lib.load().rvk_gp_predict(self._g, theta_full.ctypes.data_as(dp), hyper.ctypes.data_as(dp),
                                              theta_full.shape[0], theta_full.shape[1], hyper.shape[1],
                                              times.ctypes.data_as(dp), times.size, out.ctypes.data_as(dp)))
        return out

    def condition_device(self, theta, hyper, times, out, stream=None) -> None:
        """Stream-ordered form of ``condition`` on float64 cuda tensors (out [S, T])."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(theta.device)
        _lib.check(_lib.load().rvk_gp_predict_device(self._g, theta.data_ptr(), hyper.data_ptr(), theta.shape[0],
                                                     theta.stride(0), hyper.stride(0), times.data_ptr(),
                                                     times.numel(), out.data_ptr(), stream.cuda_stream))

    def close(self) -> None:
        if getattr(self, "_g", None):
            _lib.load().rvk_gp_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GPLogPosterior:
    """fit.py:7596-7939.  Emcee coordinates are ``free_params_names + free_hyperparams_names``
    (GPFitter.run_mcmc, fit.py:4982)."""

    def __init__(self, planet_letters, parameterisation, gp_kernel: GPKernel, priors: dict, hyperpriors: dict,
                 fixed_params: dict, fixed_hyperparams: dict, free_params_names: list, free_hyperparams_names: list,
                 time, vel, velerr, t0: float, instrument, unique_instruments, device: int = -1,
                 precision: str = "fp64", route: str = "auto") -> None:
        from .posterior import LogPosterior, LogPrior
        self.planet_letters = planet_letters
        self.parameterisation = as_parameterisation(parameterisation)   # ravest's own object accepted
        self.gp_kernel = gp_kernel
        self.priors = priors
        self.hyperpriors = hyperpriors
        self.fixed_params = fixed_params
        self.fixed_hyperparams = fixed_hyperparams
        self.free_params_names = list(free_params_names)
        self.free_hyperparams_names = list(free_hyperparams_names)
        self.time, self.vel, self.velerr, self.t0 = time, vel, velerr, t0
        self.instrument, self.unique_instruments = instrument, unique_instruments
        self.gp_log_likelihood = GPLogLikelihood(time=time, vel=vel, velerr=velerr, t0=t0, instrument=instrument,
                                                 unique_instruments=unique_instruments,
                                                 planet_letters=planet_letters,
                                                 parameterisation=self.parameterisation, gp_kernel=gp_kernel,
                                                 device=device, precision=precision)
        # The parameter half (priors, Case 1/2/3 corrections, prior-side conversion, fixed/free
        # layout) is LogPosterior's (fit.py:7694-7834 repeats fit.py:3306-3446 verbatim); its
        # likelihood engine is never used for evaluation here.
        self._pp = LogPosterior(planet_letters, self.parameterisation, priors, fixed_params, self.free_params_names,
                                time, vel, velerr, instrument, unique_instruments, t0,
                                engine=self.gp_log_likelihood.engine)
        self.log_prior = self._pp.log_prior
        self.log_hyperprior = LogPrior(hyperpriors)
        self._hyperpriors = as_priors(hyperpriors)
        (self._logprob_jacobian_correction, self._logprob_prior_renorm_correction,
         self._logprob_correction_breakdown) = (self._pp._logprob_jacobian_correction,
                                                self._pp._logprob_prior_renorm_correction,
                                                self._pp._logprob_correction_breakdown)
        missing = [k for k in HYPERPARAMS if k not in fixed_hyperparams and k not in self.free_hyperparams_names]
        if missing:
            raise KeyError(f"hyperparameters neither fixed nor free: {missing}")
        self._htemplate = np.array([float(fixed_hyperparams[k]) if k in fixed_hyperparams else np.nan
                                    for k in HYPERPARAMS])
        self._hfree_idx = np.array([HYPERPARAMS.index(k) for k in self.free_hyperparams_names], dtype=np.int64)
        self.n_free = len(self.free_params_names) + len(self.free_hyperparams_names)
        if route not in ("auto", "device", "host"):
            raise ValueError("route must be 'auto', 'device' or 'host'")
        self._route = route              # as LogPosterior.route: device priors when all are built-in
        self._dpost = None

    def _classify_planet_case(self, letter: str) -> str:
        return self._pp._classify_planet_case(letter)

    def _compute_logprob_corrections(self):
        return self._pp._compute_logprob_corrections()

    def _convert_params_for_prior_evaluation(self, free_params_dict: dict) -> dict:
        return self._pp._convert_params_for_prior_evaluation(free_params_dict)

    def _split(self, x: np.ndarray):
        nf = len(self.free_params_names)
        xp, xh = x[:, :nf], x[:, nf:]
        hyper = np.repeat(self._htemplate[None, :], x.shape[0], axis=0)
        hyper[:, self._hfree_idx] = xh
        return xp, xh, hyper

    @property
    def route(self) -> str:
        """Where the priors and hyperpriors are evaluated: "device" (DeviceGPPosterior, one host
        round trip) when every one is a built-in prior class, else "host"."""
        if self._route == "auto":
            ok = all(is_builtin(self._pp._priors[k]) for k in self._pp._prior_order) and \
                all(is_builtin(self._hyperpriors[k]) for k in self.free_hyperparams_names)
            self._route = "device" if ok else "host"
        return self._route

    def _device(self) -> "DeviceGPPosterior":
        if self._dpost is None:
            self._dpost = DeviceGPPosterior(self)
        return self._dpost

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_dpost"] = None
        return d

    def log_probability_batch(self, x) -> np.ndarray:
        """Vectorised fit.py:7836-7901 over emcee's [W, D] block."""
        x = np.ascontiguousarray(np.atleast_2d(np.asarray(x, dtype=np.float64)))
        if x.shape[1] != self.n_free:
            raise ValueError(f"expected {self.n_free} free parameters and hyperparameters, got {x.shape[1]}")
        if self.route == "device":
            return self._device()._eval(x)
        return self._host_batch(x)

    def _host_batch(self, x: np.ndarray) -> np.ndarray:
        """The host-prior form of log_probability_batch (custom priors; route="host")."""
        xp, xh, hyper = self._split(x)
        full = self._pp._full(xp)
        dead = np.any(full[:, self._pp._jit_idx] < 0, axis=1)                   # fit.py:7853-7856
        dead |= ~self.gp_kernel.valid_hyperparams_vec(hyper)                     # fit.py:7860-7867
        lp, conv_ok = self._pp._log_prior_batch(xp, full)                        # fit.py:7873-7879
        dead |= ~conv_ok
        dead |= ~np.isfinite(lp)
        with np.errstate(invalid="ignore", divide="ignore", over="ignore"):      # fit.py:7882-7885
            lhp = 0
            for i, k in enumerate(self.free_hyperparams_names):
                lhp = lhp + logpdf_vec(self._hyperpriors[k], xh[:, i])
        lhp = np.broadcast_to(np.asarray(lhp, dtype=np.float64), (x.shape[0],))
        dead |= ~np.isfinite(lhp)
        out = np.full(x.shape[0], -np.inf)
        live = ~dead
        if live.any():
            ll = self.gp_log_likelihood.batch(full[live], hyper[live])          # fit.py:7888-7891
            logprob = ll + lp[live] + lhp[live]                                  # fit.py:7898-7900
            logprob = logprob + self._logprob_jacobian_correction
            logprob = logprob + self._logprob_prior_renorm_correction
            out[live] = logprob
        return out

    __call__ = log_probability_batch

    def log_probability(self, combined_params_hyperparams: Dict[str, float]) -> float:
        """fit.py:7836-7901 for one walker ({name: value}); a dict of arrays (emcee with
        parameter_names and vectorize=True) gives every walker's value in one device call."""
        vals = [combined_params_hyperparams[n] for n in self.free_params_names + self.free_hyperparams_names]
        if np.ndim(vals[0]) > 0:
            return self.log_probability_batch(np.stack([np.asarray(v, np.float64) for v in vals], axis=1))
        return float(self.log_probability_batch(np.array([vals], dtype=np.float64))[0])

    def _negative_log_probability_for_MAP(self, combined_free_params_hyperparams_vals) -> float:
        """fit.py:7903-7939."""
        logprob = float(self.log_probability_batch(np.asarray(combined_free_params_hyperparams_vals, float))[0])
        neg = -logprob
        if not np.isfinite(neg):
            return 1e30
        return neg

    def device_posterior(self) -> "DeviceGPPosterior":
        return DeviceGPPosterior(self)


class DeviceGPPosterior:
    """``GPLogPosterior`` evaluated wholly on the GPU (include/rvk_gp.h rvk_gp_logpost): one
    prior kernel (combined row, jitter and hyperparameter checks, conversion, priors and
    hyperpriors) and the GP likelihood with its posterior epilogue.  Built-in priors only."""

    def __init__(self, gpost: GPLogPosterior) -> None:
        pp = gpost._pp
        self._gpost = weakref.ref(gpost)       # no cycle with GPLogPosterior._dpost (GC order)
        self._gll = gpost.gp_log_likelihood    # the GP handle outlives this posterior
        names = pp._names
        pf = len(names)
        kinds, srcs, pars = [], [], []
        conv_keys = {f"{dp}_{L}": (i, j) for i, L in enumerate(pp.planet_letters)
                     for j, dp in enumerate(("P", "K", "e", "w", "Tp"))}
        for k in pp._prior_order:
            kind, p = device_params(pp._priors[k])
            kinds.append(kind)
            pars.append(p)
            srcs.append(_lib.prior_src_default(*conv_keys[k]) if (pp._case3 and k in conv_keys) else names.index(k))
        n_param_prior = len(kinds)
        for k in gpost.free_hyperparams_names:
            kind, p = device_params(gpost._hyperpriors[k])
            kinds.append(kind)
            pars.append(p)
            srcs.append(pf + HYPERPARAMS.index(k))
        self.n_free = gpost.n_free
        self._kinds = np.ascontiguousarray(kinds, np.int32)
        self._srcs = np.ascontiguousarray(srcs, np.int32)
        self._pars = np.ascontiguousarray(np.reshape(pars, (-1, _lib.PRIOR_NPAR)), np.float64)
        self._free_idx = np.ascontiguousarray(np.r_[pp._free_idx, pf + gpost._hfree_idx], np.int32)
        self._tmpl = np.ascontiguousarray(np.nan_to_num(np.r_[pp._template, gpost._htemplate], nan=0.0), np.float64)
        flags = _lib.POST_CONVERT if pp._case3 else 0
        L = _lib.load()
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        self._p = L.rvk_gp_post_create(gpost.gp_log_likelihood._g, self.n_free, self._free_idx.ctypes.data_as(ip),
                                       self._tmpl.ctypes.data_as(dp), len(kinds), n_param_prior,
                                       self._kinds.ctypes.data_as(ip), self._srcs.ctypes.data_as(ip),
                                       self._pars.ctypes.data_as(dp), float(gpost._logprob_jacobian_correction),
                                       float(gpost._logprob_prior_renorm_correction), flags)
        if not self._p:
            raise _lib.RVKError(f"rvk_gp_post_create failed: {_lib.last_error()}")
        self._fn = _lib.fast().rvk_gp_logpost

    def __call__(self, x) -> np.ndarray:
        x = np.ascontiguousarray(np.atleast_2d(np.asarray(x, dtype=np.float64)))
        if x.shape[1] != self.n_free:
            raise ValueError(f"expected {self.n_free} free parameters and hyperparameters, got {x.shape[1]}")
        return self._eval(x)

    def _eval(self, x: np.ndarray) -> np.ndarray:
        """rvk_gp_logpost on a C-contiguous float64 [W, n_free] block (checked by the caller)."""
        out = np.empty(x.shape[0])
        if self._fn(self._p, _lib.addr(x), x.shape[0], x.shape[1], _lib.addr(out)):
            _lib.check(-1)
        return out

    def device(self, x, out, stream=None) -> None:
        """x: float64 cuda tensor [W, >= n_free] (unit column stride); out: float64 [W]."""
        import torch
        assert x.dtype == torch.float64 and out.dtype == torch.float64
        assert x.is_cuda and x.stride(1) == 1 and out.is_contiguous()
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        _lib.check(_lib.load().rvk_gp_logpost_device(self._p, x.data_ptr(), x.shape[0], x.stride(0), out.data_ptr(),
                                                     stream.cuda_stream))

    def reserve(self, max_walkers: int) -> None:
        _lib.check(_lib.load().rvk_gp_post_reserve(self._p, int(max_walkers)))

    def close(self) -> None:
        if getattr(self, "_p", None):
            _lib.load().rvk_gp_post_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
