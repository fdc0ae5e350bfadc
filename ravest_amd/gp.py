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
over a walker block.  The factorisation runs in fp32 on the device (config 5
is fp32); an invalid planet gives -inf like the reference's mean-model fail-fast.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import numpy as np

from . import _lib
from .param import Parameterisation, as_parameterisation, full_param_names

SUPPORTED_KERNELS = ["Quasiperiodic"]
HYPERPARAMS = ["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"]   # gp.py:37, the C-ABI hyper row order


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
                 parameterisation: Parameterisation, gp_kernel: GPKernel, device: int = -1) -> None:
        parameterisation = as_parameterisation(parameterisation)   # str, ours or ravest's own object
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

    def close(self) -> None:
        if getattr(self, "_g", None):
            _lib.load().rvk_gp_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
