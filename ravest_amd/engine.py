"""RVEngine: a device-resident RV log-likelihood handle (wraps rvk_handle).

One engine = one dataset on one MI355X.  ``loglike`` takes a [W, P_full]
host block in the C-ABI's full-parameter order (include/rvk.h) and returns the
W per-walker log-likelihoods, -inf where ravest's Planet() would raise
(fit.py:3622-3627).  ``loglike_device`` is the stream-ordered form on
device-resident torch tensors (used by bench.py and the multi-GPU path).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .param import Parameterisation, as_parameterisation

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


def _p(a: np.ndarray, ptype=_dp):
    return a.ctypes.data_as(ptype)


class RVEngine:
    def __init__(self, time, vel, velerr, inst_idx=None, n_inst: int = 1, n_planets: int = 1,
                 parameterisation="P K e w Tp", t0: float = 0.0, device: int = -1):
        L = _lib.load()
        parameterisation = as_parameterisation(parameterisation)   # str, ours or ravest's own object
        self.parameterisation = parameterisation
        model_only = time is None                     # rvk_predict only (n_epochs = 0)
        self.time = np.zeros(0) if model_only else np.ascontiguousarray(time, np.float64)
        self.vel = np.zeros(0) if model_only else np.ascontiguousarray(vel, np.float64)
        self.velerr = np.zeros(0) if model_only else np.ascontiguousarray(velerr, np.float64)
        n = self.time.size
        if not (self.vel.size == n and self.velerr.size == n):
            raise ValueError("time, vel and velerr must have the same length")
        self.inst_idx = (np.zeros(n, np.int32) if inst_idx is None
                         else np.ascontiguousarray(inst_idx, np.int32))
        self.n_epochs, self.n_inst, self.n_planets, self.t0 = n, int(n_inst), int(n_planets), float(t0)
        self.p_full = 5 * self.n_planets + 2 * self.n_inst + 2
        nul = C.POINTER(C.c_double)()
        self._h = L.rvk_create(nul if model_only else _p(self.time), nul if model_only else _p(self.vel),
                               nul if model_only else _p(self.velerr),
                               C.POINTER(C.c_int32)() if model_only else _p(self.inst_idx, _ip),
                               n, self.n_inst, self.n_planets, parameterisation.code, self.t0, int(device))
        if not self._h:
            raise _lib.RVKError(f"rvk_create failed: {_lib.last_error()}")

    # -- host-buffer path (blocking) -------------------------------------------------
    def loglike(self, theta: np.ndarray) -> np.ndarray:
        theta = np.ascontiguousarray(np.atleast_2d(theta), np.float64)
        if theta.shape[1] < self.p_full:
            raise ValueError(f"theta rows have {theta.shape[1]} values, need P_full={self.p_full}")
        out = np.empty(theta.shape[0], np.float64)
        if _lib.fast().rvk_loglike(self._h, _lib.addr(theta), theta.shape[0], theta.shape[1], _lib.addr(out)):
            _lib.check(-1)
        return out

    # -- device path (async on the given / current torch stream) ---------------------
    def loglike_device(self, theta, out, stream=None) -> None:
        """theta: float64 cuda tensor [W, >=P_full] (contiguous rows); out: float64 [W]."""
        import torch
        assert theta.dtype == torch.float64 and out.dtype == torch.float64
        assert theta.is_cuda and out.is_cuda and theta.stride(1) == 1 and out.is_contiguous()
        if stream is None:
            stream = torch.cuda.current_stream(theta.device)
        _lib.check(_lib.load().rvk_loglike_device(self._h, theta.data_ptr(), theta.shape[0], theta.stride(0),
                                                  out.data_ptr(), stream.cuda_stream))

    def _what(self, planets, trend, gamma) -> int:
        """include/rvk.h's component mask: every planet, planets 0-7 by bit, or one planet >= 8 by index."""
        planets = list(range(self.n_planets)) if planets is None else sorted({int(p) for p in planets})
        what = 0
        if planets and planets == list(range(self.n_planets)):
            what |= _lib.PRED_ALL_PLANETS
        else:
            high = [p for p in planets if p >= 8]
            if len(high) > 1:
                raise ValueError("rvk_predict selects planets >= 8 one at a time (or all planets)")
            for p in planets:
                what |= (1 << p) if p < 8 else _lib.pred_planet(p)
        if trend:
            what |= _lib.PRED_TREND
        if gamma:
            what |= _lib.PRED_GAMMA
        return what

    def predict_device(self, theta, t, out, inst=None, planets=None, trend=True, gamma=False, stream=None) -> None:
        """Device form of :meth:`predict` on torch tensors (theta [S, >=P_full], t [T], out [S, T])."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(theta.device)
        _lib.check(_lib.load().rvk_predict_device(self._h, theta.data_ptr(), theta.shape[0], theta.stride(0),
                                                  t.data_ptr(), 0 if inst is None else inst.data_ptr(), t.numel(),
                                                  self._what(planets, trend, gamma), out.data_ptr(),
                                                  stream.cuda_stream))

    def predict(self, theta: np.ndarray, t, inst=None, planets=None, trend=True, gamma=False) -> np.ndarray:
        """Posterior-predictive RV [S, T] (sum of the selected planets [+ trend] [+ gamma])."""
        theta = np.ascontiguousarray(np.atleast_2d(theta), np.float64)
        t = np.ascontiguousarray(t, np.float64)
        what = self._what(planets, trend, gamma)
        ip = None
        if inst is not None:
            inst = np.ascontiguousarray(inst, np.int32)
            ip = _p(inst, _ip)
        out = np.empty((theta.shape[0], t.size), np.float64)
        _lib.check(_lib.load().rvk_predict(self._h, _p(theta), theta.shape[0], theta.shape[1], _p(t), ip,
                                           t.size, what, _p(out)))
        return out

    def set_solver(self, solver: int) -> None:
        """0 = production solver (default); 1 = ravest's Halley iteration restated."""
        _lib.check(_lib.load().rvk_set_option(self._h, _lib.OPT_SOLVER, int(solver)))

    def set_lanes_per_walker(self, lpw: int) -> None:
        """0 = chosen per launch (default); 64, 32 or 16 lanes of a wave per walker (RVK_OPT_LPW)."""
        _lib.check(_lib.load().rvk_set_option(self._h, _lib.OPT_LPW, int(lpw)))

    def set_graph(self, on: bool) -> None:
        """RVK_OPT_GRAPH: the device stretch move replays a cached HIP graph per block of steps."""
        _lib.check(_lib.load().rvk_set_option(self._h, _lib.OPT_GRAPH, int(bool(on))))

    def set_hostio(self, mode: str) -> None:
        """RVK_OPT_HOSTIO for the blocking host-buffer calls on this handle and the posteriors
        built on it: "auto" (default), "pageable", "pinned" or "zerocopy" (include/rvk.h)."""
        _lib.check(_lib.load().rvk_set_option(self._h, _lib.OPT_HOSTIO, _lib.HOSTIO[mode]))

    def set_lds_poison(self, on) -> None:
        """RVK_OPT_LDS_POISON (tests only): the kernels fill their LDS sin/cos table with NaN
        first and the real values ~10 us later, so a read not ordered after the publishing
        barrier yields NaN results (include/rvk.h).  Applies to every kernel launched for this
        handle, its posteriors and GP objects.  on = 2: the positive control (the real values
        are never stored: every kernel the option reaches returns NaN)."""
        v = 2 if (not isinstance(on, bool) and on == 2) else int(bool(on))
        _lib.check(_lib.load().rvk_set_option(self._h, _lib.OPT_LDS_POISON, v))

    def reserve(self, max_walkers: int) -> None:
        _lib.check(_lib.load().rvk_reserve(self._h, int(max_walkers)))

    def stream_ptr(self) -> int:
        return _lib.load().rvk_stream(self._h) or 0

    def sync(self) -> None:
        _lib.check(_lib.load().rvk_sync(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.load().rvk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_kepler(M, e, device: int = -1, solver: int = 0):
    """cos E, sin E on the GPU for arrays of (M, e) (ravest _solve_kepler, model.py:23-70)."""
    M = np.ascontiguousarray(M, np.float64)
    e = np.ascontiguousarray(np.broadcast_to(e, M.shape), np.float64)
    c = np.empty_like(M)
    s = np.empty_like(M)
    _lib.check(_lib.load().rvk_solve_kepler(_p(M), _p(e), M.size, _p(c), _p(s), device, solver))
    return c, s
