"""ctypes wrapper of the CPU oracle (oracle/rv_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as
the product path.  Builds itself with ``make -C oracle`` if the .so is absent.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "librvoracle.so")
_lib = None

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        L.orc_solve_kepler_batch.argtypes = [_dp, _dp, C.c_int64, _dp, _dp, _ip]
        L.orc_compute_rv.argtypes = [_dp, C.c_int, C.c_double, C.c_double, C.c_double, _dp]
        L.orc_planet_rv.argtypes = [C.c_int, _dp, _dp, C.c_int, _dp, _dp]
        L.orc_planet_rv.restype = C.c_int
        L.orc_tc_to_tp.argtypes = [C.c_double] * 4 + [C.POINTER(C.c_double)]
        L.orc_tc_to_tp.restype = C.c_int
        L.orc_pairwise_sum.argtypes = [_dp, C.c_int64]
        L.orc_pairwise_sum.restype = C.c_double
        L.orc_loglike_batch.argtypes = [_dp, _dp, _dp, _ip, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_double, _dp, C.c_int64, C.c_int64, _dp, C.c_int]
        L.orc_loglike_batch.restype = C.c_int
        _lib = L
    return _lib


def solve_kepler(M, e):
    M = np.ascontiguousarray(M, np.float64); e = np.ascontiguousarray(np.broadcast_to(e, M.shape), np.float64)
    c = np.empty_like(M); s = np.empty_like(M); it = np.empty(M.shape, np.int32)
    lib().orc_solve_kepler_batch(M, e, M.size, c, s, it)
    return c, s, it


def compute_rv(M, e, K, w):
    M = np.ascontiguousarray(M, np.float64); out = np.empty_like(M)
    lib().orc_compute_rv(M, M.size, e, K, w, out)
    return out


def planet_rv(par_code, p5, t):
    t = np.ascontiguousarray(t, np.float64); out = np.empty_like(t); mb = np.empty_like(t)
    ok = lib().orc_planet_rv(par_code, np.ascontiguousarray(p5, np.float64), t, t.size, out, mb)
    return out if ok else None


def tc_to_tp(tc, P, e, w):
    r = C.c_double()
    ok = lib().orc_tc_to_tp(tc, P, e, w, C.byref(r))
    return r.value if ok else None


def pairwise_sum(a):
    a = np.ascontiguousarray(a, np.float64)
    return lib().orc_pairwise_sum(a, a.size)


def loglike(time, vel, velerr, inst_idx, n_inst, n_planets, par_code, t0, theta, nthreads=1):
    """Per-walker log-likelihood; theta is [W, P_full] in include/rvk.h order."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), np.float64)
    out = np.empty(theta.shape[0])
    used = lib().orc_loglike_batch(np.ascontiguousarray(time, np.float64), np.ascontiguousarray(vel, np.float64),
                                   np.ascontiguousarray(velerr, np.float64), np.ascontiguousarray(inst_idx, np.int32),
                                   len(time), n_inst, n_planets, par_code, t0, theta, theta.shape[0],
                                   theta.shape[1], out, nthreads)
    return out, used
