"""ctypes binding of librvk.so (include/rvk.h).

The shared library is built in-tree (``python -c "import __graft_entry__ as g;
g.build()"`` or ``make -C ravest_amd``) into ``ravest_amd/lib/librvk.so``.
There is no fallback: if the library is missing or a call fails, this module
raises -- the product path never silently degrades to CPU code.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "librvk.so")
# experiment hook: A/B builds of the same source (tools/variants.sh); never set in production
LIB_PATH = os.environ.get("RAVEST_AMD_LIB", LIB_PATH)

# every symbol declared in include/rvk.h
EXPORTS = ["rvk_create", "rvk_destroy", "rvk_loglike", "rvk_loglike_device", "rvk_reserve", "rvk_predict", "rvk_predict_device",
           "rvk_solve_kepler", "rvk_set_option", "rvk_stream", "rvk_sync", "rvk_device_count",
           "rvk_last_error", "rvk_version"]

OPT_SOLVER = 1

PRED_TREND = 0x0100
PRED_GAMMA = 0x0200

_lib = None


class RVKError(RuntimeError):
    pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    try:
        # PyTorch-ROCm ships its own libamdhip64 (same SONAME); load it first so the
        # process has ONE HIP runtime and torch streams are valid handles for librvk.
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RVKError(f"{LIB_PATH} not found: the HIP extension is not built "
                       "(run __graft_entry__.build() or `make -C ravest_amd`)")
    L = C.CDLL(LIB_PATH)
    dp, ip, vp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.c_void_p
    L.rvk_create.argtypes = [dp, dp, dp, ip, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_int32]
    L.rvk_create.restype = vp
    L.rvk_destroy.argtypes = [vp]
    L.rvk_destroy.restype = None
    L.rvk_loglike.argtypes = [vp, dp, C.c_int64, C.c_int64, dp]
    L.rvk_loglike_device.argtypes = [vp, vp, C.c_int64, C.c_int64, vp, vp]
    L.rvk_predict.argtypes = [vp, dp, C.c_int64, C.c_int64, dp, ip, C.c_int64, C.c_uint32, dp]
    L.rvk_predict_device.argtypes = [vp, vp, C.c_int64, C.c_int64, vp, vp, C.c_int64, C.c_uint32, vp, vp]
    L.rvk_solve_kepler.argtypes = [dp, dp, C.c_int64, dp, dp, C.c_int32, C.c_int32]
    L.rvk_set_option.argtypes = [vp, C.c_int32, C.c_int32]
    L.rvk_reserve.argtypes = [vp, C.c_int64]
    L.rvk_stream.argtypes = [vp]
    L.rvk_stream.restype = vp
    L.rvk_sync.argtypes = [vp]
    L.rvk_device_count.argtypes = []
    L.rvk_last_error.restype = C.c_char_p
    L.rvk_version.restype = C.c_int
    for name in ("rvk_loglike", "rvk_loglike_device", "rvk_predict", "rvk_predict_device", "rvk_solve_kepler", "rvk_sync",
                 "rvk_set_option", "rvk_reserve"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().rvk_last_error().decode(errors="replace")
        raise RVKError(f"librvk error {rc}: {msg}")


def last_error() -> str:
    return load().rvk_last_error().decode(errors="replace")
