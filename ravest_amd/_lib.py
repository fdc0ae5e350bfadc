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
_DEFAULT_PATH = LIB_PATH = os.path.join(_HERE, "lib", "librvk.so")
# experiment hook: A/B builds (tools/varbuild.sh, tools/ab_rev.sh); never set in production
LIB_PATH = os.environ.get("RAVEST_AMD_LIB", LIB_PATH)

# every symbol declared in include/rvk.h, include/rvk_post.h and include/rvk_gp.h
EXPORTS = ["rvk_create", "rvk_destroy", "rvk_loglike", "rvk_loglike_device", "rvk_reserve", "rvk_predict", "rvk_predict_device",
           "rvk_solve_kepler", "rvk_set_option", "rvk_stream", "rvk_sync", "rvk_device_count",
           "rvk_last_error", "rvk_version",
           "rvk_post_create", "rvk_post_destroy", "rvk_post_reserve", "rvk_logpost", "rvk_logpost_device",
           "rvk_stretch_run", "rvk_stretch_draws", "rvk_stretch_propose", "rvk_stretch_update", "rvk_stretch_table_read", "rvk_copy_to_host",
           "rvk_gp_create", "rvk_gp_destroy", "rvk_gp_loglike", "rvk_gp_loglike_device", "rvk_gp_set_precision",
           "rvk_gp_predict", "rvk_gp_predict_device", "rvk_gp_post_create", "rvk_gp_post_destroy",
           "rvk_gp_post_reserve", "rvk_gp_logpost", "rvk_gp_logpost_device", "rvk_gp_stretch_run",
           "rvk_gp_stretch_draws", "rvk_gp_stretch_propose", "rvk_gp_stretch_update"]

OPT_SOLVER = 1
OPT_GRAPH = 2
OPT_LPW = 3

PRED_TREND = 0x0100
PRED_GAMMA = 0x0200
PRED_ALL_PLANETS = 0x0400
MAX_PLANETS, MAX_INST = 32, 64


def pred_planet(p: int) -> int:
    """RVK_PRED_PLANET(p): include planet p (any index)."""
    return 0x0800 | (int(p) << 16)

# include/rvk_post.h
PRIOR_NPAR = 8
PRIOR_KIND = {"Uniform": 0, "EccentricityUniform": 1, "Normal": 2, "TruncatedNormal": 3, "HalfNormal": 4,
              "Rayleigh": 5, "VanEylen19Mixture": 6, "Beta": 7}


POST_CONVERT = 1
STRETCH_FIXED_SPLIT = 1   # include/rvk_post.h: RedBlueMove(randomize_split=False)
GP_QUASIPERIODIC = 0
GP_NHYPER = 4
# include/rvk_gp.h precision modes
GP_FP32, GP_FP32_FP64_FALLBACK, GP_FP64 = 0, 1, 2


def prior_src_default(planet: int, j: int) -> int:
    """RVK_PRIOR_SRC_DEFAULT: default parameter j (P K e w Tp) of planet `planet`, converted."""
    return -(1 + 5 * planet + j)

_lib = None


class _Tolerant:
    """Experiment hook only (RAVEST_AMD_LIB): wraps an older library so binding a symbol it lacks
    is a no-op; calling one raises AttributeError as usual."""

    class _Missing:
        argtypes = restype = None

    def __init__(self, lib) -> None:
        self.__dict__["_lib"] = lib

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            if name.startswith("rvk_"):
                return _Tolerant._Missing()
            raise


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
    if LIB_PATH != _DEFAULT_PATH:
        L = _Tolerant(L)     # A/B against an older build: symbols it lacks are skipped, not bound
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
    L.rvk_post_create.argtypes = [vp, C.c_int32, ip, dp, C.c_int32, ip, ip, dp, C.c_double, C.c_double, C.c_int32]
    L.rvk_post_create.restype = vp
    L.rvk_post_destroy.argtypes = [vp]
    L.rvk_post_destroy.restype = None
    L.rvk_post_reserve.argtypes = [vp, C.c_int64]
    L.rvk_logpost.argtypes = [vp, dp, C.c_int64, C.c_int64, dp]
    L.rvk_logpost_device.argtypes = [vp, vp, C.c_int64, C.c_int64, vp, vp]
    L.rvk_stretch_run.argtypes = [vp, vp, vp, C.c_int64, C.c_int32, C.c_double, C.c_uint64, C.c_uint64, C.c_int32,
                                  vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.rvk_stretch_draws.argtypes = [vp, C.c_int64, C.c_int32, C.c_double, C.c_uint64, C.c_uint64, C.c_int32, vp]
    L.rvk_stretch_propose.argtypes = [vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int64, C.c_int64, vp, vp]
    L.rvk_stretch_table_read.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
    L.rvk_copy_to_host.argtypes = [vp, vp, C.c_int64, C.c_int32, vp]
    L.rvk_stretch_update.argtypes = [vp, vp, vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp]
    L.rvk_gp_create.argtypes = [vp, C.c_int32]
    L.rvk_gp_create.restype = vp
    L.rvk_gp_destroy.argtypes = [vp]
    L.rvk_gp_destroy.restype = None
    L.rvk_gp_loglike.argtypes = [vp, dp, dp, C.c_int64, C.c_int64, C.c_int64, dp]
    L.rvk_gp_loglike_device.argtypes = [vp, vp, vp, C.c_int64, C.c_int64, C.c_int64, vp, vp]
    L.rvk_gp_set_precision.argtypes = [vp, C.c_int32]
    L.rvk_gp_predict.argtypes = [vp, dp, dp, C.c_int64, C.c_int64, C.c_int64, dp, C.c_int64, dp]
    L.rvk_gp_predict_device.argtypes = [vp, vp, vp, C.c_int64, C.c_int64, C.c_int64, vp, C.c_int64, vp, vp]
    L.rvk_gp_post_create.argtypes = [vp, C.c_int32, ip, dp, C.c_int32, C.c_int32, ip, ip, dp, C.c_double,
                                     C.c_double, C.c_int32]
    L.rvk_gp_post_create.restype = vp
    L.rvk_gp_post_destroy.argtypes = [vp]
    L.rvk_gp_post_destroy.restype = None
    L.rvk_gp_post_reserve.argtypes = [vp, C.c_int64]
    L.rvk_gp_logpost.argtypes = [vp, dp, C.c_int64, C.c_int64, dp]
    L.rvk_gp_logpost_device.argtypes = [vp, vp, C.c_int64, C.c_int64, vp, vp]
    L.rvk_gp_stretch_run.argtypes = list(L.rvk_stretch_run.argtypes or ())
    L.rvk_gp_stretch_draws.argtypes = list(L.rvk_stretch_draws.argtypes or ())
    L.rvk_gp_stretch_propose.argtypes = list(L.rvk_stretch_propose.argtypes or ())
    L.rvk_gp_stretch_update.argtypes = list(L.rvk_stretch_update.argtypes or ())
    for name in ("rvk_gp_loglike", "rvk_gp_loglike_device", "rvk_gp_set_precision", "rvk_gp_predict",
                 "rvk_gp_predict_device", "rvk_gp_post_reserve", "rvk_gp_logpost", "rvk_gp_logpost_device",
                 "rvk_gp_stretch_run", "rvk_gp_stretch_draws", "rvk_gp_stretch_propose", "rvk_gp_stretch_update",
                 "rvk_loglike", "rvk_loglike_device", "rvk_predict", "rvk_predict_device", "rvk_solve_kepler", "rvk_sync",
                 "rvk_set_option", "rvk_reserve", "rvk_post_reserve", "rvk_logpost", "rvk_logpost_device",
                 "rvk_stretch_run", "rvk_stretch_draws", "rvk_stretch_propose", "rvk_stretch_update",
                 "rvk_stretch_table_read", "rvk_copy_to_host"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


_fast = None


def fast() -> C.CDLL:
    """The per-call hot entry points (rvk_loglike, rvk_logpost, rvk_gp_logpost) bound with plain
    integer addresses (``addr``) instead of ctypes pointer objects: a few microseconds less per
    call on the host drop-in path, where the scalar log_probability(dict) of a MAP optimiser
    is latency-bound.  Same library, same functions."""
    global _fast
    if _fast is None:
        load()
        F = C.CDLL(LIB_PATH)
        vp, i64 = C.c_void_p, C.c_int64
        for name in ("rvk_loglike", "rvk_logpost", "rvk_gp_logpost"):
            getattr(F, name).argtypes = [vp, vp, i64, i64, vp]
            getattr(F, name).restype = C.c_int
        F.rvk_gp_loglike.argtypes = [vp, vp, vp, i64, i64, i64, vp]
        F.rvk_gp_loglike.restype = C.c_int
        _fast = F
    return _fast


def addr(a) -> int:
    """Data address of a NumPy array (cheaper than ``a.ctypes.data``)."""
    return a.__array_interface__["data"][0]


HOSTIO = {"auto": 0, "pageable": 1, "pinned": 2, "zerocopy": 3}   # include/rvk.h RVK_HOSTIO_*
OPT_HOSTIO = 4
OPT_LDS_POISON = 5


def check(rc: int) -> None:
    if rc != 0:
        msg = load().rvk_last_error().decode(errors="replace")
        raise RVKError(f"librvk error {rc}: {msg}")


def last_error() -> str:
    return load().rvk_last_error().decode(errors="replace")
