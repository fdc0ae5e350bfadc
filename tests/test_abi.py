"""The C-ABI library builds, loads and exports every symbol include/rvk.h declares (no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT


def _declared():
    names = set()
    for hdr in ("rvk.h", "rvk_post.h", "rvk_gp.h"):
        src = open(os.path.join(ROOT, "include", hdr)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"#define.*", "", src)
        names |= set(re.findall(r"\b(rvk_[a-z_]+)\s*\(", src))
    return sorted(names)


def test_header_and_library_agree():
    from ravest_amd import _lib
    L = _lib.load()
    declared = _declared()
    assert "rvk_loglike" in declared and "rvk_create" in declared
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, f"librvk.so lacks {missing}"
    assert sorted(_lib.EXPORTS) == declared


def test_version_and_errors_without_gpu():
    import torch
    from ravest_amd import _lib
    L = _lib.load()
    assert L.rvk_version() == 103          # 103: RVK_OPT_LDS_POISON value 2 (positive control)
    if torch.cuda.is_available():
        pytest.skip("this checks the no-device error path")
    t = np.linspace(0, 10, 8)
    dp = C.POINTER(C.c_double)
    h = L.rvk_create(t.ctypes.data_as(dp), t.ctypes.data_as(dp), t.ctypes.data_as(dp), None, 8, 1, 1, 0, 0.0, -1)
    assert not h
    assert _lib.last_error()          # a message, not a crash


def test_bad_arguments_fail_loudly():
    from ravest_amd import _lib
    L = _lib.load()
    dp = C.POINTER(C.c_double)
    t = np.linspace(0, 10, 8)
    # n_planets out of range is rejected before any device work
    h = L.rvk_create(t.ctypes.data_as(dp), t.ctypes.data_as(dp), t.ctypes.data_as(dp), None, 8, 1, 33, 0, 0.0, -1)
    assert not h and "n_planets" in _lib.last_error()
    h = L.rvk_create(t.ctypes.data_as(dp), t.ctypes.data_as(dp), t.ctypes.data_as(dp), None, 8, 2, 1, 0, 0.0, -1)
    assert not h and "inst_idx" in _lib.last_error()
    assert L.rvk_loglike(None, None, 1, 9, None) == -1
    # the posterior / sampler entry points check their arguments before touching a device
    assert not L.rvk_post_create(None, 1, None, None, 0, None, None, None, 0.0, 0.0, 0)
    assert "handle" in _lib.last_error()
    assert L.rvk_logpost_device(None, None, 1, 1, None, None) == -1
    assert L.rvk_stretch_run(None, None, None, 8, 1, 2.0, 0, 0, 0, None, None, None, None, None, None, None, None,
                             None) == -1
    assert L.rvk_stretch_draws(None, 8, 1, 2.0, 0, 0, 0, None) == -1
    assert L.rvk_stretch_propose(None, None, 8, 0, 0, 0, 4, None, None) == -1
    assert L.rvk_stretch_update(None, None, None, 8, 0, 0, None, None, None, None, None, None, None) == -1
    assert L.rvk_stretch_table_read(None, 0, 0, None, None, None) == -1
    assert not L.rvk_gp_create(None, 0) and "handle" in _lib.last_error()
    assert L.rvk_gp_loglike_device(None, None, None, 1, 9, 4, None, None) == -1


def test_engine_raises_without_library(monkeypatch, tmp_path):
    """The product path has no CPU fallback: a missing extension is an error."""
    from ravest_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(_lib.RVKError):
        _lib.load()
