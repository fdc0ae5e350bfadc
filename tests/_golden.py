"""Helpers to read the golden fixtures (tests/golden/, made by tools/gen_golden.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# parity tolerance: per-walker fp64 log-prob |d| <= 1e-9 * max(1, |ref|)
LL_RTOL = 1e-9
# the C oracle restates the reference op-for-op: it is pinned much tighter
ORACLE_RTOL = 1e-11


def logpost_cases():
    return sorted(os.path.basename(f)[8:-4] for f in glob.glob(os.path.join(GOLDEN, "logpost_*.npz")))


def load_case(name):
    d = np.load(os.path.join(GOLDEN, f"logpost_{name}.npz"))
    out = {k: d[k] for k in d.files if k != "meta"}
    out["meta"] = json.loads(str(d["meta"]))
    return out


def assert_ll_close(got, ref, rtol=LL_RTOL, what=""):
    got = np.asarray(got); ref = np.asarray(ref)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin), f"{what}: -inf mask differs at {np.nonzero(np.isfinite(got) != fin)[0][:10]}"
    assert np.all(got[~fin] == -np.inf), f"{what}: masked values must be -inf (never NaN)"
    err = np.abs(got[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
    assert err.size == 0 or err.max() <= rtol, f"{what}: max rel err {err.max():.3e} > {rtol:g}"
    return float(err.max()) if err.size else 0.0
