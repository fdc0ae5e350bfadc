"""Seeded random sweeps against the oracles, sized by environment variables so that one GPU call can run
a long sweep and commit its log (profiles/round6/sweep/), while the default run stays short.

  * Keplerian log-likelihood (rvk_loglike and rvk_loglike_device) against the C oracle: the shapes of
    tests/test_gpu_parity.py::_random_shapes drawn from another seed; same tolerance (1e-9 relative,
    identical -inf masks), host-buffer and device-resident results bitwise equal.
    RVK_SWEEP_LL (default 16) shapes, RVK_SWEEP_SEED (default 7).
  * fp64 GP log-likelihood against oracle/gp_oracle.py (parity unpinned at tinygp, see its header):
    n drawn over 1 .. 1200 with the kernel-shape edges (32/33, 512/513, 1120/1121) over-sampled, 1-3
    planets, 1-3 instruments; 1e-9 relative, identical masks.  RVK_SWEEP_GP (default 4) shapes.
"""
import os

import numpy as np
import pytest

from tests._golden import assert_ll_close
from tests.test_gpu_parity import _random_shapes

pytestmark = pytest.mark.gpu

SEED = int(os.environ.get("RVK_SWEEP_SEED", "7"))
N_LL = int(os.environ.get("RVK_SWEEP_LL", "16"))
N_GP = int(os.environ.get("RVK_SWEEP_GP", "4"))


@pytest.mark.parametrize("k,np_,ni,n,W,par,trend", _random_shapes(N_LL, seed=10_000 + SEED))
def test_sweep_loglike_vs_oracle(k, np_, ni, n, W, par, trend):
    import torch
    from oracle import oracle
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_dataset, make_walkers
    ds = make_dataset(np_, n, ni, seed=5000 + 97 * SEED + k, parameterisation=par, trend=trend)
    th = make_walkers(ds, W, seed=6000 + 89 * SEED + k)
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, ni, np_, ds.parameterisation, ds.t0)
    ll = eng.loglike(th)
    ref, _ = oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, ni, np_, ds.parameterisation.code, ds.t0, th)
    err = assert_ll_close(ll, ref, what=f"sweep{SEED}-{k}-np{np_}-ni{ni}-n{n}-W{W}")
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    eng.loglike_device(torch.from_numpy(th).cuda(), out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ll.view(np.uint64))
    print(f"ll k={k} np={np_} ni={ni} n={n} W={W} par={par!r} trend={trend} max_rel_err={err:.3e}")


def _gp_shapes(count, seed):
    rng = np.random.default_rng(seed)
    pars = ["P K e w Tp", "P K e w Tc", "P K secosw sesinw Tp", "P K secosw sesinw Tc"]
    edges = [1, 32, 33, 512, 513, 1120, 1121]
    out = []
    for k in range(count):
        n = int(rng.choice(edges)) if rng.random() < 0.4 else int(rng.integers(1, 1201))
        np_ = int(rng.integers(1, 4))
        ni = int(min(n, rng.integers(1, 4)))
        out.append((k, np_, ni, n, pars[k % 4], bool(rng.integers(2))))
    return out


@pytest.mark.parametrize("k,np_,ni,n,par,trend", _gp_shapes(N_GP, seed=20_000 + SEED))
def test_sweep_gp64_vs_oracle(k, np_, ni, n, par, trend):
    from oracle import gp_oracle
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_dataset, make_walkers
    ds = make_dataset(np_, n, ni, seed=7000 + 97 * SEED + k, parameterisation=par, trend=trend)
    W = 12
    rng = np.random.default_rng(8000 + 89 * SEED + k)
    th = make_walkers(ds, W, seed=8000 + 89 * SEED + k, scale=0.002)
    th[:, 5 * np_ + ni: 5 * np_ + 2 * ni] = np.abs(th[:, 5 * np_ + ni: 5 * np_ + 2 * ni])
    hy = np.column_stack([rng.uniform(2, 6, W), rng.uniform(30, 120, W), rng.uniform(0.3, 1.0, W),
                          rng.uniform(10, 40, W)])
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments,
                         ds.planet_letters, ds.parameterisation, GPKernel("Quasiperiodic"), precision="fp64")
    ll = gp.batch(th, hy)
    ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, ni, np_, ds.parameterisation.code, ds.t0,
                               th, hy)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(ll), fin), f"gp sweep {k}: mask differs"
    assert np.all(ll[~fin] == ref[~fin]), f"gp sweep {k}: non-finite values differ"
    err = np.abs(ll[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
    mx = float(err.max()) if err.size else 0.0
    assert mx <= 1e-9, f"gp sweep {k} n={n}: max rel err {mx:.3e}"
    print(f"gp k={k} np={np_} ni={ni} n={n} par={par!r} trend={trend} finite={int(fin.sum())}/{W} max_rel_err={mx:.3e}")
