"""Batched quasi-periodic GP log-likelihood (rvk_gp, the opt-in "fp32+fp64" precision: fp32 MFMA
factorisation, BASELINE config 5) against the fp64 restatement of tinygp's DirectSolver path
(oracle/gp_oracle.py; parity unpinned at the tinygp boundary, see that module's header).  The
drop-in's default precision is fp64 (the reference's, fit.py:39), tested in test_gpu_gp64.py.

Tolerance (stated): |ll - ll64| <= 3e-8 n |ll64| + 1e-3 per walker (n epochs: the fp32 Cholesky's
backward error grows with n and the covariance's condition number), 2-30x the worst error
measured on each case (n = 1024: 1.3e-5 relative vs a 3.1e-5 bar; config 5, n = 512: 2.4e-6 vs
1.5e-5); identical -inf mask (invalid planets)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL_PER_EPOCH, ATOL = 3e-8, 1e-3


def _check(ll, ref, what, n):
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(ll), fin), f"{what}: mask differs"
    assert np.all(ll[~fin] == -np.inf)
    err = np.abs(ll[fin] - ref[fin])
    tol = RTOL_PER_EPOCH * n * np.abs(ref[fin]) + ATOL
    print(f"[{what}] max |d|/|ref| {np.max(err / np.abs(ref[fin])):.3e}, worst {np.max(err / tol):.3f} x tol")
    assert np.all(err <= tol), f"{what}: worst {np.max(err / tol):.2f} x tol, max abs err {err.max():.3g}"
    return float(np.max(err / np.abs(ref[fin])))


def _gp(ds, n_inst=1):
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    return GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments,
                           ds.planet_letters, ds.parameterisation, GPKernel("Quasiperiodic"), precision="fp32+fp64")


@pytest.mark.parametrize("n,np_,ni,par,trend", [(512, 1, 1, "P K e w Tp", False), (100, 1, 2, "P K e w Tc", True),
                                                (37, 2, 1, "P K secosw sesinw Tp", False),
                                                (300, 3, 3, "P K e w Tp", True),
                                                (32, 1, 1, "P K e w Tp", False),            # one tile
                                                (33, 1, 1, "P K e w Tp", False),            # one row of padding tiles
                                                (700, 1, 1, "P K e w Tp", False),           # 8-wave shape
                                                (1024, 2, 2, "P K secosw sesinw Tc", True)])  # maximum size
def test_gp_loglike_vs_fp64_oracle(n, np_, ni, par, trend):
    from oracle import gp_oracle
    from ravest_amd.synth import make_dataset, make_walkers
    ds = make_dataset(np_, n, ni, seed=50 + n, parameterisation=par, trend=trend)
    rng = np.random.default_rng(n)
    th = make_walkers(ds, 48, seed=n, scale=0.002)
    hy = np.column_stack([rng.uniform(2, 6, 48), rng.uniform(30, 120, 48), rng.uniform(0.3, 1.0, 48),
                          rng.uniform(10, 40, 48)])
    th[:, 5 * np_ + ni: 5 * np_ + 2 * ni] = np.abs(th[:, 5 * np_ + ni: 5 * np_ + 2 * ni])   # jitters >= 0
    gp = _gp(ds)
    ll = gp.batch(th, hy)
    ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, ni, np_, ds.parameterisation.code, ds.t0,
                               th, hy)
    _check(ll, ref, f"n{n}-np{np_}", n)
    assert np.isfinite(ref).sum() >= 40


def test_gp_bjd_times():
    """BJD-scale epochs (t ~ 2.46e6 d): the covariance's phase fractions and scaled times are
    formed in fp64 relative to the data, so fp32 keeps its precision."""
    from oracle import gp_oracle
    from ravest_amd.synth import make_dataset, make_walkers
    ds = make_dataset(1, 200, 1, seed=77, t_offset=2457000.25)
    rng = np.random.default_rng(77)
    th = make_walkers(ds, 32, seed=77, scale=0.002)
    th[:, 6] = np.abs(th[:, 6])
    hy = np.column_stack([rng.uniform(2, 6, 32), rng.uniform(30, 120, 32), rng.uniform(0.3, 1.0, 32),
                          rng.uniform(10, 40, 32)])
    ll = _gp(ds).batch(th, hy)
    ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th, hy)
    _check(ll, ref, "bjd", 200)


def test_gp_config5_shape_and_paths():
    """Config 5 at its BASELINE size (1 planet + GP, 512 epochs, 4096 walkers: 16 walker
    generations per CU, every workspace slot reused): host path == device path, repeatable,
    invalid planets -inf, and parity with the fp64 oracle on walkers from the first, a middle
    and the last generation."""
    import torch
    from oracle import gp_oracle
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(4096)
    gp = _gp(ds)
    a = gp.batch(th, hy)
    b = gp.batch(th, hy)
    assert np.array_equal(a, b, equal_nan=True)
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(len(th), dtype=torch.float64, device="cuda")
    gp.device(tt, ht, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), a, equal_nan=True)
    idx = np.r_[0:12, 2040:2048, 4084:4096, np.nonzero(~np.isfinite(a))[0][:8]]
    ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[idx], hy[idx])
    _check(a[idx], ref, "config5", 512)
    assert (~np.isfinite(a)).sum() > 0


def test_gp_reference_fixture_values():
    """The reference's own GP test data (tests/test_fit.py:1549-1575): finite, and the fp64 value
    at the drop-in's default precision (fp64) to the fp64 bar."""
    from oracle import gp_oracle
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    time = np.array([0.0, 1.0, 2.0, 3.0, 4.0, 5.0])
    vel = np.array([5.0, -2.0, -5.0, 2.0, 3.0, -2.0])
    velerr = np.array([1.0, 1.1, 0.9, 0.85, 1.5, 1.2])
    inst = np.array(["HARPS"] * 6)
    ll = GPLogLikelihood(time, vel, velerr, 2.0, inst, ["HARPS"], ["b"], "P K e w Tc", GPKernel("Quasiperiodic"))
    params = {"P_b": 2.0, "K_b": 5.0, "e_b": 0.0, "w_b": np.pi / 2, "Tc_b": 0.0, "g_HARPS": 0.0, "gd": 0.0,
              "gdd": 0.0, "jit_HARPS": 2.0}
    hyper = {"gp_amp": 1.0, "gp_lambda_e": 50.0, "gp_lambda_p": 0.5, "gp_period": 10.0}
    got = ll(params, hyper)
    assert np.isfinite(got)
    row = np.array([[params[n] for n in ll.names]])
    ref = gp_oracle.gp_loglike(time, vel, velerr, np.zeros(6, np.int32), 1, 1, 1, 2.0, row,
                               np.array([[1.0, 50.0, 0.5, 10.0]]))[0]
    assert ll.precision == "fp64"
    assert abs(got - ref) <= 1e-9 * max(1.0, abs(ref))
    bad = dict(params, P_b=-1.0)                 # tests/test_fit.py:1577-1600: invalid planet -> -inf
    assert ll(bad, hyper) == -np.inf


def test_gp_narrow_shape_matches(monkeypatch):
    """The 8-waves x 2-rows launch shape (experiment hook RVK_GP_NW=8) gives the same values as
    the default 4 x 4 shape up to fp32 summation order, and passes the oracle tolerance."""
    from oracle import gp_oracle
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(64)
    base = _gp(ds).batch(th, hy)
    monkeypatch.setenv("RVK_GP_NW", "8")
    narrow = _gp(ds).batch(th, hy)
    assert np.array_equal(np.isfinite(base), np.isfinite(narrow))
    fin = np.isfinite(base)
    assert np.max(np.abs(base[fin] - narrow[fin]) / np.abs(base[fin])) < 1e-4
    ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[:16], hy[:16])
    _check(narrow[:16], ref, "narrow", 512)
