"""fp64 GP factorisation (rvk_gp64.hip): the RVK_GP_FP64 precision mode, the fp64 fallback of
the fp32 path for covariances that are not positive definite in fp32, the GP-conditioned
posterior predictive, and the GP log-posterior (GPLogPosterior, fit.py:7596-7939) against the
reference's goldens.

Oracle: oracle/gp_oracle.py (fp64 scipy restatement of tinygp 0.3's DirectSolver and
GaussianProcess.condition; parity unpinned at the tinygp boundary, see its header).
Tolerances (stated):
  * fp64 log-likelihood:  |ll - ll64| <= 1e-9 max(1, |ll64|)   (same bar as the Keplerian path)
  * ill-conditioned fp64 (condition number ~1e9): |ll - ll64| <= 1e-6 max(1, |ll64|) -- both
    sides are fp64 Cholesky factorisations whose backward errors are amplified by kappa
  * conditional mean: |mu - mu64| <= 1e-8 max|mu64| per sample
  * GP log-posterior vs the reference goldens: fp64 1e-9 (as above; the drop-in's default
    precision); the opt-in fp32+fp64: 3e-8 n |ll| + 1e-3 (tests/test_gpu_gp.py)
"""
import json
import os

import numpy as np
import pytest

from tests._golden import GOLDEN

pytestmark = pytest.mark.gpu

RTOL64 = 1e-9


def _gp(ds, precision):
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    return GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments,
                           ds.planet_letters, ds.parameterisation, GPKernel("Quasiperiodic"), precision=precision)


def _oracle(ds, th, hy):
    from oracle import gp_oracle
    return gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments),
                                len(ds.planet_letters), ds.parameterisation.code, ds.t0, th, hy)


def _check(ll, ref, rtol, what):
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(ll), fin), f"{what}: mask differs"
    assert np.all(ll[~fin] == ref[~fin]), f"{what}: non-finite values differ"
    err = np.abs(ll[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
    assert err.size == 0 or err.max() <= rtol, f"{what}: max rel err {err.max():.3e} > {rtol:g}"
    return float(err.max()) if err.size else 0.0


def _walkers(ds, W, seed, **kw):
    from ravest_amd.synth import make_walkers
    rng = np.random.default_rng(seed)
    np_, ni = len(ds.planet_letters), len(ds.unique_instruments)
    th = make_walkers(ds, W, seed=seed, scale=0.002, **kw)
    th[:, 5 * np_ + ni: 5 * np_ + 2 * ni] = np.abs(th[:, 5 * np_ + ni: 5 * np_ + 2 * ni])
    hy = np.column_stack([rng.uniform(2, 6, W), rng.uniform(30, 120, W), rng.uniform(0.3, 1.0, W),
                          rng.uniform(10, 40, W)])
    return th, hy


@pytest.mark.parametrize("n,np_,ni,par,trend", [(512, 1, 1, "P K e w Tp", False), (100, 1, 2, "P K e w Tc", True),
                                                (37, 2, 1, "P K secosw sesinw Tp", False),
                                                (300, 3, 3, "P K e w Tp", True),
                                                (32, 1, 1, "P K e w Tp", False), (33, 1, 1, "P K e w Tp", False),
                                                (1, 1, 1, "P K e w Tp", False),
                                                (700, 1, 1, "P K e w Tp", False),
                                                (1024, 2, 2, "P K secosw sesinw Tc", True),
                                                (150, 10, 12, "P K e w Tc", True),   # > 8 planets
                                                # the kernel-shape edges (rvk_gp64.hip gp64_shape): 16 tile rows
                                                # with LDS slots | 17-35 in groups of three | 36+ in groups of five
                                                (513, 1, 1, "P K e w Tp", False), (1120, 1, 2, "P K e w Tc", True),
                                                (1121, 1, 1, "P K e w Tp", False)])
def test_fp64_loglike_vs_oracle(n, np_, ni, par, trend):
    from ravest_amd.synth import make_dataset
    ds = make_dataset(np_, n, ni, seed=150 + n, parameterisation=par, trend=trend)
    th, hy = _walkers(ds, 40, n)
    ll = _gp(ds, "fp64").batch(th, hy)
    ref = _oracle(ds, th, hy)
    _check(ll, ref, RTOL64, f"n{n}")
    assert np.isfinite(ref).sum() >= 30


def test_fp64_config5_full_size():
    """Config 5 at its BASELINE size in the drop-in's default precision (fp64, 512 epochs, 4096
    walkers: 16 walker generations per CU through the per-CU workspace): host path == device
    path, repeatable, and the fp64 oracle on walkers of the first, a middle and the last
    generation, plus the masked ones."""
    import torch
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(4096)
    gp = _gp(ds, "fp64")
    a = gp.batch(th, hy)
    assert np.array_equal(a, gp.batch(th, hy), equal_nan=True)
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(len(th), dtype=torch.float64, device="cuda")
    gp.device(tt, ht, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), a, equal_nan=True)
    idx = np.r_[0:8, 2044:2052, 4088:4096, np.nonzero(~np.isfinite(a))[0][:6]]
    _check(a[idx], _oracle(ds, th[idx], hy[idx]), RTOL64, "config 5 fp64, 4096 walkers")
    assert (~np.isfinite(a)).sum() > 0 and np.isfinite(a).sum() > 0.9 * len(a)


def test_fp64_bjd_times():
    """BJD-scale epochs: tau = t_i - t_j is formed in fp64 exactly as the reference forms it."""
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 200, 1, seed=177, t_offset=2457000.25)
    th, hy = _walkers(ds, 24, 177)
    _check(_gp(ds, "fp64").batch(th, hy), _oracle(ds, th, hy), RTOL64, "bjd")


def _ill_conditioned():
    """A covariance with condition number ~1e9: large gp_amp, long lambda_e, small velerr and
    zero jitter over 300 epochs -- fp32 cannot factor it, fp64 can (and the reference, in fp64,
    returns a finite log-likelihood)."""
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 300, 1, seed=91)
    ds.velerr = np.full_like(ds.velerr, 0.02)
    th, hy = _walkers(ds, 24, 91)
    th[:, 6] = 0.0                                        # jit = 0
    hy[:, 0] = 40.0                                       # gp_amp
    hy[:, 1] = 2000.0                                     # lambda_e
    hy[:, 2] = 2.0                                        # lambda_p
    return ds, th, hy


def test_fp32_fallback_to_fp64_on_ill_conditioned_covariance():
    ds, th, hy = _ill_conditioned()
    ref = _oracle(ds, th, hy)
    assert np.isfinite(ref).sum() >= 20, "the fp64 oracle must factor these"
    ll32 = _gp(ds, "fp32").batch(th, hy)
    nan32 = np.isnan(ll32)
    assert nan32.sum() >= 5, "the case must defeat the fp32 factorisation"
    llfb = _gp(ds, "fp32+fp64").batch(th, hy)
    ll64 = _gp(ds, "fp64").batch(th, hy)
    assert not np.isnan(llfb[np.isfinite(ref)]).any(), "fallback left NaN where fp64 is finite"
    # the fallback re-evaluates exactly the fp32 NaN walkers with the fp64 kernel: same bits as fp64 mode
    assert np.array_equal(llfb[nan32], ll64[nan32], equal_nan=True)
    assert np.array_equal(llfb[~nan32], ll32[~nan32])
    _check(ll64, ref, 1e-6, "ill-conditioned fp64")


def test_fallback_device_path_and_graph_capture():
    """The fallback needs no host round trip: the device form is stream-ordered and capturable."""
    import torch
    ds, th, hy = _ill_conditioned()
    gp = _gp(ds, "fp32+fp64")
    host = gp.batch(th, hy)
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(len(th), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    gp.device(tt, ht, out, s)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy(), host, equal_nan=True)
    g = torch.cuda.CUDAGraph()
    out.fill_(0.0)
    with torch.cuda.graph(g, stream=s):
        gp.device(tt, ht, out, s)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), host, equal_nan=True)


def test_not_positive_definite_in_fp64_is_nan():
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 64, 1, seed=5)
    ds.velerr = np.zeros_like(ds.velerr)
    th, hy = _walkers(ds, 8, 5)
    th[:, 6] = 0.0
    hy[:, 1] = 1e7                                        # rank-deficient: K ~ amp^2 * periodic, no diagonal
    hy[:, 2] = 1e3
    ll = _gp(ds, "fp64").batch(th, hy)
    ref = _oracle(ds, th, hy)
    assert np.isnan(ref).all() and np.isnan(ll).all()


# ---- GP-conditioned posterior predictive -----------------------------------------------------

@pytest.mark.parametrize("n,np_,ni,par,T", [(120, 1, 1, "P K e w Tp", 300), (200, 2, 2, "P K secosw sesinw Tc", 97),
                                             (33, 1, 1, "P K e w Tc", 1), (520, 1, 1, "P K e w Tp", 64),
                                             (1120, 1, 1, "P K e w Tp", 33)])
def test_gp_condition_vs_oracle(n, np_, ni, par, T):
    from oracle import gp_oracle
    from ravest_amd.synth import make_dataset
    ds = make_dataset(np_, n, ni, seed=300 + n, parameterisation=par, trend=True)
    th, hy = _walkers(ds, 20, n)
    th[3, 2] = 1.5                                        # invalid planet: NaN row
    tq = np.linspace(ds.time.min() - 20, ds.time.max() + 20, T)
    got = _gp(ds, "fp64").condition(th, hy, tq)
    ref = gp_oracle.gp_condition(ds.time, ds.vel, ds.velerr, ds.inst_idx, ni, np_, ds.parameterisation.code, ds.t0,
                                 th, hy, tq)
    assert np.array_equal(np.isnan(got).all(axis=1), np.isnan(ref).all(axis=1))
    assert np.isnan(got[3]).all()
    ok = ~np.isnan(ref).all(axis=1)
    scale = np.max(np.abs(ref[ok]), axis=1, keepdims=True)
    assert np.all(np.abs(got[ok] - ref[ok]) <= 1e-8 * scale)


def test_gp_predictive_api_total_and_freeze():
    """GPPosteriorPredictive: rv_gp_from_samples / rv_total_from_samples / *_custom against the
    oracle (fit.py:7342-7425, 7494-7594), and freeze_params (fit.py:7137-7302)."""
    from oracle import gp_oracle
    from ravest_amd.gp import GPKernel, HYPERPARAMS
    from ravest_amd.predictive import GPPosteriorPredictive
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 150, 1, seed=404, trend=True)
    th, hy = _walkers(ds, 30, 404, frac_invalid=0.0)
    free = ["P_b", "K_b", "e_b", "w_b", "Tp_b", "g_HARPS", "jit_HARPS"]
    fixed = {n: float(ds.truth[n]) for n in ds.names if n not in free}
    th[:, ds.names.index("gd")] = fixed["gd"]
    th[:, ds.names.index("gdd")] = fixed["gdd"]
    fh = ["gp_amp", "gp_lambda_e", "gp_period"]
    hy[:, 2] = 0.7
    pp = GPPosteriorPredictive(ds.planet_letters, ds.parameterisation, fixed, free, {"gp_lambda_p": 0.7}, fh, ds.time,
                               ds.vel, ds.velerr, ds.instrument, ds.unique_instruments, ds.t0,
                               GPKernel("Quasiperiodic"))
    samples = np.concatenate([th[:, [ds.names.index(n) for n in free]],
                              hy[:, [HYPERPARAMS.index(k) for k in fh]]], axis=1)
    tq = np.linspace(-10, 1010, 211)
    gpc = pp.rv_gp_from_samples(tq, samples)
    ref = gp_oracle.gp_condition(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th, hy, tq)
    assert np.all(np.abs(gpc - ref) <= 1e-8 * np.max(np.abs(ref), axis=1, keepdims=True))
    tot = pp.rv_total_from_samples(tq, samples)
    parts = pp.rv_trend_from_samples(tq, samples) + pp.rv_planet_from_samples("b", tq, samples) + gpc
    assert np.max(np.abs(tot - parts)) <= 1e-9 * np.max(np.abs(tot))
    params = dict(zip(ds.names, th[4])) | dict(zip(HYPERPARAMS, hy[4]))
    assert np.allclose(pp.rv_gp_custom(tq, params), gpc[4], rtol=0, atol=1e-12 * np.max(np.abs(gpc[4])))
    assert np.allclose(pp.rv_total_custom(tq, params), tot[4], rtol=0, atol=1e-9 * np.max(np.abs(tot[4])))
    # freeze_params: P at a value, Tp at its posterior median
    med = float(np.median(samples[:, free.index("Tp_b")]))
    fr = pp.rv_planet_from_samples("b", tq, samples, freeze_params={"P_b": 12.5, "Tp_b": None})
    s2 = samples.copy()
    s2[:, free.index("P_b")] = 12.5
    s2[:, free.index("Tp_b")] = med
    assert np.array_equal(fr, pp.rv_planet_from_samples("b", tq, s2))
    with pytest.raises(ValueError):
        pp.rv_planet_from_samples("b", tq, samples, freeze_params={"Tc_b": 1.0})
    bad = samples.copy()
    bad[2, free.index("e_b")] = 1.2
    with pytest.raises(ValueError):
        pp.rv_gp_from_samples(tq, bad)


# ---- GP log-posterior vs the reference (tools/gen_golden.py gen_gp_logpost) -----------------------

def _gp_cases():
    import glob
    return sorted(os.path.basename(f)[7:-4] for f in glob.glob(os.path.join(GOLDEN, "gppost_*.npz")))


def _load_gp_case(name):
    d = np.load(os.path.join(GOLDEN, f"gppost_{name}.npz"))
    out = {k: d[k] for k in d.files if k != "meta"}
    out["meta"] = json.loads(str(d["meta"]))
    return out


def _gpost(c, precision, foreign=False):
    from ravest_amd import prior as P
    from ravest_amd.gp import GPKernel, GPLogPosterior
    m = c["meta"]
    mod = P
    if foreign:
        from tests import _foreign as mod
    priors = {k: getattr(mod, cls)(**kw) for k, (cls, kw) in m["priors"].items()}
    hyperpriors = {k: getattr(mod, cls)(**kw) for k, (cls, kw) in m["hyperpriors"].items()}
    par = m["parameterisation"]
    if foreign:
        par = mod.Parameterisation(par)
    return GPLogPosterior(m["planet_letters"], par, GPKernel("Quasiperiodic"), priors, hyperpriors, m["fixed"],
                          m["fixed_hyper"], m["free_names"], m["free_hyper"], c["time"], c["vel"], c["velerr"],
                          m["t0"], c["instrument"], m["unique_instruments"],
                          **({} if precision is None else {"precision": precision}))


@pytest.mark.parametrize("name", _gp_cases())
def test_gp_logpost_vs_reference(name):
    from tests._golden import assert_ll_close
    c = _load_gp_case(name)
    gp64 = _gpost(c, "fp64")
    assert gp64._logprob_jacobian_correction == c["meta"]["jacobian"]
    assert gp64._logprob_prior_renorm_correction == c["meta"]["renorm"]
    assert_ll_close(gp64.log_probability_batch(c["x"]), c["log_prob"], RTOL64, f"{name} host fp64")
    dev = gp64.device_posterior()
    assert_ll_close(dev(c["x"]), c["log_prob"], RTOL64, f"{name} device fp64")
    d = dict(zip(c["meta"]["free_names"] + c["meta"]["free_hyper"], c["x"][0]))
    assert gp64.log_probability(d) == pytest.approx(c["log_prob"][0], rel=RTOL64, abs=RTOL64)
    # the drop-in's default precision is the reference's fp64
    assert _gpost(c, None).gp_log_likelihood.precision == "fp64"
    # opt-in precision (fp32 factorisation + fp64 fallback): the fp32 tolerance
    gpd = _gpost(c, "fp32+fp64").device_posterior()(c["x"])
    fin = np.isfinite(c["log_prob"])
    assert np.array_equal(np.isfinite(gpd), fin)
    ll = c["log_like"][fin]
    assert np.all(np.abs(gpd[fin] - c["log_prob"][fin]) <= 3e-8 * len(c["time"]) * np.abs(ll) + 1e-3)


def test_gp_logpost_foreign_objects_and_device_tensor():
    """ravest's own prior / Parameterisation objects (duck-typed stand-ins, tests/_foreign.py) at
    the GP drop-in, and the torch-tensor device form."""
    import torch
    c = _load_gp_case("b")
    gp = _gpost(c, "fp64", foreign=True)
    ref = c["log_prob"]
    from tests._golden import assert_ll_close
    assert_ll_close(gp.log_probability_batch(c["x"]), ref, RTOL64, "foreign host")
    dev = gp.device_posterior()
    x = torch.from_numpy(np.ascontiguousarray(c["x"])).cuda()
    out = torch.empty(len(x), dtype=torch.float64, device="cuda")
    dev.device(x, out)
    torch.cuda.synchronize()
    assert_ll_close(out.cpu().numpy(), ref, RTOL64, "foreign device")


def test_gp_device_sampler_matches_host_sampler():
    """The device GP stretch move (rvk_gp_stretch_run, GPFitter.run_mcmc's sampler) with emcee's
    RandomState draws reproduces the host stretch move over GPLogPosterior.log_probability_batch
    draw for draw (fp64 precision: the same log-posterior code path on both sides)."""
    from ravest_amd.sampler import DeviceEnsembleSampler, EnsembleSampler
    c = _load_gp_case("a")
    gp = _gpost(c, "fp64")
    fin = np.isfinite(c["log_prob"])
    x0 = c["x"][fin][:32].copy()
    W = 32
    host = EnsembleSampler(W, x0.shape[1], gp.log_probability_batch, seed=np.random.RandomState(3))
    host.run_mcmc(x0, 12)
    dev = DeviceEnsembleSampler(gp, W, seed=np.random.RandomState(3), rng="emcee", steps_per_call=5)
    dev.run_mcmc(x0, 12)
    assert np.array_equal(host.naccepted, dev.naccepted)
    np.testing.assert_allclose(dev.get_chain(), host.get_chain(), rtol=1e-12, atol=0)
    np.testing.assert_allclose(dev.get_log_prob(), host.get_log_prob(), rtol=1e-9, atol=1e-9)
    assert host.naccepted.sum() > 0
    ph = DeviceEnsembleSampler(gp, W, seed=7)           # device Philox draws
    ph.run_mcmc(x0, 6)
    assert np.all(np.isfinite(ph.get_log_prob()))


@pytest.mark.parametrize("n,np_,ni", [(1500, 1, 1), (2048, 2, 2), (4096, 1, 1)])
def test_fp64_above_the_fp32_limit(n, np_, ni):
    """n > 1024 (the fp32 kernel's LDS panel limit): the fp64 factorisation with its accumulator
    rows grouped through the workspace, fp64 1e-9 against the oracle; the fp32 modes run the
    same fp64 kernel there (identical values)."""
    from ravest_amd.synth import make_dataset
    ds = make_dataset(np_, n, ni, seed=500 + n, trend=True)
    th, hy = _walkers(ds, 6 if n > 2048 else 12, n)
    ll = _gp(ds, "fp64").batch(th, hy)
    ref = _oracle(ds, th, hy)
    _check(ll, ref, RTOL64, f"n{n}")
    assert np.isfinite(ref).sum() >= len(ref) - 2
    assert np.array_equal(_gp(ds, "fp32+fp64").batch(th, hy), ll, equal_nan=True)
    assert np.array_equal(_gp(ds, "fp32").batch(th, hy), ll, equal_nan=True)


def test_gp_condition_above_the_fp32_limit():
    from oracle import gp_oracle
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 1500, 1, seed=1501, trend=True)
    th, hy = _walkers(ds, 6, 1501)
    tq = np.linspace(ds.time.min() - 5, ds.time.max() + 5, 120)
    got = _gp(ds, "fp64").condition(th, hy, tq)
    ref = gp_oracle.gp_condition(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th, hy, tq)
    ok = ~np.isnan(ref).all(axis=1)
    assert np.array_equal(np.isnan(got).all(axis=1), ~ok)
    scale = np.max(np.abs(ref[ok]), axis=1, keepdims=True)
    assert np.all(np.abs(got[ok] - ref[ok]) <= 1e-8 * scale)


def test_gp_condition_analytic_properties_device():
    """GP conditioning on the device (RVK_GP_FP64 COND kernel), checked by properties of
    GaussianProcess.condition that need no tinygp (its parity is unpinned):
    mu = K(tq, t) (K + diag)^-1 r is linear in the residuals r = vel - mean(theta), reproduces r
    at the data times as the diagonal vanishes, and goes to 0 as the noise grows."""
    from oracle import gp_oracle
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 60, 1, seed=61)
    th, hy = _walkers(ds, 3, 61, frac_invalid=0.0)
    hy[:] = [4.0, 80.0, 0.6, 25.0]
    m = gp_oracle.mean_model(ds.time, ds.inst_idx, 1, 1, ds.parameterisation.code, ds.t0, th[0])
    tq = np.linspace(ds.time.min(), ds.time.max(), 50)
    rng = np.random.default_rng(62)
    ra, rb = rng.normal(0, 5, ds.time.size), rng.normal(0, 5, ds.time.size)

    def cond(vel, velerr, thr, tq_):
        from ravest_amd.gp import GPKernel, GPLogLikelihood
        g = GPLogLikelihood(ds.time, vel, velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                            ds.parameterisation, GPKernel("Quasiperiodic"), precision="fp64")
        return g.condition(thr, hy[:len(thr)], tq_)

    # linearity: r_a + r_b -> mu_a + mu_b (same theta, same diagonal)
    mua, mub, muc = (cond(m + r, ds.velerr, th[:1], tq)[0] for r in (ra, rb, ra + rb))
    assert np.max(np.abs(muc - (mua + mub))) <= 1e-9 * np.max(np.abs(muc))
    # interpolation: a vanishing diagonal (velerr 1e-4, jitter 0) reproduces the residuals at the data times
    th0 = th[:1].copy()
    th0[0, 6] = 0.0                                       # jit_HARPS
    mu0 = cond(m + ra, np.full(ds.time.size, 1e-4), th0, ds.time)[0]
    assert np.max(np.abs(mu0 - ra)) <= 1e-3 * np.max(np.abs(ra))
    # noise limit: sigma = 1e6 -> mu ~ K r / sigma^2, far below the residuals
    mu_big = cond(m + ra, np.full(ds.time.size, 1e6), th0, tq)[0]
    assert np.max(np.abs(mu_big)) <= 1e-9 * np.max(np.abs(ra)) * ds.time.size * hy[0, 0] ** 2
