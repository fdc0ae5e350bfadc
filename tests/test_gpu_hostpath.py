"""The north-star drop-in path: emcee (or MAP) calling LogPosterior.log_probability[_batch]
with host arrays (fit.py:1068-1075, 548-604).  Since round 4 it routes through the device
log-posterior (rvk_logpost) when every prior is built-in, and the blocking host calls move
their arrays by one of the RVK_OPT_HOSTIO transports.  Checked here:
  * every transport returns the same bits (same kernels, only the copies differ);
  * the routed path against the reference's log_prob goldens (the stated 1e-9 tolerance) and
    against the host-prior route (bitwise where the prior arithmetic has no transcendental,
    a few ulp otherwise -- both restate scipy's formulas);
  * the scalar log_probability(dict) equals the batch row bit for bit;
  * the host stretch move over the routed drop-in equals the same move over the host route.
"""
import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation
from ravest_amd.posterior import LogPosterior
from tests._golden import assert_ll_close, load_case, logpost_cases

pytestmark = pytest.mark.gpu

MODES = ("pageable", "pinned", "zerocopy", "auto")
_TRANS = ("Rayleigh", "VanEylen19Mixture", "Beta")


def _posterior(case, route="auto"):
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    return LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                        np.array(m["unique_instruments"]), m["t0"], route=route)


@pytest.mark.parametrize("name", logpost_cases())
def test_routed_drop_in_every_transport(name):
    case = load_case(name)
    lpost = _posterior(case)
    assert lpost.route == "device"
    x = case["theta_free"]
    outs = {}
    for mode in MODES:
        lpost.log_likelihood.engine.set_hostio(mode)
        outs[mode] = lpost.log_probability_batch(x)
    for mode in MODES[1:]:
        assert np.array_equal(outs[mode], outs["pageable"], equal_nan=True), mode
    assert_ll_close(outs["auto"], case["log_prob"], what=f"routed-{name}")
    # the device form on device tensors gives the same bits as the host-buffer call
    assert np.array_equal(lpost.device_posterior()(x), outs["auto"], equal_nan=True)
    # scalar log_prob_fn (emcee parameter_names / MAP): the batch row, bit for bit
    for i in range(min(8, len(x))):
        d = dict(zip(case["meta"]["free_names"], x[i]))
        v = lpost.log_probability(d)
        assert v == outs["auto"][i] or (np.isnan(v) and np.isnan(outs["auto"][i]))


@pytest.mark.parametrize("name", logpost_cases())
def test_routed_equals_host_route(name):
    case = load_case(name)
    dev = _posterior(case, "auto")
    host = _posterior(case, "host")
    assert host.route == "host"
    x = case["theta_free"]
    a, b = dev.log_probability_batch(x), host.log_probability_batch(x)
    assert np.array_equal(np.isfinite(a), np.isfinite(b))
    kinds = {c for c, _ in case["meta"]["priors"].values()}
    fin = np.isfinite(b)
    if kinds.isdisjoint(_TRANS):
        assert np.array_equal(a, b, equal_nan=True), f"{name}: max |d| {np.max(np.abs(a[fin] - b[fin]))}"
    else:      # device log/log1p/exp vs glibc's: ulp-level, well inside the parity tolerance
        assert np.max(np.abs(a[fin] - b[fin]) / np.maximum(1, np.abs(b[fin]))) <= 1e-14


def test_custom_prior_keeps_host_route():
    case = load_case("cfg2")
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    k0 = next(iter(priors))
    inner = priors[k0]
    priors[k0] = lambda v: inner(v)           # a user callable: no device form
    lpost = LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                         m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                         np.array(m["unique_instruments"]), m["t0"])
    assert lpost.route == "host"
    assert_ll_close(lpost.log_probability_batch(case["theta_free"]), case["log_prob"], what="custom-prior")


def test_host_stretch_move_routed_equals_host_route():
    """emcee's move (host, RandomState order) over the routed drop-in and over the host route."""
    from ravest_amd.sampler import EnsembleSampler
    from ravest_amd.synth import make_posterior
    lp_dev, x0 = make_posterior(2, 64, device=0)
    lp_host, _ = make_posterior(2, 64, device=0)
    lp_host._route = "host"
    a = EnsembleSampler(64, x0.shape[1], lp_dev.log_probability_batch, seed=5)
    b = EnsembleSampler(64, x0.shape[1], lp_host.log_probability_batch, seed=5)
    a.run_mcmc(x0, 30)
    b.run_mcmc(x0, 30)
    assert np.array_equal(a.get_chain(), b.get_chain())
    assert np.array_equal(a.get_log_prob(), b.get_log_prob())
    assert np.array_equal(a.naccepted, b.naccepted) and a.naccepted.sum() > 0


def test_gp_routed_drop_in():
    from tests.test_gpu_gp64 import RTOL64, _gp_cases, _gpost, _load_gp_case
    for name in _gp_cases():
        c = _load_gp_case(name)
        gp = _gpost(c, "fp64")
        assert gp.route == "device"
        got = {}
        for mode in MODES:
            gp.gp_log_likelihood.engine.set_hostio(mode)
            got[mode] = gp.log_probability_batch(c["x"])
        for mode in MODES[1:]:
            assert np.array_equal(got[mode], got["pageable"], equal_nan=True), (name, mode)
        assert_ll_close(got["auto"], c["log_prob"], RTOL64, f"gp routed {name}")
        gp._route = "host"
        assert_ll_close(gp.log_probability_batch(c["x"]), got["auto"], 1e-12, f"gp host route {name}")
        # the GP likelihood's own host call, every transport
        th, hy = gp._pp._full(c["x"][:, :len(gp.free_params_names)]), gp._split(c["x"])[2]
        ll = {}
        for mode in MODES:
            gp.gp_log_likelihood.engine.set_hostio(mode)
            ll[mode] = gp.gp_log_likelihood.batch(th, hy)
        for mode in MODES[1:]:
            assert np.array_equal(ll[mode], ll["pageable"], equal_nan=True), (name, mode)


def test_engine_loglike_every_transport_large():
    """rvk_loglike above the zero-copy threshold (auto -> pinned DMA) and below it."""
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    ds = make_config(3, n_walkers=8192)          # 8192 x 19 x 8 B = 1.2 MB > 1 MB
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), len(ds.planet_letters),
                   ds.parameterisation, ds.t0, device=0)
    res = {}
    for mode in MODES:
        eng.set_hostio(mode)
        res[mode] = (eng.loglike(ds.theta), eng.loglike(ds.theta[:3]))
    for mode in MODES[1:]:
        assert np.array_equal(res[mode][0], res["pageable"][0])
        assert np.array_equal(res[mode][1], res["pageable"][1])
    assert np.array_equal(res["auto"][1], res["auto"][0][:3])


@pytest.mark.parametrize("name", logpost_cases())
def test_one_kernel_logpost_equals_two_kernel_path(name, monkeypatch):
    """rvk_logpost_device runs as ONE kernel (the fused sampler's lane-parallel prep on the given
    coordinates) when the posterior fits the fused limits; RVK_LOGPOST_FUSE=0 keeps the two-kernel
    form (logprior_kernel + the likelihood's posterior epilogue).  Same bits, every golden."""
    case = load_case(name)
    x = case["theta_free"]
    one = _posterior(case).device_posterior()(x)
    monkeypatch.setenv("RVK_LOGPOST_FUSE", "0")
    two = _posterior(case).device_posterior()(x)
    assert np.array_equal(one, two, equal_nan=True)
    assert_ll_close(one, case["log_prob"], what=f"one-kernel-{name}")


def test_threads_share_one_posterior():
    """Two Python threads drive the routed drop-in of ONE posterior (and the engine under it) at
    once, as a thread-pool log_prob_fn would (fit.py:1068-1075; ctypes releases the GIL in the
    call): the handle's mutex serialises the blocking calls that share its stream and staging,
    so every result equals the single-threaded one bit for bit (include/rvk.h, Threading)."""
    import threading
    case = load_case("cfg2")
    lpost = _posterior(case)
    assert lpost.route == "device"
    x = case["theta_free"]
    halves = (x[: len(x) // 2], x[len(x) // 2:])
    ref_b = [lpost.log_probability_batch(h) for h in halves]
    names = case["meta"]["free_names"]
    ref_d = [lpost.log_probability(dict(zip(names, h[0]))) for h in halves]
    eng = lpost.log_likelihood.engine
    full = lpost._full(x)
    ref_e = eng.loglike(full) if full is not None else None
    errors = []

    def work(k):
        try:
            for it in range(150):
                b = lpost.log_probability_batch(halves[k])
                if not np.array_equal(b, ref_b[k], equal_nan=True):
                    errors.append((k, it, "batch"))
                d = lpost.log_probability(dict(zip(names, halves[k][0])))
                if not (d == ref_d[k] or (np.isnan(d) and np.isnan(ref_d[k]))):
                    errors.append((k, it, "dict"))
                if ref_e is not None and it % 10 == 0 and not np.array_equal(eng.loglike(full), ref_e, equal_nan=True):
                    errors.append((k, it, "engine"))
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=work, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a thread hung"
    assert not errors, errors[:5]
