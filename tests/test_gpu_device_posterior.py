"""Device log-posterior (rvk_logpost: priors + conversion + likelihood + corrections on the GPU)
and the device-resident stretch move (rvk_stretch_run), against the reference and the host paths."""
import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation
from ravest_amd.posterior import LogPosterior
from ravest_amd.sampler import DeviceEnsembleSampler, EnsembleSampler
from tests._golden import assert_ll_close, load_case, logpost_cases

pytestmark = pytest.mark.gpu


def _posterior(case):
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    return LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                        np.array(m["unique_instruments"]), m["t0"])


@pytest.mark.parametrize("name", logpost_cases())
def test_device_posterior_vs_reference(name):
    """Every prior kind, Cases 1-3, jitter/conversion/prior masks: the reference's log_prob (goldens)."""
    case = load_case(name)
    dp = _posterior(case).device_posterior()
    got = dp(case["theta_free"])
    assert_ll_close(got, case["log_prob"], what=f"device-{name}")


@pytest.mark.parametrize("lpw", [16, 32])
def test_device_posterior_segmented_layouts(lpw):
    """The posterior epilogue in the 2- and 4-walkers-per-wave layouts (RVK_OPT_LPW)."""
    for name in ("cfg2", "n7", "case3"):
        case = load_case(name)
        lpost = _posterior(case)
        lpost.log_likelihood.engine.set_lanes_per_walker(lpw)
        assert_ll_close(lpost.device_posterior()(case["theta_free"]), case["log_prob"], what=f"lpw{lpw}-{name}")


@pytest.mark.parametrize("name", ["cfg3", "case3", "cfg4"])
def test_device_posterior_tensor_path_equals_host_path(name):
    import torch
    case = load_case(name)
    lpost = _posterior(case)
    dp = lpost.device_posterior()
    th = torch.from_numpy(np.ascontiguousarray(case["theta_free"])).cuda()
    out = torch.empty(th.shape[0], dtype=torch.float64, device="cuda")
    dp.device(th, out)
    torch.cuda.synchronize()
    dev = out.cpu().numpy()
    assert np.array_equal(dev, dp(case["theta_free"]), equal_nan=True)
    host = lpost.log_probability_batch(case["theta_free"])          # host priors + device likelihood
    assert_ll_close(dev, host, what=f"device-vs-host-{name}")


def _start(case, nw, seed):
    lpost = _posterior(case)
    ok = np.isfinite(case["log_prob"])
    x = case["theta_free"][ok]
    rng = np.random.default_rng(seed)
    x = x[rng.choice(len(x), nw, replace=len(x) < nw)]
    x = x + 1e-6 * np.abs(x) * rng.standard_normal(x.shape)
    good = np.isfinite(lpost.log_probability_batch(x))
    x[~good] = x[good][0]
    return lpost, x


@pytest.mark.parametrize("name", ["51peg", "case3"])
def test_device_sampler_reproduces_host_sampler(name):
    """rng='emcee': the device chain is the host sampler's chain (same RandomState stream)."""
    case = load_case(name)
    lpost, x0 = _start(case, 32, 3)
    host = EnsembleSampler(32, x0.shape[1], lpost.log_probability_batch, seed=np.random.RandomState(11))
    host.run_mcmc(x0, 40)
    dev = DeviceEnsembleSampler(lpost, 32, seed=np.random.RandomState(11), rng="emcee", steps_per_call=16)
    dev.run_mcmc(x0, 40)
    hc, dc = host.get_chain(), dev.get_chain()
    assert dc.shape == hc.shape == (40, 32, x0.shape[1])
    assert np.array_equal(host.naccepted, dev.naccepted)
    np.testing.assert_allclose(dc, hc, rtol=1e-12, atol=0)
    np.testing.assert_allclose(dev.get_log_prob(), host.get_log_prob(), rtol=1e-9, atol=1e-9)
    assert host.naccepted.sum() > 0


def test_device_sampler_philox_51peg():
    """Device RNG: reproducible for a seed, chain stays in the prior support, sane acceptance,
    and the stored log-probs are the posterior of the stored positions."""
    case = load_case("51peg")
    lpost, x0 = _start(case, 64, 5)
    a = DeviceEnsembleSampler(lpost, 64, seed=1234)
    a.run_mcmc(x0, 300)
    b = DeviceEnsembleSampler(lpost, 64, seed=1234, steps_per_call=64)
    b.run_mcmc(x0, 300)
    assert np.array_equal(a.get_chain(), b.get_chain())
    ch, lp = a.get_chain(), a.get_log_prob()
    assert np.all(np.isfinite(lp))
    assert 0.05 < a.acceptance_fraction.mean() < 0.9
    last = ch[-1]
    assert_ll_close(lp[-1], lpost.log_probability_batch(last), what="philox-last-step")
    # posterior mass near the data's answer: the period of 51 Peg b (4.23 d)
    names = case["meta"]["free_names"]
    if "P_b" in names:
        assert abs(np.median(ch[150:, :, names.index("P_b")]) - 4.2308) < 0.01


def test_device_sampler_nan_raises():
    case = load_case("cfg2")
    lpost, x0 = _start(case, 16, 7)
    x0[3, 0] = np.nan
    s = DeviceEnsembleSampler(lpost, 16, seed=1)
    with pytest.raises(ValueError):
        s.run_mcmc(x0, 2)


@pytest.mark.parametrize("name", logpost_cases())
def test_device_posterior_from_foreign_objects(name):
    """Built from ravest's OWN object types (tests/_foreign.py stand-ins: only the reference's
    public attributes), the device and host log-posteriors still equal the reference goldens."""
    from tests import _foreign as F
    case = load_case(name)
    lpost = LogPosterior(*F.posterior_args(case))
    assert_ll_close(lpost.device_posterior()(case["theta_free"]), case["log_prob"], what=f"foreign-device-{name}")
    assert_ll_close(lpost.log_probability_batch(case["theta_free"]), case["log_prob"], what=f"foreign-host-{name}")


def _fused_case(what, W):
    """Posteriors for the fused half-step: config 2 with every eccentricity prior kind (basic and
    transcendental), config 3 (3 planets, 2 instruments, D = 19), and the reference's Case-3
    posterior (Beta priors on e converted from secosw / sesinw, 2 planets, 2 instruments)."""
    from ravest_amd.synth import make_posterior
    if what == "case3":
        return _start(load_case("case3"), W, 13)
    cfg, prior = {"cfg2": (2, "uniform"), "cfg2_beta": (2, "beta"), "cfg2_rayleigh": (2, "rayleigh"),
                  "cfg2_vaneylen": (2, "vaneylen"), "cfg3": (3, "uniform")}[what]
    return make_posterior(cfg, W, seed=4, e_prior=prior)


@pytest.mark.parametrize("what,rng", [("cfg2", "philox"), ("cfg2", "emcee"), ("cfg2_beta", "philox"),
                                      ("cfg2_rayleigh", "philox"), ("cfg2_vaneylen", "emcee"), ("cfg3", "philox"),
                                      ("case3", "philox"), ("case3", "emcee")])
def test_fused_sampler_equals_two_kernel_path(monkeypatch, what, rng):
    """The fused half-step (proposals, full row, conversion and priors made lane-parallel in the
    likelihood kernel's prep) gives the same chain, log-probs and acceptances, bit for bit, as
    propose_kernel + the likelihood kernel (RVK_SAMPLER_FUSE=0): basic and transcendental prior
    kinds, D up to 19, the prior-side conversion."""
    W = 64 if what == "case3" else 256
    runs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("RVK_SAMPLER_FUSE", fuse)
        lpost, x0 = _fused_case(what, W)
        seed = np.random.RandomState(21) if rng == "emcee" else 99
        s = DeviceEnsembleSampler(lpost, W, seed=seed, rng=rng, steps_per_call=8)
        s.run_mcmc(x0, 24, skip_initial_state_check=(what == "case3"))
        runs.append((s.get_chain(), s.get_log_prob(), s.naccepted.copy()))
    (c1, l1, a1), (c0, l0, a0) = runs
    assert np.array_equal(c1, c0) and np.array_equal(l1, l0) and np.array_equal(a1, a0)
    assert a1.sum() > 0
    lpost, _ = _fused_case(what, W)
    assert_ll_close(l1[-1], lpost.log_probability_batch(c1[-1]), what=f"fused-{what}-last-step")


def test_many_planets_instruments_posterior_and_sampler():
    """10 planets and 20 instruments (the generic > 8-planet kernel; P_full = 92, so the
    two-kernel half-step): the device log-posterior equals the host path, and the device
    sampler reproduces the host stretch move draw for draw (emcee's RandomState stream)."""
    from ravest_amd.synth import make_dataset
    ds = make_dataset(10, 120, 20, seed=31, trend=False)
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    priors = {}
    for n in free:
        v, base = ds.truth[n], n.split("_")[0]
        priors[n] = (P.EccentricityUniform(0.99) if base == "e" else P.Uniform(-np.pi, np.pi) if base == "w"
                     else P.HalfNormal(5.0) if base == "jit" else P.Uniform(v - 0.5 * abs(v) - 1.0, v + 0.5 * abs(v) + 1.0))
    lpost = LogPosterior(ds.planet_letters, ds.parameterisation, priors, {"gd": 0.0, "gdd": 0.0}, free, ds.time,
                         ds.vel, ds.velerr, ds.instrument, ds.unique_instruments, ds.t0)
    rng = np.random.default_rng(3)
    x0 = np.array([ds.truth[n] for n in free])[None, :] * (1 + 1e-4 * rng.standard_normal((256, len(free))))
    dev = lpost.device_posterior()(x0)
    assert_ll_close(dev, lpost.log_probability_batch(x0), what="np10-ni20-device-vs-host")
    assert np.all(np.isfinite(dev))
    W = 256
    host = EnsembleSampler(W, len(free), lpost.log_probability_batch, seed=np.random.RandomState(5))
    host.run_mcmc(x0, 10)
    ds_ = DeviceEnsembleSampler(lpost, W, seed=np.random.RandomState(5), rng="emcee", steps_per_call=4)
    ds_.run_mcmc(x0, 10)
    assert np.array_equal(host.naccepted, ds_.naccepted)
    np.testing.assert_allclose(ds_.get_chain(), host.get_chain(), rtol=1e-12, atol=0)
