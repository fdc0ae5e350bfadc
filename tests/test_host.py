"""Host-side mirror of ravest's interface: priors, parameterisations, LogPosterior masks/priors.

CPU only.  The likelihood is NOT computed here: a stub engine returning 0 isolates the host
logic (scatter, jitter check, prior conversion, priors, corrections); the GPU tests compare the
full log-probability with the reference."""
import json
import pickle

import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation
from ravest_amd.posterior import LogPosterior, LogPrior
from tests._golden import GOLDEN, load_case, logpost_cases


def test_priors_vs_reference_grid():
    g = np.load(f"{GOLDEN}/priors.npz")
    spec = json.load(open(f"{GOLDEN}/priors.json"))
    for (cls, kw), ref in zip(spec, g["logp"]):
        p = getattr(P, cls)(**kw)
        vec = p.logpdf(g["x"])
        sca = np.array([p(float(x)) for x in g["x"]])
        np.testing.assert_array_equal(np.isfinite(vec), np.isfinite(ref))
        fin = np.isfinite(ref)
        np.testing.assert_allclose(vec[fin], ref[fin], rtol=1e-14, atol=1e-14, err_msg=cls)
        np.testing.assert_allclose(sca[fin], ref[fin], rtol=1e-14, atol=1e-14, err_msg=cls)


def test_beta_reference_json():
    """Reference tests/data/beta_reference.json (11 (a,b) cases x 101 points)."""
    for case in json.load(open(f"{GOLDEN}/beta_reference.json")):
        p = P.Beta(case["alpha"], case["beta"])
        x = np.array([r[0] for r in case["test_results"]])
        ref = np.array([r[1] if r[1] is not None else -np.inf for r in case["test_results"]], dtype=float)
        got = p.logpdf(x)
        fin = np.isfinite(ref)
        assert np.array_equal(np.isfinite(got), fin)
        np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-9, atol=1e-12)


def test_prior_validation_errors():
    with pytest.raises(ValueError):
        P.Uniform(1, 1)
    with pytest.raises(ValueError):
        P.EccentricityUniform(1.5)
    with pytest.raises(ValueError):
        P.Normal(0, 0)
    with pytest.raises(ValueError):
        P.VanEylen19Mixture(0.1, 0.2, 1.5)
    with pytest.raises(ValueError):
        P.Beta(0, 1)


def test_conversions_vs_reference():
    g = np.load(f"{GOLDEN}/convert.npz")
    par = Parameterisation("P K e w Tc")
    tp = np.array([par.convert_tc_to_tp(*a) for a in zip(g["tc"], g["per"], g["e"], g["w"])])
    np.testing.assert_array_equal(tp, g["tp"])
    tcb = np.array([par.convert_tp_to_tc(*a) for a in zip(g["tp"], g["per"], g["e"], g["w"])])
    np.testing.assert_array_equal(tcb, g["tc_back"])
    e, w = par.convert_secosw_sesinw_to_e_w(g["u"], g["v"])
    np.testing.assert_array_equal(e, g["e_uv"])
    np.testing.assert_array_equal(w, g["w_uv"])
    assert g["w_uv"][0] == np.pi           # sesinw = +0, secosw < 0 -> w = pi (invalid downstream)
    d, ok = Parameterisation("P K e w Tc").to_default_vec({"P": g["per"], "K": g["per"], "e": g["e"],
                                                           "w": g["w"], "Tc": g["tc"]})
    assert ok.all()
    np.testing.assert_array_equal(d["Tp"], g["tp"])
    with pytest.raises(ValueError):
        par.convert_tc_to_tp(0.0, 10.0, 1.0, 0.0)
    with pytest.raises(ValueError):
        Parameterisation("P K ecosw esinw Tp")


class _ZeroEngine:
    """Test double for the device engine: log-likelihood 0 for every walker."""
    def loglike(self, theta):
        return np.zeros(len(theta))


def _posterior(case, engine=None):
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    return LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                        np.array(m["unique_instruments"]), m["t0"], engine=engine or _ZeroEngine())


@pytest.mark.parametrize("name", logpost_cases())
def test_host_masks_priors_corrections(name):
    case = load_case(name)
    lpost = _posterior(case)
    m = case["meta"]
    assert lpost._logprob_jacobian_correction == m["jacobian"]
    assert lpost._logprob_prior_renorm_correction == m["renorm"]
    host = lpost.log_probability_batch(case["theta_free"])       # = lp + jac + renorm, or -inf
    ref_lp, ref_ll = case["log_prob"], case["log_like"]
    host_dead = ~np.isfinite(host)
    ref_dead = ~np.isfinite(ref_lp)
    assert not np.any(host_dead & ~ref_dead)                      # host never rejects a valid walker
    assert np.all(~np.isfinite(ref_ll[ref_dead & ~host_dead]))    # the rest are planet (likelihood) rejections
    fin = ~ref_dead
    np.testing.assert_allclose(host[fin], ref_lp[fin] - ref_ll[fin], rtol=0,
                               atol=1e-12 * np.maximum(1, np.abs(ref_ll[fin])).max())
    # the scalar drop-in agrees with the batch
    for i in range(min(8, len(host))):
        d = dict(zip(m["free_names"], case["theta_free"][i]))
        assert lpost.log_probability(d) == host[i] or (np.isneginf(host[i]) and np.isneginf(lpost.log_probability(d)))


def test_map_wrapper_and_pickle():
    case = load_case("cfg2")
    lpost = _posterior(case)
    row = case["theta_free"][0]
    assert lpost._negative_log_probability_for_MAP(list(row)) == -lpost.log_probability(
        dict(zip(lpost.free_params_names, row)))
    bad = row.copy()
    bad[lpost.free_params_names.index("jit_HARPS")] = -1.0
    assert lpost._negative_log_probability_for_MAP(list(bad)) == 1e30
    clone = pickle.loads(pickle.dumps(lpost.log_likelihood))
    assert clone._engine is None                                   # device handle is rebuilt lazily


def test_logprior_sum_order_and_values():
    priors = {"K_b": P.Uniform(0, 10), "jit_HARPS": P.Uniform(0, 5)}
    lp = LogPrior(priors)
    assert np.isclose(lp({"K_b": 5.0, "jit_HARPS": 2.5}), -np.log(10) - np.log(5))   # test_fit.py:520-532
    assert lp({"K_b": -5.0, "jit_HARPS": 2.0}) == -np.inf
    b = lp.batch({"K_b": np.array([5.0, -5.0]), "jit_HARPS": np.array([2.5, 2.0])})
    assert b[0] == lp({"K_b": 5.0, "jit_HARPS": 2.5}) and b[1] == -np.inf


def test_unsupported_uv_priors_raise():
    case = load_case("cfg4")
    m = dict(case["meta"])
    pri = dict(m["priors"])
    pri["secosw_b"] = ["Normal", {"mean": 0.0, "std": 0.3}]
    m["priors"] = pri
    case = dict(case)
    case["meta"] = m
    with pytest.raises(NotImplementedError):
        _posterior(case)


def test_log_probability_dict_of_arrays_is_vectorised():
    """emcee with parameter_names AND vectorize=True passes {name: array[W]}: the same values as
    the batch form, one call."""
    case = load_case("cfg2")
    lpost = _posterior(case)
    x = case["theta_free"]
    d = {n: x[:, i] for i, n in enumerate(case["meta"]["free_names"])}
    got = lpost.log_probability(d)
    assert got.shape == (len(x),)
    assert np.array_equal(got, lpost.log_probability_batch(x), equal_nan=True)
    assert lpost.log_probability({n: float(v[0]) for n, v in d.items()}) == got[0] or np.isnan(got[0])


def test_prior_subclass_keeps_its_own_formula():
    """A user subclass of a built-in prior that overrides __call__ is a custom callable: the
    routed drop-in keeps the host-prior path (its formula), and it has no device form."""
    class HalfUniform(P.Uniform):
        def __call__(self, value):
            return super().__call__(value) - np.log(2.0)

    case = load_case("cfg2")
    m = case["meta"]
    k0 = next(iter(m["priors"]))
    lpost = _posterior(case)
    lpost.log_likelihood._engine, lpost._route = None, "auto"     # as with the real engine
    assert lpost.route == "device"
    c, kw = m["priors"][k0]
    sub = HalfUniform(**kw) if c == "Uniform" else None
    if sub is None:
        pytest.skip("the first prior of the case is not a Uniform")
    assert P.as_prior(sub) is sub and not P.is_builtin(sub)
    with pytest.raises(NotImplementedError):
        P.device_params(sub)
    np.testing.assert_array_equal(P.logpdf_vec(sub, np.array([0.5 * (kw["lower"] + kw["upper"])])),
                                  [P.Uniform(**kw)(0.5 * (kw["lower"] + kw["upper"])) - np.log(2.0)])
    priors = {k: (sub if k == k0 else getattr(P, cc)(**kk)) for k, (cc, kk) in m["priors"].items()}
    lp2 = LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                       m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                       np.array(m["unique_instruments"]), m["t0"], engine=_ZeroEngine())
    host = _posterior(case).log_probability_batch(case["theta_free"])
    sub_lp = lp2.log_probability_batch(case["theta_free"])
    fin = np.isfinite(host)
    np.testing.assert_allclose(sub_lp[fin], host[fin] - np.log(2.0), rtol=0, atol=1e-9)
    lp2.log_likelihood._engine, lp2._route = None, "auto"
    assert lp2.route == "host"
