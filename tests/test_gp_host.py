"""GPKernel mirror (gp.py) and the fp64 GP oracle on CPU."""
import numpy as np
import pytest

from ravest_amd.gp import GPKernel, QuasiperiodicKernel
from ravest_amd.param import Parameter


def test_gpkernel_types_and_validation():
    """Reference tests/test_gp.py:11-120 semantics."""
    k = GPKernel("Quasiperiodic")
    assert k.get_expected_hyperparams() == ["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"]
    with pytest.raises(ValueError):
        GPKernel("SquaredExponential")
    good = {n: Parameter(v, "") for n, v in zip(k.expected_hyperparams, [1.0, 50.0, 0.5, 10.0])}
    k.validate_hyperparams(good)
    with pytest.raises(ValueError):
        k.validate_hyperparams({n: p for n, p in good.items() if n != "gp_amp"})
    with pytest.raises(ValueError):
        k.validate_hyperparams(dict(good, extra=Parameter(1.0, "")))
    for bad in (0.0, -1.0, np.inf, np.nan):
        with pytest.raises(ValueError):
            k._validate_hyperparams_values(dict({n: p.value for n, p in good.items()}, gp_period=bad))
    assert list(k.valid_hyperparams_vec(np.array([[1, 2, 3, 4], [1, 0, 3, 4], [1, 2, np.nan, 4]]))) == [True, False,
                                                                                                           False]


def test_quasiperiodic_kernel_values():
    kern = GPKernel("Quasiperiodic").build_kernel({"gp_amp": 2.0, "gp_lambda_e": 10.0, "gp_lambda_p": 0.5,
                                                   "gp_period": 3.0})
    assert isinstance(kern, QuasiperiodicKernel)
    t = np.array([0.0, 1.0, 4.5])
    K = kern(t, t)
    assert np.allclose(np.diag(K), 4.0)
    tau = 1.0
    want = 4.0 * np.exp(-2.0 * np.sin(np.pi * tau / 3.0) ** 2) * np.exp(-0.5 * (tau / 10.0) ** 2)
    assert np.isclose(K[0, 1], want) and np.allclose(K, K.T)


def test_gp_oracle_matches_dense_gaussian():
    """The fp64 oracle equals the dense multivariate-normal log-density."""
    from scipy.stats import multivariate_normal
    from oracle import gp_oracle
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(4, n_epochs=60)
    ll = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th, hy)
    for w in range(4):
        if not np.isfinite(ll[w]):
            continue
        mu = gp_oracle.mean_model(ds.time, ds.inst_idx, 1, 1, 0, ds.t0, th[w])
        C = gp_oracle.qp_kernel(ds.time, *hy[w]) + np.diag(ds.velerr ** 2 + th[w, 6] ** 2)
        assert np.isclose(ll[w], multivariate_normal(mu, C).logpdf(ds.vel), rtol=1e-10)
