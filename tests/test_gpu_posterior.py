"""The drop-in LogPosterior (host mirror + HIP likelihood) against the reference's log_probability."""
import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation
from ravest_amd.posterior import LogPosterior
from tests._golden import assert_ll_close, load_case, logpost_cases

pytestmark = pytest.mark.gpu


def _posterior(case):
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    return LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                        np.array(m["unique_instruments"]), m["t0"])


@pytest.mark.parametrize("name", logpost_cases())
def test_log_probability_batch(name):
    case = load_case(name)
    lp = _posterior(case)
    got = lp.log_probability_batch(case["theta_free"])
    assert_ll_close(got, case["log_prob"], what=name)


@pytest.mark.parametrize("name", ["cfg2", "case3", "pkewtc", "51peg"])
def test_log_probability_scalar_dropin(name):
    case = load_case(name)
    lp = _posterior(case)
    names = case["meta"]["free_names"]
    got = np.array([lp.log_probability(dict(zip(names, row))) for row in case["theta_free"][:24]])
    assert_ll_close(got, case["log_prob"][:24], what=name)
    assert all(isinstance(v, float) for v in got)


def test_loglikelihood_dict_call():
    case = load_case("cfg3")
    lp = _posterior(case)
    names = lp.log_likelihood.names
    for row, ref in zip(case["theta_full"][:8], case["log_like"][:8]):
        assert_ll_close([lp.log_likelihood(dict(zip(names, row)))], [ref], what="cfg3-dict")
