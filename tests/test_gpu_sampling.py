"""End to end: the drop-in LogPosterior on the GPU driving the stretch move on 51 Peg b (config 1)."""
import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation
from ravest_amd.posterior import LogPosterior
from ravest_amd.sampler import EnsembleSampler
from tests._golden import load_case

pytestmark = pytest.mark.gpu


def test_51peg_posterior():
    case = load_case("51peg")
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    lp = LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                      m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                      np.array(m["unique_instruments"]), m["t0"])
    x0 = case["theta_free"][:32]
    assert np.all(np.isfinite(lp.log_probability_batch(x0)))
    s = EnsembleSampler(32, len(m["free_names"]), lp.log_probability_batch, seed=51)
    s.run_mcmc(x0, 1500)
    post = s.get_chain(discard=500, flat=True)
    P_b, K_b = post[:, 0].mean(), post[:, 1].mean()
    assert abs(P_b - 4.2308) < 2e-3          # 51 Peg b period (days)
    assert 50.0 < K_b < 62.0                  # semi-amplitude (m/s), ELODIE data
    assert 0.2 < s.acceptance_fraction.mean() < 0.9
