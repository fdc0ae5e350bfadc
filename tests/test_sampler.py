"""Stretch-move sampler (emcee StretchMove semantics) on a known target. CPU only."""
import numpy as np
import pytest

from ravest_amd.sampler import EnsembleSampler, emcee_step_draws


def test_gaussian_moments():
    cov = np.array([[1.0, 0.6], [0.6, 2.0]])
    icov = np.linalg.inv(cov)
    mu = np.array([1.0, -2.0])

    def lp(x):
        d = x - mu
        return -0.5 * np.einsum("ij,jk,ik->i", d, icov, d)

    s = EnsembleSampler(32, 2, lp, seed=1)
    s.run_mcmc(mu + 0.1 * np.random.default_rng(0).standard_normal((32, 2)), 3000)
    x = s.get_chain(discard=500, flat=True)
    assert np.allclose(x.mean(0), mu, atol=0.15)
    assert np.allclose(np.cov(x.T), cov, atol=0.3)
    assert 0.3 < s.acceptance_fraction.mean() < 0.9
    assert s.get_chain().shape == (3000, 32, 2) and s.get_log_prob().shape == (3000, 32)


def test_minus_inf_rejects_nan_raises():
    def lp(x):
        out = -0.5 * np.sum(x ** 2, axis=1)
        out[x[:, 0] > 1.0] = -np.inf
        return out
    s = EnsembleSampler(8, 2, lp, seed=2)
    s.run_mcmc(np.random.default_rng(1).uniform(-0.5, 0.5, (8, 2)), 200)
    assert np.all(s.get_chain()[:, :, 0] <= 1.0)
    s2 = EnsembleSampler(8, 2, lambda x: np.full(len(x), np.nan), seed=3)
    with pytest.raises(ValueError):
        s2.run_mcmc(np.zeros((8, 2)), 1)


def test_emcee_call_order():
    """The draws are emcee 3.1's, in its order: shuffle(inds % 2), then per half rand(H),
    randint(H, size=H), H x rand()."""
    W, H = 10, 5
    a = np.random.RandomState(42)
    sets, zu, rint, au = emcee_step_draws(a, W)
    b = np.random.RandomState(42)
    inds = np.arange(W) % 2
    b.shuffle(inds)
    for split in (0, 1):
        assert np.array_equal(sets[split], np.arange(W)[inds == split])
        assert np.array_equal(zu[split], b.rand(H))
        assert np.array_equal(rint[split], b.randint(H, size=(H,)))
        assert np.array_equal(au[split], np.array([b.rand() for _ in range(H)]))
    assert np.array_equal(np.sort(np.concatenate(sets)), np.arange(W))
