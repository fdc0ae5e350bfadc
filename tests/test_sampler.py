"""Stretch-move sampler (emcee StretchMove semantics) on a known target. CPU only."""
import numpy as np
import pytest

from ravest_amd.sampler import (AutocorrError, EnsembleSampler, State, emcee_step_draws, function_1d,
                                integrated_time, walkers_independent)


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
    with pytest.raises(ValueError, match="initial log_prob was NaN"):
        s2.run_mcmc(np.random.default_rng(1).uniform(-0.5, 0.5, (8, 2)), 1)
    with pytest.raises(ValueError, match="condition number"):     # emcee's walkers_independent check
        s2.run_mcmc(np.zeros((8, 2)), 1)
    s3 = EnsembleSampler(8, 2, lambda x: np.where(x[:, 0] > 0.4, np.nan, -0.5 * np.sum(x ** 2, axis=1)), seed=3)
    with pytest.raises(ValueError, match="Probability function returned NaN"):
        s3.run_mcmc(np.random.default_rng(1).uniform(-0.5, 0.3, (8, 2)), 50)


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


def _emcee_integrated_time_literal(x, c=5):
    """emcee 3.1's integrated_time, literally (one function_1d per walker, summed in order)."""
    n_t, n_w, n_d = x.shape
    tau = np.empty(n_d)
    for d in range(n_d):
        f = np.zeros(n_t)
        for k in range(n_w):
            f += function_1d(x[:, k, d])
        f /= n_w
        taus = 2.0 * np.cumsum(f) - 1.0
        m = np.arange(len(taus)) < c * taus
        w = np.argmin(m) if np.any(m) else len(taus) - 1
        tau[d] = taus[w]
    return tau


def test_integrated_time_matches_emcee():
    rng = np.random.default_rng(3)
    # AR(1) walkers with known tau = (1 + phi) / (1 - phi)
    phi = np.array([0.5, 0.9])
    n_t, n_w = 4000, 300
    x = np.zeros((n_t, n_w, 2))
    e = rng.standard_normal((n_t, n_w, 2))
    for t in range(1, n_t):
        x[t] = phi * x[t - 1] + e[t]
    tau = integrated_time(x, tol=0)
    assert np.allclose(tau, _emcee_integrated_time_literal(x), rtol=1e-12, atol=0)
    assert np.allclose(tau, (1 + phi) / (1 - phi), rtol=0.1)
    with pytest.raises(AutocorrError):
        integrated_time(x[:200], tol=50)
    assert np.all(np.isfinite(integrated_time(x[:200], tol=50, quiet=True)))
    # the device-chain backend's estimator (torch real FFTs; a CPU tensor here, the GPU's HBM in use)
    import torch
    from ravest_amd.sampler import integrated_time_device
    xt = torch.from_numpy(x)
    assert np.allclose(integrated_time_device(xt, tol=0), tau, rtol=1e-12, atol=0)
    with pytest.raises(AutocorrError):
        integrated_time_device(xt[:200], tol=50)
    assert np.allclose(integrated_time_device(xt[:200], tol=50, quiet=True),
                       integrated_time(x[:200], tol=50, quiet=True), rtol=1e-12, atol=0)


def test_chain_accessors_follow_emcee_backend():
    s = EnsembleSampler(8, 2, lambda x: -0.5 * np.sum(x ** 2, axis=1), seed=4)
    with pytest.raises(AttributeError):
        s.get_chain()
    st = s.run_mcmc(np.random.default_rng(2).standard_normal((8, 2)), 30)
    coords, lnp, rstate = st                                  # emcee 3's State unpacking
    assert isinstance(st, State) and coords.shape == (8, 2) and lnp.shape == (8,)
    full = s.get_chain()
    assert full.shape == (30, 8, 2) and s.iteration == 30
    assert np.array_equal(s.get_chain(discard=5, thin=3), full[5 + 3 - 1::3])       # [discard + thin - 1 :: thin]
    assert np.array_equal(s.get_chain(flat=True, discard=10), full[10:].reshape(-1, 2))
    assert np.array_equal(s.get_last_sample().coords, full[-1])
    assert np.array_equal(coords, full[-1])
    s.run_mcmc(None, 5)                                       # continues from the last state
    assert s.get_chain().shape == (35, 8, 2) and np.array_equal(s.get_chain()[:30], full)
    assert s.get_autocorr_time(tol=0).shape == (2,)


def test_walkers_independent():
    rng = np.random.default_rng(0)
    assert walkers_independent(rng.standard_normal((16, 4)))
    x = rng.standard_normal((16, 4))
    x[:, 2] = 2.0 * x[:, 1]                                   # linearly dependent coordinates
    assert not walkers_independent(x)
    x = rng.standard_normal((16, 4))
    x[:, 0] = 1.0                                             # a constant coordinate
    assert not walkers_independent(x)


def ravest_convergence_loop(sampler, initial_positions, max_steps, interval, start):
    """ravest's adaptive run_mcmc loop (src/ravest/fit.py:1119-1156), restated: iterate
    sampler.sample, every `interval` steps after `start` take get_autocorr_time(tol=0) and stop
    when iteration > 50 tau and tau is stable to 1 %."""
    history = {}
    old_tau = np.inf
    for _sample in sampler.sample(initial_state=initial_positions, iterations=max_steps, progress=False):
        if sampler.iteration % interval != 0:
            continue
        if sampler.iteration < start:
            continue
        tau = sampler.get_autocorr_time(tol=0)
        history[sampler.iteration] = tau.copy()
        converged = np.all(sampler.iteration > 50 * tau) and np.all(np.abs(old_tau - tau) / tau < 0.01)
        if converged:
            break
        old_tau = tau
    return history


def test_ravest_convergence_loop_stops_early_host():
    s = EnsembleSampler(32, 2, lambda x: -0.5 * np.sum(x ** 2, axis=1), seed=5)
    hist = ravest_convergence_loop(s, np.random.default_rng(1).standard_normal((32, 2)), 20000, 250, 500)
    assert s.iteration < 20000 and s.iteration in hist
    assert s.get_chain().shape[0] == s.iteration


def test_host_sampler_store_false_semantics():
    """emcee's save_step: store=False advances the walkers, not iteration / chain / acceptances."""
    from ravest_amd.sampler import EnsembleSampler
    f = lambda x: -0.5 * np.sum(x ** 2, axis=1)          # noqa: E731
    x0 = np.random.default_rng(3).normal(size=(16, 3))
    a = EnsembleSampler(16, 3, f, seed=7)
    for _ in a.sample(x0, iterations=20, store=False):
        pass
    assert a.iteration == 0 and a.naccepted.sum() == 0
    a.run_mcmc(None, 10)
    b = EnsembleSampler(16, 3, f, seed=7)
    b.run_mcmc(x0, 30)
    assert a.iteration == 10 and np.array_equal(a.get_chain(), b.get_chain()[20:])
    c = EnsembleSampler(16, 3, f, seed=7)
    c.run_mcmc(x0, 20)
    assert np.array_equal(a.naccepted, b.naccepted - c.naccepted)


@pytest.mark.parametrize("k", [1, 3])
def test_host_sampler_thin_by_stores_every_kth_step(k):
    """emcee 3.1's thin_by: k steps per yielded step, every k-th stored, and (as in emcee's
    backend.save_step) only the stored steps' acceptances counted.  Same RandomState stream as an
    unthinned run, so the stored rows are that run's rows k-1, 2k-1, ..."""
    f = lambda x: -0.5 * np.sum(x ** 2, axis=1)          # noqa: E731
    x0 = np.random.default_rng(4).normal(size=(16, 3))
    ref = EnsembleSampler(16, 3, f, seed=9)
    acc = []
    for _ in ref.sample(x0, iterations=12 * k):
        acc.append(ref.backend.accepted.copy())
    s = EnsembleSampler(16, 3, f, seed=9)
    n_yield = sum(1 for _ in s.sample(x0, iterations=12, thin_by=k))
    assert n_yield == 12 and s.iteration == 12
    assert np.array_equal(s.get_chain(), ref.get_chain()[k - 1::k])
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob()[k - 1::k])
    per_step = np.diff(np.concatenate([np.zeros((1, 16)), np.array(acc)]), axis=0)
    assert np.array_equal(s.naccepted, per_step[k - 1::k].sum(axis=0))


def test_host_sampler_deprecated_thin():
    f = lambda x: -0.5 * np.sum(x ** 2, axis=1)          # noqa: E731
    x0 = np.random.default_rng(5).normal(size=(16, 3))
    ref = EnsembleSampler(16, 3, f, seed=2)
    ref.run_mcmc(x0, 10)
    s = EnsembleSampler(16, 3, f, seed=2)
    with pytest.warns(DeprecationWarning):
        n_yield = sum(1 for _ in s.sample(x0, iterations=10, thin=3))
    assert n_yield == 10 and s.iteration == 3                # iterations // thin rows
    assert np.array_equal(s.get_chain(), ref.get_chain()[2::3][:3])
    with pytest.raises(ValueError):
        next(s.sample(x0, iterations=3, thin_by=0))
