"""The device sampler as a drop-in for ravest's emcee usage (fit.py:1068-1160): emcee 3's randomised
split drawn on the device, ravest's adaptive convergence loop over DeviceEnsembleSampler.sample,
early stop + resume equal to an uninterrupted run, exact acceptance counts with a suspended
generator, and a run split over calls equal to one call."""
import ctypes as C

import numpy as np
import pytest

from tests._golden import load_case
from tests.test_gpu_device_posterior import _posterior, _start
from tests.test_sampler import ravest_convergence_loop

pytestmark = pytest.mark.gpu


def _table(dp, W, n, flags=0, seed=3, step0=0):
    import torch
    from ravest_amd import _lib
    L = _lib.load()
    dp.reserve(W)
    _lib.check(L.rvk_stretch_draws(dp._p, W, n, 2.0, seed, step0, flags, torch.cuda.current_stream().cuda_stream))
    H = W // 2
    out = []
    for s in range(n):
        halves = []
        for h in (0, 1):
            w, c, z = np.empty(H, np.int64), np.empty(H, np.int64), np.empty(H)
            vp = C.c_void_p
            _lib.check(L.rvk_stretch_table_read(dp._p, s, h, vp(w.ctypes.data), vp(c.ctypes.data), vp(z.ctypes.data)))
            halves.append((w, c, z))
        out.append(halves)
    return out


@pytest.mark.parametrize("W", [256, 4096, 1000])
def test_device_split_is_emcee3_randomised_balanced(W):
    """Per step: the halves partition the walkers, H each, ascending (emcee's boolean-mask order),
    complements come from the other half, z in [1/a, a]; the split changes from step to step and
    every walker lands in half 0 about half the time.  RVK_STRETCH_FIXED_SPLIT: even / odd."""
    from ravest_amd import _lib
    from ravest_amd.synth import make_posterior
    lpost, _ = make_posterior(2, 16, seed=4)
    dp = lpost.device_posterior()
    n = 64
    tab = _table(dp, W, n)
    H = W // 2
    in0 = np.zeros(W)
    sets = []
    for s in range(n):
        (w0, c0, z0), (w1, c1, z1) = tab[s]
        assert np.array_equal(np.sort(np.r_[w0, w1]), np.arange(W))
        assert np.all(np.diff(w0) > 0) and np.all(np.diff(w1) > 0)
        assert np.all(np.isin(c0, w1)) and np.all(np.isin(c1, w0))
        assert np.all((z0 >= 0.5) & (z0 <= 2.0)) and np.all((z1 >= 0.5) & (z1 <= 2.0))
        in0[w0] += 1
        sets.append(tuple(w0))
    assert len(set(sets)) == n                                # a fresh split every step
    frac = in0 / n
    assert abs(frac.mean() - 0.5) < 1e-12 and 0.3 < np.median(frac) < 0.7
    assert frac.min() > 0.05 and frac.max() < 0.95
    again = _table(dp, W, 4, step0=2)                         # keyed by the global step
    assert np.array_equal(again[0][0][0], tab[2][0][0]) and np.array_equal(again[1][1][1], tab[3][1][1])
    fixed = _table(dp, W, 2, flags=_lib.STRETCH_FIXED_SPLIT)
    assert np.array_equal(fixed[0][0][0], np.arange(0, W, 2)) and np.array_equal(fixed[1][1][0], np.arange(1, W, 2))


def test_ravest_convergence_loop_stops_early_on_51peg():
    """ravest's run_mcmc(check_convergence=True) loop (fit.py:1119-1156) driving the device sampler."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    case = load_case("51peg")
    lpost, x0 = _start(case, 64, 5)
    s = DeviceEnsembleSampler(lpost, 64, seed=2024)
    hist = ravest_convergence_loop(s, x0, 40000, 1000, 2000)
    assert s.iteration < 40000, f"no convergence: {hist}"
    assert s.iteration in hist and s.get_chain().shape == (s.iteration, 64, x0.shape[1])
    tau = hist[s.iteration]
    assert np.all(s.iteration > 50 * tau)
    names = case["meta"]["free_names"]
    if "P_b" in names:
        assert abs(np.median(s.get_chain(discard=s.iteration // 2)[:, :, names.index("P_b")]) - 4.2308) < 0.01


@pytest.mark.parametrize("rng,storage", [("philox", "device"), ("emcee", "device"), ("philox", "host"),
                                         ("emcee", "host")])
def test_early_stop_resume_equals_one_run(rng, storage):
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 64, seed=4)
    mk = lambda: DeviceEnsembleSampler(lpost, 64, seed=np.random.RandomState(9) if rng == "emcee" else 9,  # noqa: E731
                                       rng=rng, steps_per_call=32, chain_storage=storage)
    ref = mk()
    ref.run_mcmc(x0, 150)
    part = mk()
    part.run_mcmc(x0, 70)
    s = mk()
    gen = s.sample(x0, iterations=150)
    for _ in gen:
        if s.iteration == 70:              # inside the third chunk, the fourth in flight
            break
    assert np.array_equal(s.naccepted, part.naccepted)        # exact while the generator is suspended
    assert np.array_equal(s.get_chain(), part.get_chain())
    del gen
    s.run_mcmc(None, 80)
    assert np.array_equal(s.get_chain(), ref.get_chain())
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(s.naccepted, ref.naccepted)
    assert ref.naccepted.sum() > 0
    assert s.chain_storage == storage


def test_device_chain_equals_host_chain():
    """The HBM-resident chain (default) and the host-copied one are the same chain; the device
    autocorrelation estimate equals the host restatement's; yielded states read back exactly."""
    from ravest_amd.sampler import DeviceEnsembleSampler, integrated_time
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 128, seed=8)
    d = DeviceEnsembleSampler(lpost, 128, seed=21, steps_per_call=40)
    h = DeviceEnsembleSampler(lpost, 128, seed=21, steps_per_call=40, chain_storage="host")
    states = [(st.coords.copy(), st.log_prob.copy()) for st in d.sample(x0, iterations=100)]
    h.run_mcmc(x0, 100)
    assert d.chain_storage == "device" and h.chain_storage == "host"
    assert np.array_equal(d.get_chain(), h.get_chain()) and np.array_equal(d.get_log_prob(), h.get_log_prob())
    assert np.array_equal(np.stack([c for c, _ in states]), h.get_chain())
    assert np.array_equal(np.stack([lp for _, lp in states]), h.get_log_prob())
    assert np.array_equal(d.get_chain(discard=10, thin=3, flat=True), h.get_chain(discard=10, thin=3, flat=True))
    np.testing.assert_allclose(d.get_autocorr_time(tol=0), integrated_time(h.get_chain(), tol=0), rtol=1e-12)
    assert np.array_equal(d.naccepted, h.naccepted)


def test_split_runs_and_chunk_sizes_equal_one_run():
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 128, seed=6)
    a = DeviceEnsembleSampler(lpost, 128, seed=5)
    a.run_mcmc(x0, 100)
    b = DeviceEnsembleSampler(lpost, 128, seed=5, steps_per_call=7)
    b.run_mcmc(x0, 33)
    b.run_mcmc(None, 67)
    assert np.array_equal(a.get_chain(), b.get_chain()) and np.array_equal(a.naccepted, b.naccepted)
    tau = a.get_autocorr_time(tol=0)
    assert tau.shape == (x0.shape[1],) and np.all(np.isfinite(tau))


def test_fixed_split_option():
    """randomize_split=False (emcee's RedBlueMove option): even / odd halves, a valid sampler."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 64, seed=4)
    s = DeviceEnsembleSampler(lpost, 64, seed=3, randomize_split=False)
    s.run_mcmc(x0, 200)
    r = DeviceEnsembleSampler(lpost, 64, seed=3)
    r.run_mcmc(x0, 200)
    assert not np.array_equal(s.get_chain(), r.get_chain())
    assert 0.05 < s.acceptance_fraction.mean() < 0.9 and np.all(np.isfinite(s.get_log_prob()))


@pytest.mark.parametrize("storage", ["device", "host"])
def test_store_false_then_store_true(storage):
    """emcee's save_step semantics: unstored steps advance the walkers but neither `iteration`, the
    chain nor the acceptance counts; a stored run afterwards starts at row 0 and equals a sampler
    that took the same steps (same Philox positions) with the first part unstored."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 64, seed=4)
    s = DeviceEnsembleSampler(lpost, 64, seed=11, steps_per_call=16, chain_storage=storage)
    for st in s.sample(x0, iterations=40, store=False):
        pass
    assert s.iteration == 0 and int(s.naccepted.sum()) == 0
    last = (st.coords.copy(), st.log_prob.copy())
    s.run_mcmc(None, 30)
    assert s.iteration == 30 and s.get_chain().shape == (30, 64, x0.shape[1])
    ref = DeviceEnsembleSampler(lpost, 64, seed=11, steps_per_call=16, chain_storage=storage)
    ref.run_mcmc(x0, 70)
    assert np.array_equal(ref.get_chain()[39], last[0]) and np.array_equal(ref.get_log_prob()[39], last[1])
    assert np.array_equal(s.get_chain(), ref.get_chain()[40:])
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob()[40:])
    # acceptances of the 30 stored steps only
    pre = DeviceEnsembleSampler(lpost, 64, seed=11, steps_per_call=16, chain_storage=storage)
    pre.run_mcmc(x0, 40)
    assert np.array_equal(s.naccepted, ref.naccepted - pre.naccepted)
    # a generator of unstored steps stopped early, then a stored resume
    u = DeviceEnsembleSampler(lpost, 64, seed=11, steps_per_call=16, chain_storage=storage)
    n = 0
    for _ in u.sample(x0, iterations=40, store=False):
        n += 1
        if n == 23:
            break
    u.run_mcmc(None, 47)
    assert np.array_equal(u.get_chain(), ref.get_chain()[23:]) and np.array_equal(u.naccepted, ref.naccepted - _acc(lpost, x0, storage, 23))


def _acc(lpost, x0, storage, n):
    from ravest_amd.sampler import DeviceEnsembleSampler
    p = DeviceEnsembleSampler(lpost, 64, seed=11, steps_per_call=16, chain_storage=storage)
    p.run_mcmc(x0, n)
    return p.naccepted


def test_reset_does_not_replay_the_draws():
    """reset() clears the chain but the Philox draws go on (emcee's RandomState is not rewound):
    a burn-in, reset and production run with the same seed is NOT the burn-in again; a fresh
    sampler with the seed still reproduces the burn-in exactly."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 64, seed=4)
    s = DeviceEnsembleSampler(lpost, 64, seed=13)
    s.run_mcmc(x0, 50)
    burn = s.get_chain().copy()
    s.reset()
    s.run_mcmc(x0, 50)
    assert s.iteration == 50 and not np.array_equal(s.get_chain(), burn)
    f = DeviceEnsembleSampler(lpost, 64, seed=13)
    f.run_mcmc(x0, 50)
    assert np.array_equal(f.get_chain(), burn)
    # the production run used the draws of steps 50..99: a fresh sampler whose first 50 steps are
    # unstored and which then restarts from x0 at position 50 makes the same chain
    g = DeviceEnsembleSampler(lpost, 64, seed=13)
    for _ in g.sample(x0, iterations=50, store=False):
        pass
    g.run_mcmc(x0, 50)
    assert np.array_equal(g.get_chain(), s.get_chain())


@pytest.mark.parametrize("storage", ["device", "host"])
def test_device_sampler_thin_by(storage):
    """emcee 3.1's thin_by on the GPU sampler: the stored rows are the unthinned run's every k-th
    row bit for bit, iteration counts the stored steps, and naccepted only their acceptances (emcee's
    backend.save_step)."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, 128, seed=8)
    k, n = 4, 10
    ref = DeviceEnsembleSampler(lpost, 128, seed=5, steps_per_call=16)
    cum = [np.zeros(128, dtype=np.int64)]
    for _ in ref.sample(x0, iterations=n * k):
        cum.append(ref.naccepted.copy())
    acc = np.diff(np.array(cum), axis=0)
    s = DeviceEnsembleSampler(lpost, 128, seed=5, steps_per_call=16, chain_storage=storage)
    s.run_mcmc(x0, n, thin_by=k)
    assert s.iteration == n
    assert np.array_equal(s.get_chain(), ref.get_chain()[k - 1::k])
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob()[k - 1::k])
    assert np.array_equal(s.naccepted, acc[k - 1::k].sum(axis=0)) and s.naccepted.sum() > 0
