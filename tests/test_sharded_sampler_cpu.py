"""ShardedDeviceSampler's multi-rank orchestration on CPU (gloo, world sizes 2 and 3) with a host
stand-in for the device operations (tests/_toy_stretch_ops.py): the chain is bitwise the one-rank
chain, the exchange is the H per-proposal log-probabilities (8 bytes each) per half-step, a NaN in
one rank's slice makes every rank raise (none hangs in a collective), keep_chain keeps the host
chain on one rank and the autocorrelation estimate is broadcast from it, and a run stopped early
and resumed equals an uninterrupted run -- with the chain kept in the host backend and in the
"device" backend (torch tensors; on CPU here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

W, D, STEPS, SPC = 48, 3, 23, 5
LOOP_STEPS = 400


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _x0():
    return np.random.default_rng(5).standard_normal((W, D)) * 0.5


def _sampler(nan_at=None, keep="all", storage="auto"):
    from ravest_amd.distributed import ShardedDeviceSampler
    from tests._toy_stretch_ops import ToyStretchOps
    return ShardedDeviceSampler(None, W, seed=11, steps_per_call=SPC, keep_chain=keep, ops=ToyStretchOps(D, nan_at),
                                device=torch.device("cpu"), chain_storage=storage)


def _worker(rank, world, port, q, mode, storage="auto"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if mode == "chain":
            s = _sampler(storage=storage)
            s.run_mcmc(_x0(), STEPS)
            q.put((rank, s.get_chain(), s.get_log_prob(), s.naccepted.copy(), s.exchange_bytes_per_half_step))
        elif mode == "nan":
            s = _sampler(nan_at=(7, 1, W // 2 - 1))          # the last rank's slice
            try:
                s.run_mcmc(_x0(), STEPS)
                q.put((rank, "no error"))
            except ValueError as e:
                q.put((rank, str(e), s.iteration))
        elif mode == "keeploop":                           # ravest's adaptive loop, chain on rank 0 only
            from tests.test_sampler import ravest_convergence_loop
            s = _sampler(keep=0, storage=storage)
            hist = ravest_convergence_loop(s, _x0(), LOOP_STEPS, 25, 50)
            q.put((rank, s.iteration, s.naccepted.copy(), sorted(hist), s.acceptance_fraction.copy()))
        elif mode == "tau_all":                            # keep_chain="all": local estimate + guard
            s = _sampler(storage=storage)
            s.run_mcmc(_x0(), 60)
            short = None
            try:
                s.get_autocorr_time()                      # tol=50 on 60 steps: too short on every rank
            except Exception as e:
                short = type(e).__name__
            q.put((rank, short, s.get_autocorr_time(tol=0)))
        elif mode == "tau_disagree":                       # one rank's estimate differs in the last bit
            from ravest_amd.distributed import _DevicePipeline
            s = _sampler(storage=storage)
            s.run_mcmc(_x0(), 60)
            if rank == 1:
                base = _DevicePipeline.get_autocorr_time
                _DevicePipeline.get_autocorr_time = lambda self, **kw: np.nextafter(base(self, **kw), np.inf)
            try:
                s.get_autocorr_time(tol=0)
                q.put((rank, "no error"))
            except RuntimeError as e:
                q.put((rank, str(e)))
        elif mode == "keep":
            s = _sampler(keep=0, storage=storage)
            s.run_mcmc(_x0(), STEPS)
            tau = s.get_autocorr_time(tol=0)
            try:
                s.get_chain()
                has = True
            except RuntimeError:
                has = False
            q.put((rank, has, tau))
    finally:
        dist.destroy_process_group()


def _spawn(world, mode, storage="auto"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, storage)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,storage", [(2, "host"), (3, "host"), (2, "device")])
def test_sharded_chain_equals_one_rank(world, storage):
    ref = _sampler()
    ref.run_mcmc(_x0(), STEPS)
    for rank, chain, lnp, nacc, xb in _spawn(world, "chain", storage):
        assert np.array_equal(chain, ref.get_chain()), rank
        assert np.array_equal(lnp, ref.get_log_prob()), rank
        assert np.array_equal(nacc, ref.naccepted), rank
        assert xb == (W // 2) * 8                          # the exchange: H log-probs per half-step
    assert ref.naccepted.sum() > 0 and ref.iteration == STEPS


def test_nan_raises_on_every_rank():
    res = _spawn(2, "nan")
    assert all(r[1] == "Probability function returned NaN" for r in res), res
    assert all(r[2] == 5 for r in res)                     # the chunk with step 7 starts at step 5


@pytest.mark.parametrize("storage", ["host", "device"])
def test_keep_chain_on_one_rank_and_broadcast_tau(storage):
    res = _spawn(2, "keep", storage)
    assert res[0][1] and not res[1][1]
    assert np.array_equal(res[0][2], res[1][2]) and np.all(np.isfinite(res[0][2]))


@pytest.mark.parametrize("storage", ["host", "device"])
def test_early_stop_and_resume_equals_one_run(storage):
    ref = _sampler()
    ref.run_mcmc(_x0(), STEPS)
    s = _sampler(storage=storage)
    for st in s.sample(_x0(), iterations=STEPS):
        if s.iteration == 12:                              # inside the third chunk; the fourth is in flight
            break
    assert s.iteration == 12
    assert np.array_equal(s.naccepted, _nacc_at(12))     # exact inside a chunk, generator suspended
    s.run_mcmc(None, STEPS - 12)
    assert np.array_equal(s.get_chain(), ref.get_chain())
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(s.naccepted, ref.naccepted)
    if storage == "device":
        from ravest_amd.sampler import _DeviceBackend, integrated_time
        assert isinstance(s.backend, _DeviceBackend) and s.chain_storage == "device"
        np.testing.assert_allclose(s.get_autocorr_time(tol=0), integrated_time(ref.get_chain(), tol=0),
                                   rtol=1e-12, atol=0)
        st = s.get_last_sample()
        assert np.array_equal(st.coords, ref.get_chain()[-1]) and np.array_equal(st.log_prob, ref.get_log_prob()[-1])


def _nacc_at(k):
    r = _sampler()
    r.run_mcmc(_x0(), k)
    return r.naccepted


def test_device_chain_moves_to_host_when_it_no_longer_fits():
    """chain_storage="auto" keeps the chain in device memory while it fits; a run that would not
    fit moves the chain to host memory and goes on with the chunked copy-out -- same chain."""
    ref = _sampler()
    ref.run_mcmc(_x0(), STEPS)
    s = _sampler(storage="device")
    s.run_mcmc(_x0(), 12)
    assert s.chain_storage == "device"
    s._device_chain_fits = lambda iterations: False
    s.run_mcmc(None, STEPS - 12)
    assert s.chain_storage == "host" and isinstance(s.get_chain(), np.ndarray)
    assert np.array_equal(s.get_chain(), ref.get_chain())
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(s.naccepted, ref.naccepted)


@pytest.mark.parametrize("storage", ["host", "device"])
def test_convergence_loop_with_chain_on_one_rank(storage):
    """keep_chain=0: the ranks that keep no chain still count iteration and acceptances, so
    ravest's convergence loop (fit.py:1123-1131) makes the same collective get_autocorr_time
    calls on every rank and stops at the same step (before: those ranks never left
    iteration 0 and every rank blocked in the broadcast)."""
    res = _spawn(2, "keeploop", storage)
    ref = _sampler()
    from tests.test_sampler import ravest_convergence_loop
    hist = ravest_convergence_loop(ref, _x0(), LOOP_STEPS, 25, 50)
    for rank, it, nacc, checks, af in res:
        assert it == ref.iteration and it > 0, rank
        assert np.array_equal(nacc, ref.naccepted), rank
        assert checks == sorted(hist), rank
        assert np.all(np.isfinite(af)) and np.array_equal(af, ref.acceptance_fraction), rank


def test_autocorr_time_local_with_keep_chain_all():
    """keep_chain="all": get_autocorr_time is computed on each rank, and one guard all-reduce
    makes the ranks agree: same estimate everywhere, and a too-short chain raises emcee's
    AutocorrError on every rank (none is left waiting in a collective)."""
    res = _spawn(2, "tau_all")
    assert all(r[1] == "AutocorrError" for r in res), res
    assert np.array_equal(res[0][2], res[1][2]) and np.all(np.isfinite(res[0][2]))


def test_autocorr_time_disagreement_raises_on_every_rank():
    """if one rank's estimate differs (another FFT plan, another GPU SKU), every rank
    raises instead of one leaving ravest's convergence loop while the others hang."""
    res = _spawn(2, "tau_disagree")
    assert all("disagree" in r[1] for r in res), res


def _per_step_acceptances(n):
    """Per-step acceptance vectors of an unthinned run (differences of the cumulative counts)."""
    r = _sampler()
    cum = [np.zeros(W, dtype=np.int64)]
    for _ in r.sample(_x0(), iterations=n):
        cum.append(r.naccepted.copy())
    return r, np.diff(np.array(cum), axis=0)


@pytest.mark.parametrize("k,storage", [(3, "host"), (4, "device"), (1, "device")])
def test_device_pipeline_thin_by(k, storage):
    """emcee 3.1's thin_by on the device pipeline (DeviceEnsembleSampler / ShardedDeviceSampler):
    k steps per yielded step, every k-th stored -- the unthinned chain's rows k-1, 2k-1, ... bit for
    bit (the draws are keyed by the global step) -- and emcee's accounting: iteration counts the
    stored steps, naccepted only their acceptances."""
    n = 7
    ref, acc = _per_step_acceptances(n * k)
    s = _sampler(storage=storage)
    ys = list(s.sample(_x0(), iterations=n, thin_by=k))
    assert len(ys) == n and s.iteration == n
    assert np.array_equal(s.get_chain(), ref.get_chain()[k - 1::k])
    assert np.array_equal(s.get_log_prob(), ref.get_log_prob()[k - 1::k])
    assert np.array_equal(s.naccepted, acc[k - 1::k].sum(axis=0))
    assert np.array_equal(np.asarray(ys[-1].coords), ref.get_chain()[-1])
    s.run_mcmc(None, 2, thin_by=k)                   # continues: 2 more stored rows
    assert s.iteration == n + 2


def test_device_pipeline_thin_deprecated():
    """The deprecated thin=k: every step yielded, every k-th stored (iterations // k rows)."""
    ref, acc = _per_step_acceptances(11)
    s = _sampler()
    with pytest.warns(DeprecationWarning):
        ys = list(s.sample(_x0(), iterations=11, thin=3))
    assert len(ys) == 11 and s.iteration == 3
    assert np.array_equal(s.get_chain(), ref.get_chain()[2:9:3])
    assert np.array_equal(s.naccepted, acc[2:9:3].sum(axis=0))
    with pytest.raises(ValueError):
        next(s.sample(None, iterations=2, thin_by=0))
