"""Multi-process walker sharding (world_size 2, gloo on CPU): the N>1 path of bench.py /
ShardedLogProbability, with a toy per-walker function standing in for the GPU likelihood."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ravest_amd.distributed import shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _toy(theta):
    return -0.5 * np.sum(theta ** 2, axis=1) + theta[:, 0]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedLogProbability
    from ravest_amd.sampler import EnsembleSampler
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sh = ShardedLogProbability(_toy)
        rng = np.random.default_rng(rank)               # different data per rank ...
        theta = sh.broadcast(rng.standard_normal((37, 3)))   # ... until rank 0's block is broadcast
        got = sh(theta)
        ok = bool(np.array_equal(got, _toy(theta)))
        # a short sampler run is identical on every rank (same seed, same gathered log-probs)
        s = EnsembleSampler(16, 3, sh, seed=7)
        s.run_mcmc(np.random.default_rng(3).standard_normal((16, 3)) * 0.1, 20)
        q.put((rank, ok, float(s.get_chain()[-1].sum())))
    finally:
        dist.destroy_process_group()


def _oracle_eval(ds):
    """The injected per-shard evaluator: the C oracle on CPU tensors (the GPU run injects
    DevicePosterior.device / RVEngine.loglike_device)."""
    from oracle import oracle

    def ev(theta, out):
        ll, _ = oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments),
                               len(ds.planet_letters), ds.parameterisation.code, ds.t0, theta.numpy(), nthreads=1)
        out.copy_(torch.from_numpy(ll))
    return ev


def _sharded_worker(rank, world, port, q):
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDevicePosterior
    from ravest_amd.synth import make_dataset, make_walkers
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ds = make_dataset(2, 96, 2, seed=4)
        res = {}
        for W in (64, 37, 5):
            theta = torch.from_numpy(make_walkers(ds, W, seed=4))
            sh = ShardedDevicePosterior(_oracle_eval(ds))
            res[W] = sh(theta).numpy().tolist()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_device_posterior(world):
    """ShardedDevicePosterior itself (not a toy): every rank ends with the whole block's
    log-probs, bitwise equal to one process evaluating all walkers, for even and ragged W."""
    from ravest_amd.synth import make_dataset, make_walkers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ds = make_dataset(2, 96, 2, seed=4)
    for W in (64, 37, 5):
        theta = torch.from_numpy(make_walkers(ds, W, seed=4))
        ref = torch.empty(W, dtype=torch.float64)
        _oracle_eval(ds)(theta, ref)
        for r in range(world):
            assert np.array_equal(np.array(res[r][W]), ref.numpy()), (W, r)


def test_shard_bounds_cover():
    for n in (0, 1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_gloo_world2_allgather_and_sampler():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] for r in res)
    assert res[0][2] == res[1][2]
