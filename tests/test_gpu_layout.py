"""Layout independence: a walker's log-probability has the same BITS whatever the lanes-per-walker
layout, the batch it is evaluated in, or the GPU shard it lands on (results
bitwise identical across GPU counts), and the fused sampler kernel agrees with the plain one.

The segmented kernel (32 / 16 lanes per walker, chosen for large batches) keeps one accumulator
per lane of the one-wave-per-walker layout and reduces in that layout's order, so every check
here is np.array_equal, not a tolerance."""
import numpy as np
import pytest
import torch

from ravest_amd.engine import RVEngine
from ravest_amd.synth import CONFIGS, make_config, make_dataset, make_posterior, make_walkers

pytestmark = pytest.mark.gpu


def _engine(ds):
    return RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), len(ds.planet_letters),
                    ds.parameterisation, ds.t0, device=0)


CASES = [  # (n_planets, n_epochs, n_inst, seed, parameterisation, trend)
    (1, 256, 1, 2, "P K e w Tp", False),
    (3, 1024, 2, 3, "P K e w Tp", False),
    (2, 512, 1, 4, "P K secosw sesinw Tc", False),
    (1, 37, 1, 9, "P K e w Tc", True),      # ragged: fewer epochs than lanes
    (2, 200, 3, 10, "P K e w Tp", True),    # 3 instruments + trend, 200 = 3*64 + 8
]


@pytest.mark.parametrize("np_, n, ni, seed, par, trend", CASES)
def test_lanes_per_walker_bitwise(np_, n, ni, seed, par, trend):
    ds = make_dataset(np_, n, ni, seed=seed, parameterisation=par)
    theta = make_walkers(ds, 1024, seed=seed)
    if trend:
        theta[:, -2] = 0.01 * np.random.default_rng(seed).standard_normal(len(theta))
        theta[::3, -1] = 1e-5
    eng = _engine(ds)
    outs = {}
    for lpw in (64, 32, 16):
        eng.set_lanes_per_walker(lpw)
        outs[lpw] = eng.loglike(theta)
    assert np.isfinite(outs[64]).sum() > 900
    assert np.array_equal(outs[64], outs[32]), "32 lanes per walker differ from 64"
    assert np.array_equal(outs[64], outs[16]), "16 lanes per walker differ from 64"


def test_batch_size_bitwise():
    """The same walkers in a 4096 batch (one wave per walker) and inside a 16384 batch
    (segmented layout) and one at a time."""
    ds = make_config(3)
    eng = _engine(ds)
    big = eng.loglike(ds.theta)
    assert np.array_equal(eng.loglike(ds.theta[8192:12288]), big[8192:12288])
    assert np.array_equal(eng.loglike(ds.theta[5:6]), big[5:6])
    assert np.array_equal(eng.loglike(ds.theta[100:163]), big[100:163])


def test_config4_shards_bitwise():
    """Config 4's 65536 walkers: the concatenation of every rank's contiguous shard at N = 2, 4, 8
    (each shard a separate launch, as on its own GPU) equals the N = 1 evaluation bit for bit."""
    from ravest_amd.distributed import shard_bounds
    c = CONFIGS[4]
    ds = make_dataset(c["n_planets"], c["n_epochs"], c["n_inst"], seed=c["seed"])
    theta = make_walkers(ds, c["n_walkers"], seed=c["seed"])
    eng = _engine(ds)
    th = torch.from_numpy(theta).cuda()
    full = torch.empty(len(theta), dtype=torch.float64, device="cuda")
    eng.loglike_device(th, full)
    ref = full.cpu().numpy()
    for world in (2, 4, 8, 3):
        parts = []
        for r in range(world):
            lo, hi = shard_bounds(len(theta), world, r)
            o = torch.empty(hi - lo, dtype=torch.float64, device="cuda")
            eng.loglike_device(th[lo:hi], o)
            parts.append(o)
        got = torch.cat(parts).cpu().numpy()
        assert np.array_equal(got, ref), f"world={world}"


def test_device_posterior_layouts_bitwise():
    lpost, x0 = make_posterior(4, 8192, device=0)
    dp = lpost.device_posterior()
    eng = lpost.log_likelihood.engine
    eng.set_lanes_per_walker(64)
    a = dp(x0)
    eng.set_lanes_per_walker(32)
    b = dp(x0)
    eng.set_lanes_per_walker(0)
    assert np.isfinite(a).sum() > 7000
    assert np.array_equal(a, b)


def test_sampler_logprob_equals_plain_kernel():
    """The fused stretch-move kernel (one wave per walker) stores, for the last step, exactly
    the log-posterior the plain kernel gives those positions in a 16384-walker (segmented) batch."""
    from ravest_amd.sampler import DeviceEnsembleSampler
    lpost, x0 = make_posterior(2, 16384, device=0)
    dp = lpost.device_posterior()
    lp0 = dp(x0)
    good = np.isfinite(lp0)
    x0[~good] = x0[good][:(~good).sum()]
    s = DeviceEnsembleSampler(lpost, len(x0), seed=7)
    s.run_mcmc(x0, 3)
    last = s.get_chain()[-1]
    assert np.array_equal(s.get_log_prob()[-1], dp(last))
