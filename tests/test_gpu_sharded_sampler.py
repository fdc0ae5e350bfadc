"""ShardedDeviceSampler (ravest_amd/distributed.py, include/rvk_post.h rvk_stretch_draws /
rvk_stretch_propose / rvk_stretch_update): every rank evaluates a slice of each half-step's
proposals, the H log-posteriors are all-gathered (H x 8 bytes) and every rank applies the
accept / reject to the whole half.  One rank on the GPU (the propose / update kernels, no
collective), two ranks over gloo on one MI355X, and two ranks over RCCL when the box has two
GPUs; the chain, log-probs and acceptance counts must equal the single-GPU DeviceEnsembleSampler
with the same Philox seed bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _single(W, steps, randomize=True):
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, W, seed=4)
    s = DeviceEnsembleSampler(lpost, W, seed=77, steps_per_call=5, randomize_split=randomize)
    s.run_mcmc(x0, steps)
    return s


@pytest.mark.parametrize("randomize", [True, False])
def test_sharded_sampler_one_rank_equals_single_gpu(randomize):
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDeviceSampler
    from ravest_amd.synth import make_posterior
    assert not (dist.is_available() and dist.is_initialized())
    W, steps = 256, 12
    lpost, x0 = make_posterior(2, W, seed=4)
    sh = ShardedDeviceSampler(lpost, W, seed=77, steps_per_call=4, randomize_split=randomize)
    sh.run_mcmc(x0, steps)
    ref = _single(W, steps, randomize)
    assert np.array_equal(sh.get_chain(), ref.get_chain())
    assert np.array_equal(sh.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(sh.naccepted, ref.naccepted)
    assert sh.exchange_bytes_per_half_step == (W // 2) * 8


def _single_gp(W, steps):
    from ravest_amd.sampler import DeviceEnsembleSampler
    from tests._sharded_sampler_worker import gp_posterior
    gp, x0 = gp_posterior(W)
    s = DeviceEnsembleSampler(gp, W, seed=77, steps_per_call=5)
    s.run_mcmc(x0, steps)
    return s


def test_sharded_gp_sampler_one_rank_equals_single_gpu():
    """GPFitter.run_mcmc's sampler sharded (rvk_gp_stretch_draws / _propose / _update) equals the
    single-GPU rvk_gp_stretch_run chain bit for bit (no process group: one rank)."""
    from ravest_amd.distributed import ShardedDeviceSampler
    from tests._sharded_sampler_worker import gp_posterior
    W, steps = 32, 8
    gp, x0 = gp_posterior(W)
    sh = ShardedDeviceSampler(gp, W, seed=77, steps_per_call=3)
    sh.run_mcmc(x0, steps)
    ref = _single_gp(W, steps)
    assert np.array_equal(sh.get_chain(), ref.get_chain())
    assert np.array_equal(sh.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(sh.naccepted, ref.naccepted) and ref.naccepted.sum() > 0
    assert sh.exchange_bytes_per_half_step == (W // 2) * 8


def _run_ranks(tmp_path, backend, port, W=256, steps=40, nproc=2, gp=False):
    out = tmp_path / f"chain_{backend}_{nproc}{'_gp' if gp else ''}.npz"
    env = dict(os.environ, RVK_TEST_BACKEND=backend, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "_sharded_sampler_worker.py"),
           str(out), str(W), str(steps)] + (["gp"] if gp else [])
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    assert int(got["world"]) == nproc
    ref = _single_gp(W, steps) if gp else _single(W, steps)
    assert np.array_equal(got["chain"], ref.get_chain())
    assert np.array_equal(got["lnp"], ref.get_log_prob())
    assert np.array_equal(got["nacc"], ref.naccepted)
    assert int(got["xbytes"]) == (W // 2) * 8
    assert got["nacc"].sum() > 0
    tau_ref = ref.get_autocorr_time(tol=0)
    # long enough that every walker has moved: a finite estimate for every parameter, so the
    # broadcast from the chain's rank is checked on real values, not on NaN == NaN
    assert np.all(np.isfinite(tau_ref)), tau_ref
    assert np.array_equal(got["tau"], tau_ref)
    for tag in ("even", "padded"):
        if f"post_{tag}" in got.files:
            assert np.array_equal(got[f"post_{tag}"], got[f"post_{tag}_ref"]), tag
    return got


def test_sharded_sampler_two_ranks_gloo(tmp_path):
    _run_ranks(tmp_path, "gloo", 29533)


def test_sharded_gp_sampler_two_ranks_gloo(tmp_path):
    """GPFitter.run_mcmc's sampler over two ranks (gloo, both on cuda:0): each rank evaluates half of
    every half-step's GP proposals; the chain equals the single-GPU GP sampler's bit for bit."""
    _run_ranks(tmp_path, "gloo", 29536, W=32, steps=60, gp=True)


def test_rccl_world_one_gp(tmp_path):
    _run_ranks(tmp_path, "nccl", 29537, W=32, steps=60, nproc=1, gp=True)


def test_rccl_world_one(tmp_path):
    """Every RCCL branch on a one-GPU box: a world-size-1 "nccl" process group (torch.distributed.run,
    one process) drives ShardedDeviceSampler's all-gather of the H log-posteriors (RCCL, in place on
    device buffers), its get_autocorr_time broadcast from the chain's rank, and
    ShardedDevicePosterior's in-place all_gather_into_tensor; chain, log-probs, acceptance counts,
    tau and the gathered log-probs equal the single-GPU evaluation bit for bit."""
    got = _run_ranks(tmp_path, "nccl", 29535, nproc=1)
    assert "post_even" in got.files


def test_sharded_sampler_two_ranks_rccl(tmp_path):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("the RCCL form needs two GPUs (the driver's 8-GPU node)")
    _run_ranks(tmp_path, "nccl", 29534)


def test_sharded_unfused_path_equals_single_gpu():
    """P_full > 64 (1 planet, 29 instruments): the two-kernel half-step.  One GPU runs propose_kernel
    + the 64-lane sampling kernel over the whole half; the sharded form (rvk_stretch_propose) runs
    propose_kernel + the plain posterior kernel over its slice, whose lanes-per-walker layout is
    chosen per launch (32 lanes at 8192 proposals).  The per-walker reduction does not depend on
    the layout (tests/test_gpu_layout.py), so the chains are equal bit for bit."""
    from ravest_amd import prior as P
    from ravest_amd.distributed import ShardedDeviceSampler
    from ravest_amd.posterior import LogPosterior
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_dataset
    ds = make_dataset(1, 96, 29, seed=17)
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    assert len(ds.names) > 64
    priors = {}
    for n in free:
        v, base = ds.truth[n], n.split("_")[0]
        priors[n] = (P.EccentricityUniform(0.99) if base == "e" else P.Uniform(-np.pi, np.pi) if base == "w"
                     else P.HalfNormal(5.0) if base == "jit" else P.Uniform(v - 0.5 * abs(v) - 1.0, v + 0.5 * abs(v) + 1.0))
    lpost = LogPosterior(ds.planet_letters, ds.parameterisation, priors, {"gd": 0.0, "gdd": 0.0}, free, ds.time,
                         ds.vel, ds.velerr, ds.instrument, ds.unique_instruments, ds.t0)
    W = 16384
    rng = np.random.default_rng(3)
    x0 = np.array([ds.truth[n] for n in free])[None, :] * (1 + 1e-4 * rng.standard_normal((W, len(free))))
    a = DeviceEnsembleSampler(lpost, W, seed=19, steps_per_call=3)
    a.run_mcmc(x0, 6)
    b = ShardedDeviceSampler(lpost, W, seed=19, steps_per_call=3)
    b.run_mcmc(x0, 6)
    assert np.array_equal(a.get_chain(), b.get_chain()) and np.array_equal(a.get_log_prob(), b.get_log_prob())
    assert np.array_equal(a.naccepted, b.naccepted) and a.naccepted.sum() > 0
