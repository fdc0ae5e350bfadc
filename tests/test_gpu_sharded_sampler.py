"""ShardedDeviceSampler (ravest_amd/distributed.py, include/rvk_post.h rvk_stretch_half): the
device stretch move split over ranks by proposal slices, with the updated rows all-gathered every
half-step.  Rehearsed here with 2 ranks on one MI355X over gloo (the 8-GPU RCCL run is the
driver's); the chain, log-probs and acceptance counts must equal the single-GPU device sampler
with the same Philox seed bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _single(W, steps):
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, W, seed=4)
    s = DeviceEnsembleSampler(lpost, W, seed=77, steps_per_call=5)
    s.run_mcmc(x0, steps)
    return s


def test_sharded_sampler_one_rank_equals_single_gpu():
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDeviceSampler
    from ravest_amd.synth import make_posterior
    assert not (dist.is_available() and dist.is_initialized())
    W, steps = 256, 12
    lpost, x0 = make_posterior(2, W, seed=4)
    sh = ShardedDeviceSampler(lpost, W, seed=77)
    sh.run_mcmc(x0, steps)
    ref = _single(W, steps)
    assert np.array_equal(sh.get_chain(), ref.get_chain())
    assert np.array_equal(sh.get_log_prob(), ref.get_log_prob())
    assert np.array_equal(sh.naccepted, ref.naccepted)


def test_sharded_sampler_two_ranks_gloo(tmp_path):
    W, steps = 256, 10
    out = tmp_path / "chain.npz"
    env = dict(os.environ, RVK_TEST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", os.path.join(ROOT, "tests", "_sharded_sampler_worker.py"),
           str(out), str(W), str(steps)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    ref = _single(W, steps)
    assert np.array_equal(got["chain"], ref.get_chain())
    assert np.array_equal(got["lnp"], ref.get_log_prob())
    assert np.array_equal(got["nacc"], ref.naccepted)
    assert got["nacc"].sum() > 0
