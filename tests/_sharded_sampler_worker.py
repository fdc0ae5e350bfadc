"""Worker of tests/test_gpu_sharded_sampler.py: one rank of ShardedDeviceSampler (launched by
torch.distributed.run).  Backend from RVK_TEST_BACKEND (gloo: every rank on cuda:0, the gathers
staged through host memory; nccl: one GPU per rank, RCCL -- also at world size 1, where every
collective still runs through RCCL); rank 0 writes the chain to argv[1].

Besides the sampler (keep_chain=0: the chain on rank 0 only, get_autocorr_time computed there and
broadcast) it drives ShardedDevicePosterior on a config-2 walker block whose size divides the
world (the in-place all-gather) and, when the world is > 1, one that does not (the padded
branch), and records one evaluation of the whole block on this rank for the bitwise check."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gp_posterior(W):
    """A GP log-posterior of the reference's golden case a and W finite starting walkers."""
    from tests.test_gpu_gp64 import _gpost, _load_gp_case
    c = _load_gp_case("a")
    gp = _gpost(c, "fp64")
    return gp, np.ascontiguousarray(c["x"][np.isfinite(c["log_prob"])][:W])


def main():
    import torch
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDevicePosterior, ShardedDeviceSampler
    from ravest_amd.synth import make_config, make_posterior
    backend = os.environ.get("RVK_TEST_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    world, rank = dist.get_world_size(), dist.get_rank()
    W, steps = int(sys.argv[2]), int(sys.argv[3])
    gp = len(sys.argv) > 4 and sys.argv[4] == "gp"
    if gp:                                           # GPFitter.run_mcmc's posterior (reference goldens, case a)
        lpost, x0 = gp_posterior(W)
    else:
        lpost, x0 = make_posterior(2, W, seed=4, device=local)
    s = ShardedDeviceSampler(lpost, W, seed=77, steps_per_call=4, keep_chain=0)
    assert s.grouped
    s.run_mcmc(x0, steps)
    tau = s.get_autocorr_time(tol=0)                 # computed on rank 0, broadcast to every rank
    res = {}
    if backend == "nccl" and not gp:                 # device-resident posterior sharding (config 4's form)
        from ravest_amd.engine import RVEngine
        ds = make_config(2, n_walkers=4096 + 3)
        eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=local)
        th = torch.from_numpy(ds.theta).cuda()
        sh = ShardedDevicePosterior(eng.loglike_device)
        assert sh.grouped
        for tag, n in (("even", 4096 - 4096 % world), ("padded", 4096 + 3)):
            if tag == "padded" and n % world == 0:
                continue                             # world 1: every block divides
            out = sh(th[:n])
            ref = torch.empty(n, dtype=torch.float64, device=th.device)
            eng.loglike_device(th[:n], ref)
            torch.cuda.synchronize()
            res[f"post_{tag}"] = out.cpu().numpy()
            res[f"post_{tag}_ref"] = ref.cpu().numpy()
    if rank == 0:
        np.savez(sys.argv[1], chain=s.get_chain(), lnp=s.get_log_prob(), nacc=s.naccepted, x0=x0,
                 xbytes=s.exchange_bytes_per_half_step, tau=tau, world=world, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
