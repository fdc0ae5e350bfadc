"""Worker of tests/test_gpu_sharded_sampler.py: one rank of ShardedDeviceSampler (launched by
torch.distributed.run).  Backend from RVK_TEST_BACKEND (gloo: every rank on cuda:0, the gathers
staged through host memory; nccl: one GPU per rank, RCCL); rank 0 writes the chain to argv[1]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDeviceSampler
    from ravest_amd.synth import make_posterior
    backend = os.environ.get("RVK_TEST_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    W, steps = int(sys.argv[2]), int(sys.argv[3])
    lpost, x0 = make_posterior(2, W, seed=4, device=local)
    s = ShardedDeviceSampler(lpost, W, seed=77, steps_per_call=4, keep_chain=0)
    s.run_mcmc(x0, steps)
    if dist.get_rank() == 0:
        np.savez(sys.argv[1], chain=s.get_chain(), lnp=s.get_log_prob(), nacc=s.naccepted, x0=x0,
                 xbytes=s.exchange_bytes_per_half_step)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
