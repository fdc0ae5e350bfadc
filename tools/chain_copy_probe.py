"""Probe: ways to land a sampler chunk's chain (device [n, W, D] fp64) in host memory.
Prints ms per 58.7 MB chunk (256 steps x 4096 walkers x 7 dims) for each way."""
import time

import numpy as np
import torch


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


dev = torch.device("cuda", 0)
n, W, D = 256, 4096, 7
src = torch.randn(n, W, D, dtype=torch.float64, device=dev)
nb = src.numel() * 8
res = {"bytes": nb}
res["cpu_pageable"] = t(lambda: src.cpu())
res["pinned_fresh_alloc+copy"] = t(lambda: torch.empty(src.shape, dtype=src.dtype, pin_memory=True).copy_(src))
stage = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
res["pinned_reused_copy"] = t(lambda: stage.copy_(src))
res["np_empty_copy_from_pinned"] = t(lambda: np.copyto(np.empty(src.shape), stage.numpy()))
res["torch_parallel_copy_into_np_empty"] = t(lambda: torch.from_numpy(np.empty(src.shape)).copy_(stage))
big = np.empty((8,) + tuple(src.shape))
res["np_preallocated_touched_copy"] = t(lambda: np.copyto(big[1], stage.numpy()))
res["copy_to_pageable_torch"] = t(lambda: torch.from_numpy(np.empty(src.shape)).copy_(src))
res["threads"] = torch.get_num_threads()
for k, v in res.items():
    print(f"{k:40s} {v}")
