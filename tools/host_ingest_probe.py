"""Probe: landing a sampler chunk (58.7 MB) in fresh pageable host memory: plain np.empty vs an
mmap with MADV_HUGEPAGE, single- and multi-threaded copies from pinned staging."""
import mmap
import time

import numpy as np
import torch


def fresh_hp(nbytes):
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m.madvise(mmap.MADV_HUGEPAGE)
    except Exception as e:
        print("madvise failed", e)
    return m


shape = (256, 4096, 7)
nb = int(np.prod(shape)) * 8
src = torch.randn(shape, dtype=torch.float64, device="cuda")
stage = torch.empty(shape, dtype=torch.float64, pin_memory=True)
stage.copy_(src)
torch.cuda.synchronize()
print("THP:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
      open("/sys/kernel/mm/transparent_hugepage/defrag").read().strip())
for name, mk in (("np.empty", lambda: np.empty(shape)),
                 ("mmap+MADV_HUGEPAGE", lambda: np.frombuffer(fresh_hp(nb), dtype=np.float64).reshape(shape))):
    for how in ("numpy", "torch"):
        ts = []
        for _ in range(5):
            dst = mk()
            t0 = time.perf_counter()
            if how == "numpy":
                np.copyto(dst, stage.numpy())
            else:
                torch.from_numpy(dst).copy_(stage)
            ts.append(time.perf_counter() - t0)
        print(f"{name:22s} {how:6s} {1e3 * np.median(ts):7.2f} ms  {nb / np.median(ts) / 1e9:6.1f} GB/s")
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    p = torch.empty((8,) + shape, dtype=torch.float64, pin_memory=True)
    ts.append(time.perf_counter() - t0)
    del p
print("pinned alloc 470 MB (cached allocator may reuse):", [round(1e3 * t, 2) for t in ts], "ms")
t0 = time.perf_counter()
keep = [torch.empty(shape, dtype=torch.float64, pin_memory=True) for _ in range(8)]
print("8 fresh pinned 58.7 MB buffers:", round(1e3 * (time.perf_counter() - t0), 2), "ms")
