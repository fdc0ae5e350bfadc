"""Per-phase trace of the config-2 likelihood kernel (build with -DRVK_LL_TRACE=1, tools/ll_trace.sh):
for 4 sampled blocks x 4 waves: s_memrealtime at entry/exit (100 MHz, global) and s_memtime (shader
cycles) after the first-epoch loads, the prep, the barrier, the epoch loop, the reduction, the store."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd import _lib
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import CONFIGS, make_dataset, make_walkers
    c = CONFIGS[2]
    ds = make_dataset(c["n_planets"], c["n_epochs"], c["n_inst"], seed=c["seed"])
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    th = make_walkers(ds, W, seed=c["seed"])
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
    eng.reserve(W)
    t = torch.from_numpy(th).cuda()
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    for _ in range(50):
        eng.loglike_device(t, out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        eng.loglike_device(t, out)
    b.record()
    torch.cuda.synchronize()
    print(f"W={W}: {a.elapsed_time(b) / 50 * 1e3:.2f} us per launch (eager, incl. launch gaps)")
    buf = np.zeros((16, 8), dtype=np.uint64)
    assert _lib.load().rvk_ll_trace_dump(buf.ctypes.data_as(C.c_void_p)) == 0
    r0 = buf[:, 0].astype(np.int64).min()
    print("wave  start_ns  end_ns | cycles: prep  barrier  epochs  reduce  store(+tail)")
    for i in range(16):
        b = buf[i].astype(np.int64)
        print(f"{i:3d} {(b[0]-r0)*10:8d} {(b[7]-r0)*10:8d} | {b[2]-b[1]:6d} {b[3]-b[2]:7d} {b[4]-b[3]:7d} {b[5]-b[4]:7d} {b[6]-b[5]:7d}")


if __name__ == "__main__":
    main()
