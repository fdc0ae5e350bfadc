"""Per-step phase trace of the fp64 GP kernel (build with tools/gp64_trace.sh: -DRVK_GP64_TRACE=1):
for the first walker of block 0, per wave and step k, s_memtime (cycles) at: step start, after
the factor (owner) / immediately (others), after the accumulation (before B1), after B1, after S1
(before B2), after B2, after S2."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd import _lib
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ds, th, hy = make_gp_config(W, n_epochs=512)
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                         ds.parameterisation, GPKernel("Quasiperiodic"), device=0, precision="fp64")
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    gp.device(tt, ht, out)
    torch.cuda.synchronize()
    buf = np.zeros((8, 32, 8), dtype=np.uint64)
    assert _lib.load().rvk_gp64_trace_dump(buf.ctypes.data_as(C.c_void_p)) == 0
    b = buf.astype(np.int64)
    t0 = b[:, 0, 0].min()
    print("k | per wave: factor/idle  accum  B1wait  S1  B2wait  S2   (cycles); step total")
    for k in range(16):
        row = []
        for wv in range(8):
            x = b[wv, k]
            row.append(f"{x[1]-x[0]:6d}/{x[2]-x[1]:6d}/{x[3]-x[2]:6d}/{x[4]-x[3]:5d}/{x[5]-x[4]:5d}/{x[6]-x[5]:5d}")
        tot = b[:, k, 6].max() - b[:, k, 0].min() if k < 15 else b[:, k, 3].max() - b[:, k, 0].min()
        print(f"{k:2d} tot {tot:7d} | " + " ".join(row))
    print("walker total cycles:", b[:, 15, 3].max() - t0)
    # per wave, summed over steps 0..14: factor/idle, accumulation, B1 wait, S1, B2 wait, S2
    d = np.diff(b[:, :15, :7], axis=2).sum(axis=1)
    names = ["factor/idle", "accum", "B1wait", "S1", "B2wait", "S2"]
    for wv in range(8):
        print(f"wave {wv}: " + "  ".join(f"{n} {int(v)}" for n, v in zip(names, d[wv])))
    # which SIMD each wave of a workgroup runs on (HW_REG_HW_ID bits 5:4), over all blocks
    hw = np.zeros((1024, 8), dtype=np.uint32)
    lib = _lib.load()
    if callable(getattr(lib, "rvk_gp64_hwid_dump", None)) and lib.rvk_gp64_hwid_dump(hw.ctypes.data_as(C.c_void_p)) == 0:
        from collections import Counter
        simd = (hw[:256] >> 4) & 3
        pats = Counter(tuple(int(x) for x in r) for r in simd)
        print("wave -> SIMD patterns over 256 blocks (waves 0..7):")
        for pat, cnt in pats.most_common(8):
            print(f"  {pat}: {cnt}")


if __name__ == "__main__":
    main()
