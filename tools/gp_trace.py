"""Per-phase s_memtime trace of the GP kernel (build with -DRVK_GP_TRACE=1, tools/gp_trace.sh):
one config-5 launch, then the first walker of block 0, per step k and wave: factor, next-column
accumulation, B1 wait, S1, B2 wait, S2 (cycles)."""
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
                         ds.parameterisation, GPKernel("Quasiperiodic"), device=0, precision="fp32+fp64")
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    for _ in range(2):
        gp.device(tt, ht, out)
    torch.cuda.synchronize()
    buf = np.zeros((8, 32, 8), dtype=np.uint64)
    lib = _lib.load()
    assert lib.rvk_gp_trace_dump(buf.ctypes.data_as(C.c_void_p)) == 0
    nw = 4 if buf[4:].max() == 0 else 8
    t0 = buf[:nw, 0, 0].min()
    names = ["factor", "part1", "B1wait", "S1", "B2wait", "S2"]
    tot = np.zeros(6)
    for k in range(16):
        row = []
        for w in range(nw):
            d = np.diff(buf[w, k, :7].astype(np.int64))
            tot += d
            row.append("/".join(f"{x:6d}" for x in d))
        print(f"k={k:2d} start {int(buf[0, k, 0] - t0):8d}  " + " | ".join(row))
    print("totals over waves:", dict(zip(names, tot.tolist())))
    print("walker cycles:", int(buf[:nw, 15, 3].max() - t0))
    for w in range(nw):
        hw = int(buf[w, 31, 7])
        print(f"wave {w}: HW_ID 0x{hw:08x} wave_id {hw & 15} simd {(hw >> 4) & 3} cu {(hw >> 8) & 15} se {(hw >> 13) & 7}")


if __name__ == "__main__":
    main()
