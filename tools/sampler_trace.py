"""Per-phase trace of the fused stretch-move half-step (loglike_kernel SAMPLE == 2) on the config-2
posterior (build: TUS=rvk_sample1 VAROUT=varlib/trace tools/varbuild.sh lltrace:-DRVK_LL_TRACE=1).  For sampled blocks x 4 waves of the
last launch: s_memrealtime at entry/exit (100 MHz) and s_memtime (shader cycles) after the
preload, the prep (proposal + planet constants), the barrier, the epoch loop, the reduction."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd import _lib
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    lpost, x0 = make_posterior(2, W, device=0)
    s = DeviceEnsembleSampler(lpost, W, seed=5)
    s.run_mcmc(x0, 16)
    torch.cuda.synchronize()
    buf = np.zeros((16, 8), dtype=np.uint64)
    L = _lib.load()
    dump = getattr(L, "rvk_ll_trace_dump_s1", None) or L.rvk_ll_trace_dump   # the sampler unit's stamps
    assert dump(buf.ctypes.data_as(C.c_void_p)) == 0
    r0 = buf[:12, 0].astype(np.int64).min()
    print("wave  start_ns  end_ns | cycles: preload->pass  prep (rows wait / compute)  epochs  reduce+epilogue")
    for i in range(12):
        b = buf[i].astype(np.int64)
        rows = f"({b[6]-b[3]:5d} / {b[2]-b[6]:5d})" if b[6] else ""
        print(f"{i:3d} {(b[0]-r0)*10:8d} {(b[7]-r0)*10:8d} | {b[3]-b[1]:6d} {b[2]-b[3]:7d} {rows} {b[4]-b[2]:7d} {b[5]-b[4]:7d}")


if __name__ == "__main__":
    main()
