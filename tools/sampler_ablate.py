"""Which part of DeviceEnsembleSampler's pipeline slows the device steps?  8 x rvk_stretch_run(256)
back to back: alone; + a D2H copy of each chunk on a copy stream; + a host memcpy of 58 MB per
chunk; + both.  GPU ms per chunk from events around each call."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from ravest_amd import _lib
    from ravest_amd.posterior import DevicePosterior
    from ravest_amd.sampler import _host_array
    from ravest_amd.synth import make_posterior
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lpost, x0 = make_posterior(2, 4096, device=0)
    W, D, n = 4096, x0.shape[1], 256
    dp = DevicePosterior(lpost)
    x = torch.from_numpy(x0).to(dev)
    lp = torch.empty(W, dtype=torch.float64, device=dev)
    dp.device(x, lp)
    bufs = [(torch.empty((n, W, D), dtype=torch.float64, device=dev), torch.empty((n, W), dtype=torch.float64, device=dev))
            for _ in range(2)]
    stage = [torch.empty((n, W, D), dtype=torch.float64, pin_memory=True) for _ in range(2)]
    nacc = torch.zeros(W, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    L = _lib.load()
    st = torch.cuda.current_stream(dev)
    cs = torch.cuda.Stream(dev)
    host = _host_array((8 * n, W, D))
    out = {}
    for mode in ("alone", "d2h", "memcpy", "both", "alone"):
        evs = []
        step = 0
        for k in range(8):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            ch, lc = bufs[k % 2]
            _lib.check(L.rvk_stretch_run(dp._p, x.data_ptr(), lp.data_ptr(), W, n, 2.0, 7, step, 0, 0, 0, 0, 0,
                                         ch.data_ptr(), lc.data_ptr(), nacc.data_ptr(), status.data_ptr(),
                                         st.cuda_stream))
            b.record(st)
            step += n
            if mode in ("d2h", "both"):
                cs.wait_event(b)
                with torch.cuda.stream(cs):
                    stage[k % 2].copy_(ch, non_blocking=True)
            if mode in ("memcpy", "both") and k > 0:
                torch.from_numpy(host[(k - 1) * n:k * n]).copy_(stage[(k - 1) % 2])
            evs.append((a, b))
        torch.cuda.synchronize()
        out.setdefault(mode, []).append([round(a.elapsed_time(b), 3) for a, b in evs])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
