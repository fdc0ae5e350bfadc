"""Per-phase cost of a blocking host-buffer call (rvk_loglike, RVK_HOSTIO_AUTO), config 2.

Phases timed separately (median us):
  * py+ctypes: engine.loglike's Python work around the C call (np.ascontiguousarray, np.empty);
  * memcpy_in: the user's theta copied into pinned fine-grained staging (what HostIO does);
  * launch_sync: the kernel on device-resident input with the output in HBM, launch + stream
    synchronize wall time (the floor of any blocking call);
  * kernel_hbm / kernel_zerocopy: event-timed kernel with theta in HBM vs read from pinned host
    memory over PCIe (the zero-copy transport);
  * call_<mode>: the whole rvk_loglike call per transport.
Usage: python tools/host_phase_probe.py [W]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med_us(fn, n=300):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


def main():
    import torch
    from ravest_amd import _lib
    from ravest_amd.synth import make_posterior
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    lpost, x0 = make_posterior(2, W, device=0)
    eng = lpost.log_likelihood.engine
    theta = np.ascontiguousarray(lpost._full(x0))
    W, P = theta.shape
    res = {"W": W, "P_full": P, "theta_bytes": theta.nbytes}
    L, F = _lib.load(), _lib.fast()
    out = np.empty(W)
    for mode in ("pageable", "pinned", "zerocopy", "auto"):
        eng.set_hostio(mode)
        res[f"call_{mode}_us"] = med_us(lambda: eng.loglike(theta))
    eng.set_hostio("auto")
    res["raw_ctypes_call_us"] = med_us(lambda: F.rvk_loglike(eng._h, _lib.addr(theta), W, P, _lib.addr(out)))
    res["py_wrapper_us"] = med_us(lambda: (np.ascontiguousarray(np.atleast_2d(theta), np.float64), np.empty(W)))
    pin = torch.empty(theta.shape, dtype=torch.float64, pin_memory=True)
    pn = pin.numpy()
    res["memcpy_in_us"] = med_us(lambda: np.copyto(pn, theta))
    small = np.empty(W)
    pin_o = torch.empty(W, dtype=torch.float64, pin_memory=True).numpy()
    res["memcpy_out_us"] = med_us(lambda: np.copyto(small, pin_o))
    st = torch.cuda.current_stream()
    th_d = torch.from_numpy(theta).cuda()
    o_d = torch.empty(W, dtype=torch.float64, device="cuda")

    def dev_call(src_ptr):
        L.rvk_loglike_device(eng._h, src_ptr, W, P, o_d.data_ptr(), st.cuda_stream)
        st.synchronize()
    res["launch_sync_us"] = med_us(lambda: dev_call(th_d.data_ptr()))
    res["launch_sync_zerocopy_in_us"] = med_us(lambda: dev_call(pin.data_ptr()))
    def dev_query(src_ptr):
        L.rvk_loglike_device(eng._h, src_ptr, W, P, o_d.data_ptr(), st.cuda_stream)
        while not st.query():
            pass
    res["launch_queryspin_us"] = med_us(lambda: dev_query(th_d.data_ptr()))
    po = torch.empty(W, dtype=torch.float64, pin_memory=True)
    pov = po.numpy().view(np.int64)
    SENT = np.int64(0x7FF4DEADBEEF0001)

    def dev_sentinel(src_ptr):
        pov[:] = SENT
        L.rvk_loglike_device(eng._h, src_ptr, W, P, po.data_ptr(), st.cuda_stream)
        while (pov == SENT).any():
            pass
    res["launch_sentinelspin_us"] = med_us(lambda: dev_sentinel(th_d.data_ptr()))
    res["launch_sentinelspin_zerocopy_in_us"] = med_us(lambda: dev_sentinel(pin.data_ptr()))
    st.synchronize()
    res["sentinel_out_ok"] = bool(np.array_equal(po.numpy(), eng.loglike(theta)))
    for name, ptr in (("kernel_hbm_us", th_d.data_ptr()), ("kernel_zerocopy_in_us", pin.data_ptr())):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in ev:
            a.record(st)
            L.rvk_loglike_device(eng._h, ptr, W, P, o_d.data_ptr(), st.cuda_stream)
            b.record(st)
        torch.cuda.synchronize()
        res[name] = float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3)
    ref = eng.loglike(theta)
    assert np.array_equal(o_d.cpu().numpy(), ref)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
