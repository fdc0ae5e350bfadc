"""Config 5 (1 planet + quasi-periodic GP, 512 epochs, 4096 walkers, fp32 factorisation):
GP log-likelihood walker-evals/s on one MI355X (HIP events around a 5-launch graph replay),
and the fp64 CPU restatement (oracle/gp_oracle.py, one core) on a bounded sample.

usage: python tools/gp_bench.py [W=4096] [n_epochs=512] [precision=fp32+fp64]
"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import torch
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    prec = sys.argv[3] if len(sys.argv) > 3 else "fp32+fp64"
    ds, th, hy = make_gp_config(W, n_epochs=n)
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                         ds.parameterisation, GPKernel("Quasiperiodic"), device=0, precision=prec)
    tt, ht = torch.from_numpy(th).cuda(), torch.from_numpy(hy).cuda()
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    gp.device(tt, ht, out, s)
    torch.cuda.synchronize()
    reps = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        gp.device(tt, ht, out, s)
        b.record(s)
        torch.cuda.synchronize()
        reps.append(a.elapsed_time(b))
    ms = float(np.median(reps))
    flop = W * (n ** 3 / 3.0 + 2.0 * n * n)   # Cholesky + forward solve (per walker)
    res = {"config": f"config 5: 1 planet + QP GP, {n} epochs, {W} walkers, precision {prec}", "ms_per_eval": ms,
           "walker_evals_per_s": W / (ms * 1e-3), "chol_tflops": flop / (ms * 1e-3) / 1e12,
           "n_masked": int((~np.isfinite(out.cpu().numpy())).sum())}
    from oracle import gp_oracle
    k = 16
    if prec == "fp64":
        ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[:64], hy[:64])
        got = out.cpu().numpy()[:64]
        fin = np.isfinite(ref)
        res["max_rel_err_vs_fp64_oracle_64w"] = float(np.max(np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])))
        res["mask_identical"] = bool(np.array_equal(np.isfinite(got), fin))
    t0 = time.perf_counter()
    gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[:k], hy[:k])
    cpu = (time.perf_counter() - t0) / k
    res["cpu_oracle_walker_evals_per_s_1core"] = 1.0 / cpu
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
