"""bench.py -- walker log-prob throughput of the MI355X RV engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

A "step" is one pass of the hot path over one batch: the per-walker
log-likelihood of a W-walker ensemble (config 2: 1 planet x 256 epochs x
4096 walkers per GPU, fp64) with theta already resident in HBM, i.e. one
rvk_loglike_device launch.  With N > 1 each rank evaluates its own 4096-walker
shard (weak scaling) and the per-walker log-probs are all-gathered over RCCL
(the exchange back to the stretch move); all-gathers are
pipelined one step behind the kernels on RCCL's stream.

Rank 0 prints ONE JSON line (metric/value = Kepler solves/s over all GPUs,
plus the roofline of the dominant kernel measured live with HIP events and a
bounded CPU baseline of the C oracle on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VECTOR_PEAK_TF = 78.6     # MI355X FP64 vector peak (spec; half the FP32 vector rate)
FP32_MFMA_PEAK_TF = 157.3      # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
FP64_MATRIX_PEAK_TF = 78.6     # MI355X FP64 matrix peak (spec; v_mfma_f64_16x16x4_f64), dense
BYTES_PER_WALKER_EPOCH = 28    # t, v, sigma fp64 + int32 inst


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--walkers", type=int, default=None, help="walkers per GPU (default: config's, 4096 for cfg 2)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sampler", action="store_true", help="skip the device stretch-move measurement")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-buffer drop-in latencies")
    ap.add_argument("--group", action="store_true",
                    help="start the process group and take the N>1 code path (RCCL all-gathers) even at N=1")
    ap.add_argument("--graph-steps", type=int, default=50, help="steps captured per HIP graph")
    ap.add_argument("--gather", choices=["graph", "stream", "none"], default="graph",
                    help="N>1 (RCCL): the K launches and the all-gathers captured in one HIP graph (default) "
                         "or issued from the host per group")
    ap.add_argument("--gather-steps", type=int, default=None,
                    help="N>1: steps whose log-probs one all-gather carries (default K: one gather per region)")
    ap.add_argument("--streams", type=int, default=1, help="independent streams per graph (--launch graph)")
    ap.add_argument("--launch", choices=["eager", "graph"], default="graph",
                    help="timed loop: G-step HIP graph replays (default) or back-to-back stream launches")
    ap.add_argument("--no-gp", action="store_true", help="skip the config-5 GP likelihood measurement")
    ap.add_argument("--no-predictive", action="store_true", help="skip the posterior-predictive measurement")
    ap.add_argument("--no-configs", action="store_true", help="skip the config-3 / config-4 sub-measurements")
    return ap.parse_args()


def cpu_baseline(ds, theta, budget_s):
    """Time the C oracle (oracle/rv_oracle.c, OpenMP over walkers) on a bounded sample."""
    from oracle import oracle
    threads = host_threads()
    n_ep, n_pl = len(ds.time), len(ds.planet_letters)
    sample = theta[: min(len(theta), 4096)]
    oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                   ds.parameterisation.code, ds.t0, sample[:64], nthreads=threads)   # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        _, used = oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                                 ds.parameterisation.code, ds.t0, sample, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    solves = reps * len(sample) * n_ep * n_pl
    # single-core scalar leg (emcee's serial map), ~1/4 of the budget
    one = sample[:256]
    r1, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < budget_s / 4:
        oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl,
                       ds.parameterisation.code, ds.t0, one, nthreads=1)
        r1 += 1
    el1 = time.perf_counter() - t1
    # vectorised NumPy leg (the reference arithmetic over a whole walker block
    # with NumPy arrays, one thread -- what a ravest user gets without numba), ~1/4 of the budget
    from threadpoolctl import threadpool_limits
    from oracle import np_oracle
    blk = sample[:512]
    r2, t2 = 0, time.perf_counter()
    with threadpool_limits(1):
        while time.perf_counter() - t2 < budget_s / 4:
            np_oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl, ds.t0, blk)
            r2 += 1
    el2 = time.perf_counter() - t2
    return {"value": solves / el, "unit": "Kepler solves/s", "cores": used, "kind": "port",
            "per_core_value": solves / el / max(1, used), "host_cpus": host_cpu_info(),
            "sample": f"{reps} x {len(sample)} walkers x {n_ep} epochs x {n_pl} planet(s) of the same "
                      f"config-{ds.cfg} ensemble, C oracle (oracle/rv_oracle.c, fp64, OpenMP), {el:.1f} s",
            "single_core_value": r1 * len(one) * n_ep * n_pl / el1,
            "numpy_vectorised_value": r2 * len(blk) * n_ep * n_pl / el2,
            "numpy_sample": f"{r2} x {len(blk)} walkers, oracle/np_oracle.py (NumPy over [W, N] arrays, 1 thread), "
                            f"{el2:.1f} s"}


def host_threads() -> int:
    """Threads for the CPU baseline: every CPU this process may run on (sched_getaffinity),
    but no more than the job's CPU share when the launcher states one (OMP_NUM_THREADS: the
    GPU pool sets it to the 16 CPUs one GPU's job may use, and its rules forbid worker pools
    beyond that share; nproc there shows the whole multi-GPU host, which other GPUs' jobs
    share).  The line reports both counts (cpu_baseline.host_cpus) and the per-core rate."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def host_cpu_info() -> dict:
    return {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "threads_used": host_threads()}


def agreement(ds, theta, ll, world, k: int = 512) -> dict:
    """Log-prob agreement of the measured kernel's output with the C restatement of the reference
    (oracle/rv_oracle.c, pinned to the reference's golden vectors) on the first k walkers of this
    rank, against the stated fp64 tolerance |d| <= 1e-9 max(1, |ref|) and an identical -inf mask;
    for N > 1, `ranks_bitwise_identical` is set by main(): the all-gathered block of every rank's
    results against rank 0's own single evaluation of all N x W walkers."""
    from oracle import oracle
    ref, _ = oracle.loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments),
                            len(ds.planet_letters), ds.parameterisation.code, ds.t0, theta[:k],
                            nthreads=host_threads())
    got = ll[:k]
    fin = np.isfinite(ref)
    rel = np.abs(got[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
    return {"walkers_checked": int(k), "mask_identical": bool(np.array_equal(np.isfinite(got), fin)),
            "max_rel_err": float(rel.max()) if rel.size else 0.0, "tolerance": 1e-9,
            "ranks_bitwise_identical": None}


# MI355X VALU issue costs (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost' / SIMD-32: a wave64
# instruction issues over 2 cycles; fp64 runs at half the fp32 rate -> 4; transcendentals 8 (f32),
# 16 (f64, assumed at the same 1/2 ratio)); 1024 SIMDs at 2.4 GHz.
N_SIMD, CLOCK_HZ = 1024, 2.4e9


def valu_roofline(pmc: dict | None, kern_ms: float) -> dict | None:
    """The binding resource of the likelihood kernel: fp64 VALU.  From the PMC counters of the
    same kernel (profiles/pmc_config<N>.json, separate rocprofv3 --pmc passes): the fp64 FLOP
    rate against the 78.6 TF fp64 vector peak, and an issue-cycle estimate (instructions x
    their SIMD issue cycles / (1024 SIMDs x 2.4 GHz x kernel time))."""
    if not pmc:
        return None
    c = pmc.get("counters_per_launch", {})
    if not c.get("SQ_INSTS_VALU_FLOPS_FP64"):
        return None
    t = kern_ms * 1e-3
    f64 = c["SQ_INSTS_VALU_FLOPS_FP64"] * 64 / t / 1e12     # per-wave-instruction FLOP count x 64 lanes
    f32 = c.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) * 64 / t / 1e12
    n64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
    tr64, tr32 = c.get("SQ_INSTS_VALU_TRANS_F64", 0.0), c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    other = max(0.0, c.get("SQ_INSTS_VALU", 0.0) - n64 - tr64 - tr32)
    cycles = 4 * n64 + 16 * tr64 + 8 * tr32 + 2 * other
    return {"bound": "valu-fp64", "fp64_tflops": f64, "peak_fp64_tflops": FP64_VECTOR_PEAK_TF,
            "fp64_flop_frac": f64 / FP64_VECTOR_PEAK_TF, "fp32_tflops": f32,
            "issue_cycle_frac_est": cycles / (N_SIMD * CLOCK_HZ * t),
            "valu_insts_per_launch": c.get("SQ_INSTS_VALU"), "kernel": pmc.get("kernel"),
            "source": (pmc.get("source") or "") + " (profiles/%s)" % pmc.get("_file", "")}


def csrc_digest() -> str:
    """sha256 over the kernel sources and build flags (ravest_amd/csrc/*, include/*.h,
    ravest_amd/Makefile), names and bytes, sorted: the provenance stamp of every
    profiles/pmc_*.json (tools/pmc_summary.py writes it; the .git directory does not travel
    to the GPU box, so the stamp is a content hash, not a commit id)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "ravest_amd", "csrc", "*")) +
                   glob.glob(os.path.join(ROOT, "include", "*.h")) + [os.path.join(ROOT, "ravest_amd", "Makefile")])
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.relpath(f, ROOT).encode() + b"\0")
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def load_pmc_file(name):
    """A committed PMC summary, or None when it was measured on other kernel sources than this
    tree's (its csrc_sha256 stamp differs from csrc_digest()): a stale counter file must not
    turn a kernel change into a silently wrong fraction."""
    p = os.path.join(ROOT, "profiles", name)
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        d["_file"] = name
        if d.get("csrc_sha256") != csrc_digest():
            return None
        return d
    return None


def pmc_provenance(name) -> dict:
    p = os.path.join(ROOT, "profiles", name)
    stamp = None
    if os.path.exists(p):
        with open(p) as f:
            stamp = json.load(f).get("csrc_sha256")
    return {"file": "profiles/" + name, "csrc_sha256": stamp, "tree_csrc_sha256": csrc_digest(),
            "matches_tree": stamp is not None and stamp == csrc_digest()}


def graph_kernel_ms(launch, G: int = 20, reps: int = 10) -> float:
    """Average duration of `launch(stream)` (one kernel launch) inside G-launch HIP graph replays,
    HIP events on the replay stream, median over reps."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    cap = torch.cuda.Stream(dev)
    for _ in range(3):
        launch(cap)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for _ in range(G):
            launch(cap)
    g.replay()
    torch.cuda.synchronize(dev)
    st = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(st)
        g.replay()
        b.record(st)
    torch.cuda.synchronize(dev)
    return float(np.median([a.elapsed_time(b) for a, b in evs])) / G


def config_line(cfg: int, W: int | None = None, label: str | None = None) -> dict:
    """One more BASELINE config on this GPU (theta resident in HBM): kernel ms (HIP events around
    graph replays), Kepler solves/s, the algorithmic-HBM and fp64-VALU rooflines, and log-prob
    agreement with the C oracle on 512 walkers."""
    import torch
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    ds = make_config(cfg, n_walkers=W)
    ds.cfg = cfg
    W = len(ds.theta)
    n_ep, n_pl = len(ds.time), len(ds.planet_letters)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), n_pl, ds.parameterisation,
                   ds.t0, device=dev.index)
    th = torch.from_numpy(ds.theta).to(dev)
    out = torch.empty(W, dtype=torch.float64, device=dev)
    ms = graph_kernel_ms(lambda st: eng.loglike_device(th, out, st))
    torch.cuda.synchronize(dev)
    ll = out.cpu().numpy()
    alg = W * (n_ep * BYTES_PER_WALKER_EPOCH + ds.theta.shape[1] * 8 + 8)
    gbs = alg / (ms * 1e-3) / 1e9
    pmc = load_pmc_file(f"pmc_{label or 'config%d' % cfg}.json")
    return {"config": f"config {cfg}: {n_pl} planet(s), {n_ep} epochs, {W} walkers, {len(ds.unique_instruments)} "
                      f"instrument(s), fp64, theta resident in HBM",
            "kernel_ms": ms, "kepler_solves_per_s": W * n_ep * n_pl / (ms * 1e-3),
            "walker_evals_per_s": W / (ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "traffic": (pmc or {}).get("fabric_bytes_per_launch"),
                         "valu": valu_roofline(pmc, ms),
                         "pmc": pmc_provenance(f"pmc_{label or 'config%d' % cfg}.json")},
            "n_masked_walkers": int((~np.isfinite(ll)).sum()),
            "logprob_agreement": agreement(ds, ds.theta, ll, 1)}


def config4_sharded_line(world: int, rank: int, backend: str, grouped: bool = False, reps: int = 20) -> dict:
    """Config 4 as BASELINE names it: 65536 walkers (2 planets x 512 epochs) split over the N
    ranks (strong scaling, 65536/N contiguous walkers each) by ShardedDevicePosterior: each rank
    launches rvk_loglike_device on its slice and the per-walker log-probs are all-gathered (RCCL
    over xGMI) into every rank's [65536] buffer.  Timed: reps x (launch + all-gather) from a
    common start (barrier + sync) to each rank's own synchronize, max over ranks.  Checked: the gathered block equals rank 0's own single
    evaluation of all 65536 walkers, bit for bit."""
    import torch
    import torch.distributed as dist
    from ravest_amd.distributed import ShardedDevicePosterior
    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import make_config
    ds = make_config(4)
    Wt = len(ds.theta)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), len(ds.planet_letters),
                   ds.parameterisation, ds.t0, device=dev.index)
    th = torch.from_numpy(ds.theta).to(dev)
    out = torch.empty(Wt, dtype=torch.float64, device=dev)
    if world > 1 and backend != "nccl":
        return {"skipped": "gloo rehearsal: the device-resident all-gather needs RCCL (backend nccl)"}
    sh = ShardedDevicePosterior(eng.loglike_device)
    for _ in range(3):
        sh(th, out)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        sh(th, out)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0                    # this rank's end; max over ranks below
    ref = torch.empty(Wt, dtype=torch.float64, device=dev)
    eng.loglike_device(th, ref)
    torch.cuda.synchronize(dev)
    same = bool(np.array_equal(ref.cpu().numpy(), out.cpu().numpy()))
    if world > 1:
        t = torch.tensor([el, 0.0 if same else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, same = float(t[0]), bool(t[1] == 0.0)
    n_ep, n_pl = len(ds.time), len(ds.planet_letters)
    solves = Wt * n_ep * n_pl * reps
    return {"config": f"config 4: {n_pl} planets, {n_ep} epochs, {Wt} walkers sharded over {world} GPU(s) "
                      f"({Wt // world} per rank), RCCL all-gather of the log-probs into every rank",
            "ms_per_eval": el / reps * 1e3, "kepler_solves_per_s": solves / el, "walker_evals_per_s": Wt * reps / el,
            "scaling": "strong", "n_gpus": world,
            "bitwise_identical_to_single_gpu": same}


def _stretch_raw_ms(lpost, x0, steps: int, warm: int = 16, seed: int = 1234, flags: int = 0) -> tuple:
    """ms per emcee step of rvk_stretch_run alone (state, draws and chain in HBM, no host copies),
    HIP events on the launch stream; and the acceptance fraction."""
    import torch
    from ravest_amd import _lib
    from ravest_amd.posterior import DevicePosterior
    W, D = x0.shape
    dp = DevicePosterior(lpost)
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.from_numpy(x0).to(dev)
    lp = torch.empty(W, dtype=torch.float64, device=dev)
    dp.device(x, lp)
    chain = torch.empty((steps, W, D), dtype=torch.float64, device=dev)
    lnpc = torch.empty((steps, W), dtype=torch.float64, device=dev)
    nacc = torch.zeros(W, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    L = _lib.load()
    st = torch.cuda.current_stream(dev)

    def run(n, step0):
        _lib.check(L.rvk_stretch_run(dp._p, x.data_ptr(), lp.data_ptr(), W, n, 2.0, seed, step0, flags, 0, 0, 0, 0,
                                     chain.data_ptr(), lnpc.data_ptr(), nacc.data_ptr(), status.data_ptr(),
                                     st.cuda_stream))
    run(warm, 0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    run(steps, warm)
    b.record(st)
    torch.cuda.synchronize(dev)
    acc = float(nacc.sum().item()) / ((steps + warm) * W)
    if int(status.item()):
        raise RuntimeError("NaN log-probability in the sampler benchmark")
    return a.elapsed_time(b) / steps, acc


def sampler_line(W: int, steps: int = 256, e2e_steps: int = 2048) -> dict:
    """Device-resident stretch move on the config-2 posterior: (1) ms per emcee
    step of rvk_stretch_run alone (proposals, priors, likelihood, accept/reject, chain into HBM;
    emcee 3's randomised split drawn on the device); (2) the wall-clock a Fitter user sees:
    DeviceEnsembleSampler.run_mcmc of e2e_steps steps from call to return with the chain kept in
    HBM (the default), then get_chain() (one copy to host memory), and the same run with the
    chain copied to host memory chunk by chunk (chain_storage="host"); next to the host stretch
    move driving the same posterior (numpy + LogPosterior.log_probability_batch)."""
    import torch
    from ravest_amd.sampler import DeviceEnsembleSampler, EnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, W, device=torch.cuda.current_device())
    D = x0.shape[1]
    dev_ms, acc = _stretch_raw_ms(lpost, x0, steps)
    e2e = {}
    for storage in ("device", "host"):
        s = DeviceEnsembleSampler(lpost, W, seed=1234, chain_storage=storage)
        s.run_mcmc(x0, 2 * s.steps_per_call)             # warm: buffers, pinned staging
        s.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.run_mcmc(x0, e2e_steps)
        t1 = time.perf_counter()
        chain = s.get_chain()
        t2 = time.perf_counter()
        assert chain.shape == (e2e_steps, W, D)
        e2e[storage] = ((t1 - t0) / e2e_steps * 1e3, (t2 - t1) * 1e3)
        del s, chain
    host = host_stretch_ms(lpost, x0)
    host_ms = host["routed_ms_per_step"]
    variants = {}
    for name, cfg, prior, Wv in (("config2_beta_e", 2, "beta", W), ("config2_vaneylen_e", 2, "vaneylen", W),
                                 ("config3", 3, "uniform", 16384)):
        lp_v, x_v = make_posterior(cfg, Wv, device=torch.cuda.current_device(), e_prior=prior)
        ms_v, acc_v = _stretch_raw_ms(lp_v, x_v, 64 if cfg == 3 else steps)
        variants[name] = {"walkers": Wv, "free_parameters": x_v.shape[1], "e_prior": prior, "ms_per_step": ms_v,
                          "walker_steps_per_s": Wv / (ms_v * 1e-3), "acceptance": acc_v}
    return {"what": f"device stretch move (rvk_stretch_run), config-2 posterior, {W} walkers, {D} free parameters, "
                    "Philox draws with emcee 3's randomised split, chain in HBM", "ms_per_step": dev_ms,
            "posteriors": variants,
            "walker_steps_per_s": W / (dev_ms * 1e-3), "acceptance": acc,
            "run_mcmc_e2e_ms_per_step": e2e["device"][0], "run_mcmc_e2e_over_kernel": e2e["device"][0] / dev_ms,
            "get_chain_ms": e2e["device"][1],
            "run_mcmc_e2e_host_chain_ms_per_step": e2e["host"][0],
            "run_mcmc_e2e_host_chain_over_kernel": e2e["host"][0] / dev_ms,
            "run_mcmc_e2e_note": f"DeviceEnsembleSampler.run_mcmc of {e2e_steps} steps, call to return: chain kept in "
                                 "HBM (default; get_chain_ms = the one copy of the whole chain to host memory "
                                 "afterwards) / chain_storage='host' (256-step chunks copied to host memory on a "
                                 "copy stream while the next chunk runs)",
            "host_stretch_move_ms_per_step": host_ms, "host_stretch_move": host,
            "speedup_vs_host": host_ms / dev_ms}


def _med_us(fn, reps: int) -> float:
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def host_stretch_ms(lpost, x0, steps: int = 40) -> dict:
    """emcee's stretch move on the host (sampler.EnsembleSampler: emcee 3.1's numpy step, its
    RandomState call order) driving the drop-in LogPosterior.log_probability_batch -- the
    north-star integration (fit.py:1068-1075) -- ms per step, median of 3 runs, with the phases
    split: the sampler's own numpy work (the same step over a zero log-prob) and the drop-in's
    two calls per step; plus the same step over the round-3 route (host priors, pageable copies)."""
    from ravest_amd.sampler import EnsembleSampler
    W, D = x0.shape

    def per_step(fn):
        s = EnsembleSampler(W, D, fn, seed=1)
        s.run_mcmc(x0, 2)
        runs = []
        for _ in range(3):
            s.reset()
            t0 = time.perf_counter()
            s.run_mcmc(x0, steps)
            runs.append((time.perf_counter() - t0) / steps * 1e3)
        return float(np.median(runs))

    eng = lpost.log_likelihood.engine
    routed = per_step(lpost.log_probability_batch)
    zero = per_step(lambda q: np.zeros(len(q)))
    q = np.ascontiguousarray(x0[: W // 2])
    call_us = _med_us(lambda: lpost.log_probability_batch(q), 200)
    saved = lpost._route
    lpost._route = "host"
    eng.set_hostio("pageable")
    old = per_step(lpost.log_probability_batch)
    old_call_us = _med_us(lambda: lpost.log_probability_batch(q), 100)
    lpost._route = saved
    eng.set_hostio("auto")
    return {"routed_ms_per_step": routed, "sampler_numpy_ms_per_step": zero,
            "drop_in_us_per_call": call_us, "drop_in_calls_per_step": 2,
            "round3_route_ms_per_step": old, "round3_route_us_per_call": old_call_us,
            "note": f"{W} walkers, {W // 2} per call; routed = device priors (rvk_logpost) + RVK_HOSTIO_AUTO; "
                    "round3 route = host numpy/scipy priors + pageable copies (route='host', RVK_HOSTIO_PAGEABLE)"}


def host_path_line(W: int = 4096) -> dict:
    """The host-buffer drop-in calls a ravest user makes: LogPosterior
    .log_probability_batch at emcee's half-ensemble (W/2 walkers), the scalar
    log_probability(dict) MAP calls O(10^3) times (fit.py:548-604), and the raw rvk_loglike of W
    walkers, per RVK_OPT_HOSTIO transport (median us per call); and a Powell MAP on the 51 Peg
    golden (ravest's find_map_estimate: scipy.optimize.minimize(method="Powell") over
    _negative_log_probability_for_MAP)."""
    from scipy.optimize import minimize

    from ravest_amd import prior as P
    from ravest_amd.param import Parameterisation
    from ravest_amd.posterior import LogPosterior
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, W, device=0)
    eng = lpost.log_likelihood.engine
    H = W // 2
    q = np.ascontiguousarray(x0[:H])
    d1 = dict(zip(lpost.free_params_names, x0[0]))
    full = np.ascontiguousarray(lpost._full(x0))
    res = {}
    for mode in ("pageable", "pinned", "zerocopy", "auto"):
        eng.set_hostio(mode)
        res[mode] = {"log_probability_batch_H_us": _med_us(lambda: lpost.log_probability_batch(q), 200),
                     "log_probability_dict_us": _med_us(lambda: lpost.log_probability(d1), 400),
                     "rvk_loglike_W_us": _med_us(lambda: eng.loglike(full), 200)}
    eng.set_hostio("auto")
    lpost._route = "host"
    res["round3_route_host_priors"] = {"log_probability_batch_H_us": _med_us(lambda: lpost.log_probability_batch(q), 100),
                                       "log_probability_dict_us": _med_us(lambda: lpost.log_probability(d1), 200)}
    lpost._route = "device"
    # Powell MAP on the reference's 51 Peg b golden posterior (tests/golden/logpost_51peg.npz)
    g = np.load(os.path.join(ROOT, "tests", "golden", "logpost_51peg.npz"))
    m = json.loads(str(g["meta"]))
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    lp51 = LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], g["time"], g["vel"], g["velerr"], g["instrument"],
                        np.array(m["unique_instruments"]), m["t0"], device=0)
    start = g["theta_free"][np.argmax(g["log_prob"])]
    lp51._negative_log_probability_for_MAP(start)
    t0 = time.perf_counter()
    r = minimize(lp51._negative_log_probability_for_MAP, start, method="Powell")
    el = time.perf_counter() - t0
    return {"what": f"host-buffer drop-in calls, config-2 posterior ({W} walkers, {x0.shape[1]} free parameters); "
                    "median us per call", "per_transport": res,
            "map_51peg_powell": {"evaluations": int(r.nfev), "seconds": el, "us_per_evaluation": el / r.nfev * 1e6,
                                 "success": bool(r.success), "neg_log_post": float(r.fun)}}


def config4_sampler_line(world: int, rank: int, backend: str, grouped: bool = False, steps: int = 32) -> dict:
    """Config 4 as a sampler: 65536 walkers (2 planets x 512 epochs, 14 free parameters).  N = 1:
    DeviceEnsembleSampler's kernel (rvk_stretch_run, one fused kernel per half-step); N > 1:
    ShardedDeviceSampler (each rank evaluates 32768 / N proposals per half-step, the 32768
    log-posteriors all-gathered: 256 KB per half-step), run_mcmc timed from a common start (barrier) to each rank's own end, max over
    ranks, chain kept on rank 0's host."""
    import torch
    import torch.distributed as dist
    from ravest_amd.synth import make_posterior
    W = 65536
    lpost, x0 = make_posterior(4, W, device=torch.cuda.current_device())
    D = x0.shape[1]
    if not grouped:
        ms, acc = _stretch_raw_ms(lpost, x0, steps, warm=4)
        return {"what": f"config-4 posterior, {W} walkers, {D} free parameters, 1 GPU, rvk_stretch_run (chain in HBM)",
                "ms_per_step": ms, "walker_steps_per_s": W / (ms * 1e-3),
                "kepler_solves_per_s": W * 512 * 2 / (ms * 1e-3), "acceptance": acc}
    from ravest_amd.distributed import ShardedDeviceSampler
    s = ShardedDeviceSampler(lpost, W, seed=1234, steps_per_call=steps, keep_chain=0)
    s.run_mcmc(x0, 4)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run_mcmc(None, steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0                    # this rank's end; max over ranks below
    t = torch.tensor([el], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t[0]) / steps * 1e3
    how = "RCCL all-gather" if backend == "nccl" else f"{backend} all-gather through host memory (rehearsal, not a GPU number)"
    return {"what": f"config-4 posterior, {W} walkers, {D} free parameters, ShardedDeviceSampler over {world} ranks "
                    f"({how} of {W // 2} log-probs per half-step = {s.exchange_bytes_per_half_step} B)",
            "ms_per_step": ms, "walker_steps_per_s": W / (ms * 1e-3), "kepler_solves_per_s": W * 512 * 2 / (ms * 1e-3),
            "acceptance": float(s.acceptance_fraction.mean()), "n_gpus": world}


def mfma_pmc(pmc, flop: float, mops_key: str):
    """From a GP kernel's PMC summary: the matrix pipe's busy fraction (SQ_VALU_MFMA_BUSY_CYCLES
    over 1024 SIMDs / GRBM_GUI_ACTIVE over 8 XCDs) and the MFMA FLOP issued (MOPS x 512) against
    the algorithmic FLOP; None when the counters are missing or stale."""
    if not pmc:
        return None
    c = pmc.get("counters_per_launch", {})
    res = {"pmc": pmc.get("_file")}
    if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
        res["mfma_busy_frac"] = (c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024) / (c["GRBM_GUI_ACTIVE"] / 8)
    if c.get(mops_key):
        res["mfma_flop_issued_over_algorithmic"] = c[mops_key] * 512 / flop
    return res


def gp_line(W: int = 4096, n: int = 512, reps: int = 10) -> dict:
    """Config 5: batched quasi-periodic GP log-likelihood, 1 planet, 512
    epochs, 4096 walkers, fp32 factorisation (rvk_gp_loglike_device), theta/hyper resident in
    HBM; HIP events around `reps` back-to-back launches on the launch stream.  Roofline: fp32
    MFMA, algorithmic FLOP per walker = n^3/3 (Cholesky) + 2 n^2 (the carried rhs).  CPU
    baseline: the fp64 restatement (oracle/gp_oracle.py, scipy Cholesky), one BLAS thread."""
    import torch
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(W, n_epochs=n)
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                         ds.parameterisation, GPKernel("Quasiperiodic"), device=torch.cuda.current_device(),
                         precision="fp32+fp64")
    dev = torch.device("cuda", torch.cuda.current_device())
    tt, ht = torch.from_numpy(th).to(dev), torch.from_numpy(hy).to(dev)
    out = torch.empty(W, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    for _ in range(2):
        gp.device(tt, ht, out, st)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        gp.device(tt, ht, out, st)
    b.record(st)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    flop = W * (n ** 3 / 3.0 + 2.0 * n * n)
    tf = flop / (ms * 1e-3) / 1e12
    from threadpoolctl import threadpool_limits
    from oracle import gp_oracle
    k = 24
    with threadpool_limits(1):
        gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[:2], hy[:2])
        t0 = time.perf_counter()
        ref = gp_oracle.gp_loglike(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, 0, ds.t0, th[:k], hy[:k])
        cpu_s = (time.perf_counter() - t0) / k
    # the reference's precision (fp64 throughout, RVK_GP_FP64): same batch, same timing method
    gp64 = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments,
                           ds.planet_letters, ds.parameterisation, GPKernel("Quasiperiodic"),
                           device=torch.cuda.current_device(), precision="fp64")
    out64 = torch.empty(W, dtype=torch.float64, device=dev)
    gp64.device(tt, ht, out64, st)
    a.record(st)
    for _ in range(2):
        gp64.device(tt, ht, out64, st)
    b.record(st)
    torch.cuda.synchronize(dev)
    ms64 = a.elapsed_time(b) / 2
    tf64 = flop / (ms64 * 1e-3) / 1e12
    o64, o32 = out64.cpu().numpy()[:k], out.cpu().numpy()[:k]
    fin = np.isfinite(ref)
    rel = lambda x: float(np.max(np.abs(x[fin] - ref[fin]) / np.abs(ref[fin]))) if fin.any() else 0.0   # noqa: E731
    pmc32, pmc64 = load_pmc_file("pmc_config5.json"), load_pmc_file("pmc_config5_fp64.json")
    return {"config": f"config 5: 1 planet + quasi-periodic GP, {n} epochs, {W} walkers, fp32 factorisation",
            "ms_per_eval": ms, "walker_evals_per_s": W / (ms * 1e-3),
            "roofline": {"bound": "mfma", "achieved": tf, "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s",
                         "frac": tf / FP32_MFMA_PEAK_TF,
                         "traffic": (pmc32 or {}).get("fabric_bytes_per_launch"),
                         "pmc": pmc_provenance("pmc_config5.json"), "mfma_counters": mfma_pmc(pmc32, flop,
                                                                                          "SQ_INSTS_VALU_MFMA_MOPS_F32"),
                         "note": "algorithmic FLOP = W*(n^3/3 + 2n^2) per launch / launch duration; traffic = "
                                 "L2 memory-side (fabric) bytes per launch, FETCH_SIZE x 2 + WRITE_SIZE as "
                                 "MI355X_MICROARCH.md prescribes (PMC, profiles/pmc_config5.json): it counts "
                                 "Infinity-Cache hits too -- the workspace tiles re-read by the left-looking "
                                 "update -- so it bounds HBM bytes from above"},
            "n_masked_walkers": int((~np.isfinite(out.cpu().numpy())).sum()),
            "precision": "fp32 factorisation, fp64 re-evaluation of walkers it rejects (opt-in: precision='fp32+fp64'; "
                         "the drop-in's default is fp64, the 'fp64' entry)",
            "max_rel_err_vs_fp64_oracle": rel(o32),
            "fp64": {"precision": "fp64 factorisation (the default: the reference's precision)",
                     "ms_per_eval": ms64, "walker_evals_per_s": W / (ms64 * 1e-3),
                     "roofline": {"bound": "mfma", "achieved": tf64, "peak": FP64_MATRIX_PEAK_TF, "unit": "TFLOP/s",
                                  "frac": tf64 / FP64_MATRIX_PEAK_TF,
                                  "traffic": (pmc64 or {}).get("fabric_bytes_per_launch"),
                                  "pmc": pmc_provenance("pmc_config5_fp64.json"),
                                  "mfma_counters": mfma_pmc(pmc64, flop, "SQ_INSTS_VALU_MFMA_MOPS_F64")},
                     "max_rel_err_vs_fp64_oracle": rel(o64),
                     "mask_identical": bool(np.array_equal(np.isfinite(o64), fin))},
            "cpu_baseline": {"value": 1.0 / cpu_s, "unit": "walker evals/s", "cores": 1, "kind": "port",
                             "sample": f"{k} walkers, fp64 restatement (oracle/gp_oracle.py, scipy LAPACK, 1 thread)"}}


def predictive_line(eng, theta, S: int = 100_000, T: int = 1000, reps: int = 5) -> dict:
    """Posterior predictive (fit.py:2690-2824): total RV (planets + trend) of
    S posterior samples at T times, one rvk_predict_device launch over the dense [S, T] fp64
    grid (samples resampled from the config-2 walker block, times spanning the data), HIP events
    around `reps` launches.  Roofline: the [S, T] fp64 output written to HBM (8 B per solve);
    the Kepler solves are the same fp64-VALU work as the likelihood's."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    rng = np.random.default_rng(7)
    good = theta[np.all(np.isfinite(theta), axis=1)]
    samples = good[rng.integers(0, len(good), S)]
    samples = samples[(samples[:, 2] >= 0) & (samples[:, 2] < 1) & (samples[:, 1] > 0)]   # valid planets only
    S = len(samples)
    th = torch.from_numpy(np.ascontiguousarray(samples)).to(dev)
    tq = torch.linspace(0.0, 1000.0, T, dtype=torch.float64, device=dev)
    out = torch.empty((S, T), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    eng.predict_device(th, tq, out, stream=st)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        eng.predict_device(th, tq, out, stream=st)
    b.record(st)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    nbytes = S * T * 8 + S * th.shape[1] * 8 + T * 8
    gbs = nbytes / (ms * 1e-3) / 1e9
    ok = bool(torch.isfinite(out).all().item())
    del out
    pmc = load_pmc_file("pmc_predictive.json")
    return {"what": f"posterior predictive, {S} samples x {T} times, 1 planet + trend, fp64 [S, T] output in HBM",
            "ms_per_call": ms, "kepler_solves_per_s": S * T / (ms * 1e-3), "all_finite": ok,
            "roofline": {"bound": "valu-fp64", "valu": valu_roofline(pmc, ms),
                         "pmc": pmc_provenance("pmc_predictive.json"),
                         "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                 "traffic": (pmc or {}).get("fabric_bytes_per_launch")},
                         "note": "the Kepler solves bind it (fp64 VALU, 'valu': PMC counters of the same kernel, "
                                 "null unless measured on this tree's sources); hbm = 8*S*T output + 8*S*P_full "
                                 "samples + 8*T times per launch / launch time"}}


def n1_steps(args, eng, th_d, W: int, dev, ll):
    """The N = 1 timed loop.  graph (default): G-step HIP graphs replayed (S independent streams
    per graph); eager: K stream-ordered launches issued back to back through the C-ABI entry point
    (ctypes call pre-bound).  Measured on MI355X, config 2: at K = 20 (one replay) graph 8.6-8.7 us
    vs eager 8.9 us wall per step (eager's kernels run 0.25 us shorter, its host issue costs
    more); at K = 200 both 7.6 us.  Returns (elapsed s, kernel ms: HIP events around each group
    of G launches in the timed region / G, G)."""
    import torch
    stream = torch.cuda.current_stream(dev)
    G = max(1, min(args.graph_steps, args.steps))
    while args.steps % G:                            # time exactly K steps
        G -= 1
    S = max(1, args.streams)
    outs = torch.empty(G, W, dtype=torch.float64, device=dev)
    from ravest_amd import _lib
    ll_fn = _lib.load().rvk_loglike_device
    call_args = [(eng._h, th_d.data_ptr(), W, th_d.stride(0), outs[j].data_ptr(), stream.cuda_stream)
                 for j in range(G)]

    def run_group():
        for a in call_args:
            if ll_fn(*a):
                _lib.check(-1)

    if args.launch == "graph":
        cap = torch.cuda.Stream(dev)
        side = [torch.cuda.Stream(dev) for _ in range(S)]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            for st in side:
                st.wait_stream(cap)
            for j in range(G):
                eng.loglike_device(th_d, outs[j], side[j % S])
            for st in side:
                cap.wait_stream(st)
        g.replay()                                   # warm replay
        launch_group = g.replay                      # replayed on `stream`
    else:
        launch_group = run_group
    launch_group()
    torch.cuda.synchronize(dev)
    if not np.array_equal(outs[G - 1].cpu().numpy(), ll):
        raise RuntimeError("timed-loop launch result differs from the first eager launch")
    out1 = torch.empty(W, dtype=torch.float64, device=dev)
    for _ in range(max(1, args.warmup)):             # the W untimed warmup steps, right before the region
        eng.loglike_device(th_d, out1, stream)
    rep_ev = []
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps // G):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        launch_group()
        b.record(stream)
        rep_ev.append((a, b))
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    kern_ms = float(sum(a.elapsed_time(b) for a, b in rep_ev)) / args.steps
    return el, kern_ms, G


def grouped_steps(args, eng, th_d, W: int, world: int, backend: str, dev) -> dict:
    """The N > 1 timed loop (weak scaling; also run at world 1 by --group).

    K steps in R = K / G groups of G launches; after each group its G x W log-probs are
    all-gathered (RCCL over xGMI) into a buffer of their own (no buffer is reused inside the
    region, so no gather waits for an earlier one).  Default G = K: ONE all-gather of all K
    steps' log-probs at the end of the region.  --gather graph (the default with RCCL): the
    whole region -- the K launches on one stream and the R all-gathers on RCCL's stream -- is
    captured once into one HIP graph and the timed region is one replay, so the host issues one
    call instead of K launches and R collectives.  --gather stream: the same work issued from
    the host every region (one G-launch graph replay + one async all-gather per group).  gloo
    (the 1-GPU rehearsal): stream form, gathers staged through host memory.  --gather none: the
    graph without the gathers (probe only; the bitwise check then fails by construction).
    Measured at RCCL world 1 on one MI355X (tools/group_sweep.sh, profiles/round6/): graph, G = 20
    8.39-8.68 us per step against 8.68-9.32 for the N = 1 line of the same session; each further
    gather inside the graph adds ~20-25 us per region (G = 10: 10.3-11.5, G = 5: 12.3-14.4, G = 2:
    16.6-17.5) although the gather itself is a 3 us copy at world 1 -- the cost is the forked
    branch's cross-queue dependencies, not the bytes; host-issued (stream, G = 20) 10.6-10.8.

    Timing: the region starts at a common point (barrier + synchronize on every rank, then
    each rank's clock), ends on each rank when its own stream work (kernels and gathers) has
    completed (synchronize), and the elapsed times are MAX-reduced after the region -- no
    collective other than the gathers inside it.  kernel_ms: HIP events around a K-launch
    graph of the kernel alone on this rank's stream, replayed right before the region (the
    gather kernels would overlap events inside the captured region)."""
    import torch
    import torch.distributed as dist
    K = args.steps
    G = min(args.gather_steps or K, K)
    while K % G:
        G -= 1
    R = K // G
    mode = args.gather if backend == "nccl" else "stream"
    stream = torch.cuda.current_stream(dev)
    outs = [torch.empty(G, W, dtype=torch.float64, device=dev) for _ in range(R)]
    gath = [torch.empty(world * G * W, dtype=torch.float64, device=dev) for _ in range(R)]
    cap = torch.cuda.Stream(dev)

    def issue_all(st):
        """K launches on `st` and R async all-gathers (the current stream must be `st`)."""
        works = []
        for r in range(R):
            for j in range(G):
                eng.loglike_device(th_d, outs[r][j], st)
            if mode != "none":                        # "none": the same graph without the gathers (probe)
                works.append(dist.all_gather_into_tensor(gath[r], outs[r].view(-1), async_op=True))
        for w in works:
            w.wait()

    # warm every gather buffer and RCCL's channels eagerly (the communicator exists already:
    # init_process_group(device_id=...) initialises it eagerly)
    if backend == "nccl":
        with torch.cuda.stream(cap):
            issue_all(cap)
        torch.cuda.synchronize(dev)

    graph = None
    if mode in ("graph", "none"):
        ok, err = 1, ""
        try:
            if os.environ.get("RVK_BENCH_NO_CAPTURE") == os.environ.get("RANK", "0"):   # exercises the fallback
                raise RuntimeError("capture refused on this rank by RVK_BENCH_NO_CAPTURE")
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=cap, capture_error_mode="thread_local"):
                issue_all(cap)
        except Exception as e:                        # capture of the collective refused on this rank
            ok, err, graph = 0, str(e), None
        torch.cuda.synchronize(dev)
        # The choice must be the same on every rank: a rank that replays a graph holding the
        # all-gather while another took the host-issued form would wait in that gather for a
        # peer that never joins it.  Capture runs nothing, so no collective has run yet.
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 1:
            graph.replay()                            # warm replay
            torch.cuda.synchronize(dev)
            region = graph.replay
        else:                                         # host-issued form on every rank
            why = err or "on another rank"
            print(f"bench.py: HIP-graph capture of the all-gather failed ({why}); using --gather stream",
                  file=sys.stderr, flush=True)
            graph, mode = None, "stream"
    if graph is None:
        gg = []
        for r in range(R):                            # G-launch kernel graphs, one per output buffer
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                for j in range(G):
                    eng.loglike_device(th_d, outs[r][j], cap)
            gg.append(g)
        for g in gg:
            g.replay()
        torch.cuda.synchronize(dev)

        def region():
            works = []
            for r in range(R):
                gg[r].replay()
                if backend == "nccl":
                    works.append(dist.all_gather_into_tensor(gath[r], outs[r].view(-1), async_op=True))
                else:
                    hb = torch.empty(world * G * W, dtype=torch.float64)
                    dist.all_gather_into_tensor(hb, outs[r].view(-1).cpu())
                    gath[r].copy_(hb)
            for w in works:
                w.wait()

    kern_ms = graph_kernel_ms(lambda st: eng.loglike_device(th_d, outs[0][0], st), G=K)
    out1 = torch.empty(W, dtype=torch.float64, device=dev)
    for _ in range(max(1, args.warmup)):             # the W untimed warmup steps, right before the region
        eng.loglike_device(th_d, out1, stream)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    region()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"el": float(t[0]), "kern_ms": float(t[1]), "G": G, "R": R, "mode": mode,
            "last": gath[R - 1].view(world, G, W)[:, G - 1, :].reshape(-1)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RVK_BENCH_BACKEND=gloo: rehearsal of the N>1 path on a 1-GPU box (ranks share cuda:0, the
    # all-gather goes through host memory); the real multi-GPU run uses RCCL ("nccl").
    backend = os.environ.get("RVK_BENCH_BACKEND", "nccl")
    grouped = world > 1 or args.group        # --group: the N>1 path (collectives) on one GPU
    if grouped:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29541"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from ravest_amd.engine import RVEngine
    from ravest_amd.synth import CONFIGS, make_dataset, make_walkers
    c = CONFIGS[args.config]
    W = args.walkers or (c["n_walkers"] if args.config != 4 else c["n_walkers"] // 8)
    ds = make_dataset(c["n_planets"], c["n_epochs"], c["n_inst"], seed=c["seed"])
    ds.cfg = args.config
    theta_all = make_walkers(ds, W * world, seed=c["seed"])
    theta = theta_all[rank * W:(rank + 1) * W]
    n_ep, n_pl, n_in = len(ds.time), len(ds.planet_letters), len(ds.unique_instruments)

    eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, n_in, n_pl, ds.parameterisation, ds.t0,
                   device=dev.index)
    eng.reserve(W)                                   # no allocation inside captured launches
    th_d = torch.from_numpy(theta).to(dev)
    stream = torch.cuda.current_stream(dev)

    # ---- isolated per-launch kernel duration (HIP events on the launch stream) -----------
    out1 = torch.empty(W, dtype=torch.float64, device=dev)
    for _ in range(max(1, args.warmup)):
        eng.loglike_device(th_d, out1, stream)
    torch.cuda.synchronize(dev)
    ll = out1.cpu().numpy()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record(stream)
        eng.loglike_device(th_d, out1, stream)
        b.record(stream)
    torch.cuda.synchronize(dev)
    eager_ms = float(np.median([a.elapsed_time(b) for a, b in ev]))   # includes event/launch overhead

    # PCIe-inclusive host-buffer path (rvk_loglike: H2D theta, kernel, D2H), for DESIGN.md only
    # median of 200 blocking calls (skipped with --no-host-path: these zero-copy launches of the same
    # kernel read theta over PCIe, so they would mix into a profile's per-kernel average)
    host_ms = None if args.no_host_path else _med_us(lambda: eng.loglike(theta), 200) * 1e-3

    # ---- the timed steps -------------------------------------------------------------------
    G, S, gmode = None, max(1, args.streams), None
    ranks_same = None
    if grouped:
        res = grouped_steps(args, eng, th_d, W, world, backend, dev)
        el, kern_ms, G, gmode = res["el"], res["kern_ms"], res["G"], res["mode"]
        # every rank's results, as gathered, against THIS rank's own single launch over all
        # world x W walkers (a different batch size, so possibly a different lane layout):
        # bitwise identical means the shard split changes nothing
        got = res["last"].cpu().numpy()
        th_all = torch.from_numpy(theta_all).to(dev)
        ref_all = torch.empty(world * W, dtype=torch.float64, device=dev)
        eng.loglike_device(th_all, ref_all, stream)
        torch.cuda.synchronize(dev)
        bad = 0.0 if np.array_equal(got, ref_all.cpu().numpy()) and np.array_equal(got[rank * W:(rank + 1) * W], ll) \
            else 1.0
        t = torch.tensor([bad], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ranks_same = bool(t[0] == 0.0)
        del th_all, ref_all
    else:
        el, kern_ms, G = n1_steps(args, eng, th_d, W, dev, ll)

    solves = W * n_ep * n_pl * args.steps * world
    value = solves / el
    if rank == 0:
        alg_bytes = W * (n_ep * BYTES_PER_WALKER_EPOCH + theta.shape[1] * 8 + 8)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        pmc = load_pmc_file(f"pmc_config{args.config}.json")
        traffic = pmc.get("fabric_bytes_per_launch") if pmc else None
        valu = valu_roofline(pmc, kern_ms)
        line = {
            "metric": "walker-log-prob evals/sec (= Kepler solves/sec) at 1/2/4/8 MI355X",
            "value": value, "unit": "Kepler solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"config {args.config}: {n_pl} planet(s), {n_ep} epochs, {W} walkers per GPU, "
                                   f"fp64, theta resident in HBM" + (
                                       (", RCCL all-gather of log-probs" if backend == "nccl" else
                                        f", {backend} all-gather of log-probs (host-staged rehearsal)")
                                       if world > 1 else ""),
                       "n_planets": n_pl, "n_epochs": n_ep, "walkers_per_gpu": W, "n_inst": n_in,
                       "parameterisation": ds.parameterisation.parameterisation,
                       "parallelism": f"walker-shard x{world}"},
            "walker_evals_per_s": W * world * args.steps / el,
            "kernel_ms": kern_ms,
            "eager_event_ms": eager_ms,
            "host_path_ms_per_call": host_ms,
            "launch": ((f"{G}-step HIP graphs, {S} streams" if args.launch == "graph" else
                        "back-to-back stream launches") if not grouped else
                       (f"all {args.steps} launches + {args.steps // G} all-gathers (one per {G} steps) captured in one "
                        "HIP graph, one replay" if gmode == "graph" else
                        f"{G}-step HIP graph replays, 1 async all-gather per {G} steps issued from the host")),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "achieved_per_step": alg_bytes / (el / args.steps) / 1e9,
                         "valu": valu, "pmc": pmc_provenance(f"pmc_config{args.config}.json"),
                         "note": "achieved = algorithmic bytes W*(28*N_epochs + 8*P_full + 8) per launch (SURVEY "
                                 "§8(d)) / average kernel duration (HIP events around each group of G "
                                 "launches in the timed region / G); traffic = L2 memory-side (fabric) bytes per launch, "
                                 "FETCH_SIZE x 2 + WRITE_SIZE (PMC; counts Infinity-Cache hits, so an upper bound "
                                 "on HBM bytes: the epoch arrays are re-read from L2/MALL). The binding resource "
                                 "is fp64 VALU issue: 'valu' (PMC counters of the same kernel, null unless "
                                 "pmc.matches_tree: measured on this tree's kernel sources)."},
        }
        line["n_masked_walkers"] = int((~np.isfinite(ll)).sum())
        line["logprob_agreement"] = agreement(ds, theta, ll, world)
        line["logprob_agreement"]["ranks_bitwise_identical"] = ranks_same
        if world == 1 and args.config == 2 and not args.no_configs:
            line["config3"] = config_line(3)
            line["config4_shard"] = config_line(4, W=8192)
        if world == 1 and not args.no_sampler:
            line["sampler"] = sampler_line(W)
        if world == 1 and not args.no_host_path:
            line["host_path"] = host_path_line(W)
        if world == 1 and not args.no_gp:
            line["gp_config5"] = gp_line()
        if world == 1 and not args.no_predictive:
            line["predictive"] = predictive_line(eng, theta)
        if world == 1 and not args.no_cpu_baseline:     # rank 0 at N = 1 only (the other ranks would wait)
            line["cpu_baseline"] = cpu_baseline(ds, theta, args.cpu_seconds)
    if not args.no_configs:
        c4 = config4_sharded_line(world, rank, backend, grouped)   # collective: every rank takes part
        if rank == 0:
            line["config4_sharded"] = c4
    if not args.no_sampler:
        c4s = config4_sampler_line(world, rank, backend, grouped)  # collective for N > 1
        if rank == 0:
            line["config4_sampler"] = c4s
    if rank == 0:
        if grouped:
            line["process_group"] = {"backend": backend, "world_size": world, "gather": gmode,
                                     "note": "timed loop with the N>1 path (grouped_steps): each group's log-probs "
                                             "all-gathered into a buffer of its own; the region starts after a "
                                             "barrier + synchronize, ends at each rank's own synchronize, max over "
                                             "ranks; kernel_ms from a kernel-only K-launch graph before the region"}
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
