"""Per-launch kernel timing (HIP events on the launch stream) for solver/config A/B in ONE process."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_config, make_dataset, make_walkers

def timeit(eng, th, out, reps=20, rounds=7, G=20):
    """us per launch: HIP events around replays of a G-launch HIP graph (as bench.py), median of rounds."""
    cap = torch.cuda.Stream()
    for _ in range(3):
        eng.loglike_device(th, out, cap)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for _ in range(G):
            eng.loglike_device(th, out, cap)
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    res = []
    for r in range(rounds):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in evs:
            a.record(s); g.replay(); b.record(s)
        torch.cuda.synchronize()
        res.append(np.median([a.elapsed_time(b) for a, b in evs]) / G)
    return float(np.median(res)) * 1e3  # us


def main():
    from ravest_amd import _lib
    from ravest_amd.engine import solve_kepler
    g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/kepler_grid.npz"))
    c, s_ = solve_kepler(g["M"], g["e"])
    tol = (1e-15 + 8e-16 * np.abs(g["M"])) / (1 - g["e"])
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH),
                      "kepler_grid_max_err_over_tol": float(max((np.abs(c - g["cosE"]) / tol).max(), (np.abs(s_ - g["sinE"]) / tol).max()))}), flush=True)
    out_rows = []
    cases = [("cfg2", make_config(2)), ("cfg3", make_config(3)), ("cfg4-shard", make_config(4, n_walkers=8192))]
    ds = make_dataset(1, 256, 1, seed=2, parameterisation="P K e w Tc"); ds.theta = make_walkers(ds, 4096, seed=2)
    cases.append(("cfg2-Tc", ds))
    ds = make_dataset(2, 512, 1, seed=4, parameterisation="P K secosw sesinw Tc"); ds.theta = make_walkers(ds, 8192, seed=4)
    cases.append(("cfg4-secosw-Tc", ds))
    ds = make_dataset(3, 256, 2, seed=6); ds.theta = make_walkers(ds, 4096, seed=6)
    cases.append(("np3-2inst", ds))
    for name, ds in cases:
        eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), len(ds.planet_letters),
                       ds.parameterisation, ds.t0, device=0)
        eng.reserve(len(ds.theta))
        if os.environ.get("KB_LPW"):
            eng.set_lanes_per_walker(int(os.environ["KB_LPW"]))
        th = torch.from_numpy(ds.theta).cuda(); out = torch.empty(len(ds.theta), dtype=torch.float64, device="cuda")
        row = {"case": name, "W": len(ds.theta), "N": len(ds.time), "NP": len(ds.planet_letters)}
        for solver in ((0, 1) if os.environ.get("KB_BOTH") else (0,)):
            eng.set_solver(solver)
            us = timeit(eng, th, out)
            solves = len(ds.theta) * len(ds.time) * len(ds.planet_letters)
            row[f"s{solver}_us"] = us
            row[f"s{solver}_solves_per_s"] = solves / (us * 1e-6)
        out_rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
