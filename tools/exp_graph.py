"""Experiment: can timing events be captured inside a HIP graph with our C-ABI launches?"""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_config
ds = make_config(2)
eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0, device=0)
th = torch.from_numpy(ds.theta).cuda()
G = 50
outs = [torch.empty(len(ds.theta), dtype=torch.float64, device="cuda") for _ in range(G)]
ref = eng.loglike(ds.theta)
res = {}
# eager, events per launch
s = torch.cuda.current_stream()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
for j in range(G):
    evs[j][0].record(s); eng.loglike_device(th, outs[j], s); evs[j][1].record(s)
torch.cuda.synchronize()
res["eager_event_ms"] = float(np.mean([a.elapsed_time(b) for a, b in evs]))
t0 = time.perf_counter()
for j in range(G):
    eng.loglike_device(th, outs[j], s)
torch.cuda.synchronize(); res["eager_wall_ms_per_step"] = (time.perf_counter() - t0) / G * 1e3
# graph, single stream
g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
with torch.cuda.graph(g, stream=cs):
    for j in range(G):
        eng.loglike_device(th, outs[j])
g.replay(); torch.cuda.synchronize()
res["graph_ok"] = bool(np.array_equal(outs[G - 1].cpu().numpy(), ref))
t0 = time.perf_counter()
for r in range(20):
    g.replay()
torch.cuda.synchronize(); res["graph1_wall_ms_per_step"] = (time.perf_counter() - t0) / (20 * G) * 1e3
# graph with events inside
try:
    g2 = torch.cuda.CUDAGraph()
    evg = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
    with torch.cuda.graph(g2, stream=cs):
        for j in range(G):
            evg[j][0].record(); eng.loglike_device(th, outs[j]); evg[j][1].record()
    g2.replay(); torch.cuda.synchronize()
    res["graph_events_ms"] = float(np.mean([a.elapsed_time(b) for a, b in evg]))
except Exception as ex:
    res["graph_events_err"] = repr(ex)[:300]
# graph with S parallel streams (independent batches)
for S in (2, 4):
    g3 = torch.cuda.CUDAGraph()
    side = [torch.cuda.Stream() for _ in range(S)]
    with torch.cuda.graph(g3, stream=cs):
        for st in side:
            st.wait_stream(cs)
        for j in range(G):
            with torch.cuda.stream(side[j % S]):
                eng.loglike_device(th, outs[j])
        for st in side:
            cs.wait_stream(st)
    g3.replay(); torch.cuda.synchronize()
    ok = all(np.array_equal(o.cpu().numpy(), ref) for o in outs)
    t0 = time.perf_counter()
    for r in range(20):
        g3.replay()
    torch.cuda.synchronize(); res[f"graph{S}s_wall_ms_per_step"] = (time.perf_counter() - t0) / (20 * G) * 1e3
    res[f"graph{S}s_ok"] = ok
# host path (PCIe-inclusive, blocking)
t0 = time.perf_counter()
for r in range(50):
    eng.loglike(ds.theta)
res["host_path_ms_per_call"] = (time.perf_counter() - t0) / 50 * 1e3
print(json.dumps(res))
