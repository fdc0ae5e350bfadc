"""One-screen summary of a bench.py JSON line (the headline, the kernel, the rooflines, the
sub-lines' times).  usage: python tools/bench_summary.py bench.json"""
import json
import sys


def main(path):
    lines = [l for l in open(path) if l.lstrip().startswith("{")]
    d = json.loads(lines[-1])
    us = lambda ms: None if ms is None else round(ms * 1e3, 3)
    print(f"value {d['value']:.4e} {d['unit']}  step {us(d['ms_per_step'])} us  kernel {us(d.get('kernel_ms'))} us  "
          f"host call {us(d.get('host_path_ms_per_call'))} us")
    r = d.get("roofline", {})
    print("roofline", {k: r.get(k) for k in ("bound", "achieved", "peak", "frac", "traffic")})
    s = d.get("sampler", {})
    print("sampler", {k: v for k, v in s.items() if isinstance(v, (int, float)) and "ms" in k})
    g = d.get("gp_config5", {})
    if g:
        print("gp fp32+fp64", g.get("ms_per_eval"), "fp64", g.get("fp64", {}).get("ms_per_eval"))
    hp = d.get("host_path", {})
    if hp:
        print("host_path", {k: v for k, v in hp.items() if isinstance(v, (int, float))})
        for t, v in (hp.get("per_transport") or {}).items():
            print("  ", t, v)
    for k in ("config3", "config4_shard", "config4_sharded", "predictive"):
        v = d.get(k)
        if isinstance(v, dict):
            print(k, {a: b for a, b in v.items() if isinstance(b, (int, float)) and ("ms" in a or "per_s" in a)})


if __name__ == "__main__":
    main(sys.argv[1])
