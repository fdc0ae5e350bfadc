import glob, json, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/kb_*.log")):
    v = f.split("kb_librvk_")[1].rsplit("_", 1)[0]
    for l in open(f):
        if l.startswith("{") and '"case"' in l:
            r = json.loads(l); d[r["case"]][v].append(r["s0_us"])
for case, vs in d.items():
    print(case.ljust(16), "  ".join(f"{v}:{min(x):.1f}" for v, x in sorted(vs.items())))
