#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the predictive kernel vs plain fills of the same block (tools/probe_write.py).
OUT=${1:-gpurun_out/pmc_write}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python tools/probe_write.py > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
meta = json.loads([l for l in open(out + "/p1.log") if l.startswith("{")][-1])
res = {"meta": meta, "kernels": {k: {c: sum(x) / len(x) for c, x in d.items()} for k, d in v.items()}}
json.dump(res, open(out + "/write_probe.json", "w"), indent=1)
for k, d in res["kernels"].items():
    print(k, {c: round(x) for c, x in d.items()})
PY
