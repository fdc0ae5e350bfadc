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
meta = json.loads([l for l in open(out + "/p1.log") if l.startswith("{")][-1])
res = {"meta": meta, "cases": []}
per = {}
for i, cnt in ((1, "WRITE_SIZE"), (2, "FETCH_SIZE")):
    rows = []
    for f in glob.glob(f"{out}/p{i}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == cnt]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    big = [r for r in rows if float(r["Counter_Value"]) > 1e5 or "predict" in r["Kernel_Name"] or "Fill" in r["Kernel_Name"]]
    big = [r for r in big if "predict" in r["Kernel_Name"] or "Fill" in r["Kernel_Name"]]
    per[cnt] = big
n = len(meta["cases"])
for k, (label, nbytes) in enumerate(meta["cases"]):
    d = {"case": label, "bytes": nbytes}
    for cnt, rows in per.items():
        sel = rows[3 * k: 3 * k + 3]
        if len(sel) == 3:
            d["kernel"] = sel[0]["Kernel_Name"][:80]
            d[cnt + "_KB"] = sum(float(r["Counter_Value"]) for r in sel) / 3
    if "WRITE_SIZE_KB" in d:
        d["write_ratio"] = d["WRITE_SIZE_KB"] * 1024 / nbytes
    res["cases"].append(d)
json.dump(res, open(out + "/write_probe.json", "w"), indent=1)
for d in res["cases"]:
    print(d["case"], round(d.get("write_ratio", -1), 3), d.get("kernel", "")[:50])
PY
