"""Summarise rocprofv3 --pmc passes for the dominant loglike kernel into profiles/pmc_config<c>.json.

Per-launch values = the counter summed over the kernel's dispatches / number of dispatches.
gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) reads 1/2 of the bytes of a wide
coalesced stream -> doubled; WRITE_SIZE (KB) is read as-is.
"""
import csv, glob, json, os, sys
from collections import defaultdict

out_dir, cfg = sys.argv[1], sys.argv[2]
kfilter = sys.argv[3] if len(sys.argv) > 3 else None   # kernel-name substring (default: the plain loglike launch)

def plain_loglike(name):
    """loglike_kernel<NP, MULTI, SOLVER, TP, SAMPLE[, BLK]> with SAMPLE = 0 (not the sampler's), or
    the segmented loglike_seg_kernel the launcher picks for W >= 8192 (configs 3 and 4)."""
    if "loglike_seg_kernel<" in name:
        return True
    if "loglike_kernel<" not in name:
        return False
    args = name.split("loglike_kernel<", 1)[1].split(">(", 1)[0].split(", ")
    return len(args) >= 5 and args[4] in ("false", "0")


vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(os.path.join(out_dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if kfilter is not None:
            if kfilter not in name:
                continue
        elif not plain_loglike(name):
            continue
        c = row["Counter_Name"]
        vals[name][c] += float(row["Counter_Value"])
        disp[name][c].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
# the measured kernel: the matching instantiation with the most dispatches
kname = max(disp, key=lambda k: max(len(v) for v in disp[k].values())) if disp else None
per = {c: vals[kname][c] / max(1, len(disp[kname][c])) for c in vals[kname]} if kname else {}
src = (f"rocprofv3 --pmc passes over `python tools/gp_bench.py` (tools/pmc_gp.sh)" if kfilter else
       f"rocprofv3 --pmc passes over `python bench.py --config {cfg} --steps 20 --warmup 5 --no-cpu-baseline --no-sampler` (tools/pmc.sh)")
res = {"kernel": kname, "counters_per_launch": per, "source": src}
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    res["hbm_bytes_per_launch"] = (2 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
if "SQ_INSTS_VALU" in per:
    res["valu_insts_per_launch"] = per["SQ_INSTS_VALU"]

p = os.path.join(out_dir, f"pmc_config{cfg}.json")
json.dump(res, open(p, "w"), indent=1)
print(json.dumps(res, indent=1))
