"""Summarise rocprofv3 --pmc passes for the dominant loglike kernel into pmc_<label>.json (copy to profiles/).

Per-launch values = the counter summed over the kernel's dispatches / number of dispatches.
gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) reads 1/2 of the bytes of a wide
coalesced stream -> doubled; WRITE_SIZE (KB) is read as-is.
"""
import csv, glob, json, os, sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest   # noqa: E402  (the provenance stamp bench.py checks)

out_dir, cfg = sys.argv[1], sys.argv[2]
label = f"config{cfg}" if cfg.isdigit() else cfg          # profiles/pmc_<label>.json
kfilter = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] else None   # kernel-name substring (default: the plain loglike launch)
cmd = sys.argv[4] if len(sys.argv) > 4 else None         # the profiled command, for the record

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
src = (f"rocprofv3 --pmc passes over `{cmd}`" if cmd else
       f"rocprofv3 --pmc passes over `python tools/gp_bench.py` (tools/pmc_gp.sh)" if kfilter else
       f"rocprofv3 --pmc passes over `python bench.py --config {cfg} --steps 20 --warmup 5 --no-cpu-baseline --no-sampler` (tools/pmc.sh)")
res = {"kernel": kname, "counters_per_launch": per, "source": src, "csrc_sha256": csrc_digest()}
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    # L2 memory-side (fabric) bytes: counts Infinity-Cache hits, so an upper bound on HBM bytes
    res["fabric_bytes_per_launch"] = (2 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
if "SQ_INSTS_VALU" in per:
    res["valu_insts_per_launch"] = per["SQ_INSTS_VALU"]

p = os.path.join(out_dir, f"pmc_{label}.json")
json.dump(res, open(p, "w"), indent=1)
print(json.dumps(res, indent=1))
