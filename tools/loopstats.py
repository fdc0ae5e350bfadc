"""Per-basic-block VALU/SALU/memory instruction counts of one kernel in device assembly.

usage: python tools/loopstats.py <file.s> <mangled-name-substring>
(make the .s with: hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o rvk.s csrc/rvk.hip)
"""
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l and l.rstrip().endswith(key.split()[-1] + ":") or
             (l.startswith("_Z") and key in l and ": ;" in l))
stats, bb, tot = [], None, {"v": 0, "f64": 0, "f32": 0, "tr": 0, "mov": 0, "s": 0}
for l in lines[start + 1:]:
    s = l.strip()
    if s.startswith("s_endpgm"):
        break
    if re.match(r"^\.LBB\S+:", s) or re.match(r"^; %bb\.\d+:", s):
        bb = {"name": s.split(":")[0].replace("; ", ""), "v": 0, "f64": 0, "f32": 0, "tr": 0, "mov": 0, "s": 0, "mem": 0, "br": "",
              "comm": l[l.find(";"):] if ";" in l else ""}
        stats.append(bb)
        continue
    if bb is None:
        bb = {"name": "entry", "v": 0, "f64": 0, "f32": 0, "tr": 0, "mov": 0, "s": 0, "mem": 0, "br": "", "comm": ""}
        stats.append(bb)
    if not s or s.startswith(";") or s.startswith("."):
        continue
    op = s.split()[0]
    if op.startswith("v_"):
        bb["v"] += 1
        if "f64" in op:
            bb["f64"] += 1
        elif "f32" in op:
            bb["f32"] += 1
        if re.match(r"v_(sin|cos|rcp|rsq|sqrt|log|exp)_", op):
            bb["tr"] += 1
        if op.startswith("v_mov"):
            bb["mov"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        bb["br"] += op.replace("s_cbranch_", "") + " " + s.split()[-1] + "; "
    elif op.startswith("s_"):
        bb["s"] += 1
    if op.startswith(("global_", "ds_", "buffer_", "scratch_", "flat_", "s_load")):
        bb["mem"] += 1
for b in stats:
    print(f"{b['name']:12s} v={b['v']:4d} f64={b['f64']:3d} f32={b['f32']:3d} tr={b['tr']:2d} mov={b['mov']:2d} "
          f"s={b['s']:3d} mem={b['mem']:2d} {b['br'][:48]:48s} {b['comm'][:44]}")
