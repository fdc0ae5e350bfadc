"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage output (VGPRs, scratch, occupancy per kernel).

usage: python tools/resources.py [build/rvk_resource.txt] [filter-substring]
"""
import re
import subprocess
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "build/rvk_resource.txt"
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows, cur = [], None
for line in open(path):
    m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\S+) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = n.replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    if filt in n:
        print(f"{n:55s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} sgpr {r.get('SGPRs', '?'):>3s} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} occ {r.get('Occupancy [waves/SIMD]', '?')}")
