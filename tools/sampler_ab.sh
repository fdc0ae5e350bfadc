#!/bin/bash
# Fused half-step A/B: sampler_variants on the in-tree library and varlib/librvk_*.so (REPS interleaved),
# then the phase trace of every varlib/trace/librvk_lltrace*.so.   bash tools/sampler_ab.sh TAG [REPS] [posteriors]
TAG=${1:?tag}; REPS=${2:-3}; shift 2; POST=${@:-uniform beta vaneylen}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python tools/sampler_variants.py $POST > $O/sv_main_$rep.log 2>&1 || { tail -20 $O/sv_main_$rep.log; exit 1; }
  for so in $(ls varlib/librvk_*.so 2>/dev/null); do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 200 python tools/sampler_variants.py $POST > $O/sv_${v}_$rep.log 2>&1 || { tail -20 $O/sv_${v}_$rep.log; exit 1; }
  done
done
for so in $(ls varlib/trace/librvk_lltrace*.so 2>/dev/null); do
  v=$(basename $so .so)
  RAVEST_AMD_LIB=$so timeout -k 10 120 python tools/sampler_trace.py > $O/trace_$v.txt 2>&1 || { tail -20 $O/trace_$v.txt; exit 1; }
done
python - $O <<'PY'
import json, glob, sys, collections
o = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(o + "/sv_*_*.log")):
    lib = f.split("/sv_")[1].rsplit("_", 1)[0]
    for line in open(f):
        try:
            d = json.loads(line)
        except Exception:
            continue
        for k, v in d.items():
            res[k][lib].append(round(v["ms_per_step"] * 1e3, 2))
for k, libs in res.items():
    print(k, dict(libs))
PY
echo "sampler_ab: done"
