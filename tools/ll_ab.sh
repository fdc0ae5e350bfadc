#!/bin/bash
# Likelihood-kernel change: parity + layout GPU tests on the in-tree library, kbench A/B against
# varlib/librvk_*.so (interleaved), and one PMC pass of the config-2 VALU counters per library.
#   bash tools/ll_ab.sh TAG [REPS]
TAG=${1:?tag}; REPS=${2:-3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_lds_poison.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
VARS=$(ls varlib/librvk_*.so 2>/dev/null)
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python tools/kbench.py > $O/kb_main_$rep.log 2>&1 || { tail -20 $O/kb_main_$rep.log; exit 1; }
  for so in $VARS; do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 200 python tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || { tail -20 $O/kb_${v}_$rep.log; exit 1; }
  done
done
python - $O <<'PY'
import json, glob, sys, collections
o = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(o + "/kb_*_*.log")):
    lib = f.split("/kb_")[1].rsplit("_", 1)[0]
    for line in open(f):
        d = json.loads(line)
        if "case" in d:
            res[d["case"]][lib].append(round(d["s0_us"], 3))
for case, libs in res.items():
    print(case, {k: v for k, v in libs.items()})
PY
CMD="python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline --no-sampler --no-gp --no-predictive --no-configs --no-host-path"
for lib in main $VARS; do
  n=$(basename $lib .so)
  if [ $lib = main ]; then unset RAVEST_AMD_LIB; else export RAVEST_AMD_LIB=$lib; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc_$n -o run -- $CMD > $O/pmc_$n.log 2>&1 || { tail -5 $O/pmc_$n.log; exit 1; }
  python - $O/pmc_$n <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "loglike_kernel<1, false, 0, true, 0, 1024>" not in k: continue
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
vals = collections.defaultdict(list)
for d, c in agg.items():
    for n, v in c.items(): vals[n].append(v)
print(sys.argv[1], {n: sum(v) / len(v) for n, v in vals.items()}, "dispatches", len(agg))
PY
  rm -rf $O/pmc_$n
done
unset RAVEST_AMD_LIB
echo "ll_ab: done"
