#!/bin/bash
# config 5 fp64 GP (n = 512) plus n = 700: the in-tree library against varlib/librvk_<name>.so variants,
# GP parity tests on each variant first, then 3 interleaved reps.  usage: bash tools/gp64_n512_ab.sh TAG names...
O=gpurun_out/${1:-g64n}; shift
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
ms() { python -c "import json;print(round(json.load(open('$1'))['ms_per_eval'],3))"; }
for n in ${NS:-512 700}; do
  for rep in 1 2 3; do
    timeout -k 10 120 python tools/gp_bench.py 4096 $n fp64 > $O/base_${n}_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
    line="n=$n base $(ms $O/base_${n}_$rep.json)"
    for v in "$@"; do
      RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 120 python tools/gp_bench.py 4096 $n fp64 > $O/${v}_${n}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
      line="$line $v $(ms $O/${v}_${n}_$rep.json)"
    done
    echo "$line"
  done
done
