#!/bin/bash
# fp64 GP at n = 700 and 1024 (the 5-row shapes): the in-tree library against varlib/librvk_<name>.so,
# GP parity tests on the variant first, then 3 interleaved reps.  usage: bash tools/gp64_shape_ab.sh TAG name
O=gpurun_out/${1:-g64shape}; v=$2
mkdir -p $O
export TMPDIR=/tmp
RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
echo "$v: $(tail -1 $O/pytest_$v.log)"
for n in 700 1024; do
  for rep in 1 2 3; do
    timeout -k 10 120 python tools/gp_bench.py 4096 $n fp64 > $O/base_${n}_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
    RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 120 python tools/gp_bench.py 4096 $n fp64 > $O/${v}_${n}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "n=$n base $(python -c "import json;print(json.load(open('$O/base_${n}_$rep.json'))['ms_per_eval'])") $v $(python -c "import json;print(json.load(open('$O/${v}_${n}_$rep.json'))['ms_per_eval'])")"
  done
done
