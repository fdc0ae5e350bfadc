#!/bin/bash
# fp64 GP A/B of prebuilt variant libraries (varlib/librvk_<name>.so): the GP parity tests on each variant,
# then config-5 fp64 timings, base and variants interleaved.  usage: bash tools/gp64_var_ab.sh TAG name...
O=gpurun_out/${1:-g64v}; shift
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
  timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
  echo "base $(cut -c1-300 $O/base_$rep.json)"
  for v in "$@"; do
    RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$v $(cut -c1-300 $O/${v}_$rep.json)"
  done
done
echo done
