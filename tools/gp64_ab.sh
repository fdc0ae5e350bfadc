#!/bin/bash
# fp64 GP kernel A/B: GP parity tests on the built library, then config-5 fp64 timings base vs variants.
O=gpurun_out/${1:-g64ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_posterior.py -x -q --timeout 120 --timeout-method thread > $O/pytest_base.log 2>&1 || { tail -40 $O/pytest_base.log; exit 1; }
echo "base: $(tail -1 $O/pytest_base.log)"
for rep in 1 2; do
  timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
  echo "base $(cut -c1-400 $O/base_$rep.json)"
  for so in build/variants/librvk_*.so; do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$v $(cut -c1-400 $O/${v}_$rep.json)"
  done
done
echo done
