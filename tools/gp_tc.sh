#!/bin/bash
# GP two-column A/B: parity of the variant library, then config-5 timings base vs variants (alternating).
O=gpurun_out/${1:-gptc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py tests/test_gpu_gp64.py -x -q --timeout 120 --timeout-method thread > $O/pytest_base.log 2>&1 || { tail -40 $O/pytest_base.log; exit 1; }
echo "base: $(tail -1 $O/pytest_base.log)"
for so in build/variants/librvk_*.so; do
  v=$(basename $so .so)
  RAVEST_AMD_LIB=$so timeout -k 10 200 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
  timeout -k 10 100 python tools/gp_bench.py 4096 512 fp32 > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
  echo "base $(cut -c1-220 $O/base_$rep.json)"
  for so in build/variants/librvk_*.so; do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 100 python tools/gp_bench.py 4096 512 fp32 > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$v $(cut -c1-220 $O/${v}_$rep.json)"
  done
done
echo done
