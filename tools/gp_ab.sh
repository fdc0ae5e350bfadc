#!/bin/bash
# GP kernel: parity tests once, then config-5 timings: base, variants in build/variants, env shapes.
O=gpurun_out/${1:-gpab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gp.log 2>&1 || { tail -40 $O/pytest_gp.log; exit 1; }
tail -1 $O/pytest_gp.log
for rep in 1 2; do
timeout -k 10 100 python tools/gp_bench.py > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
echo "base $(cut -c80-150 $O/base_$rep.json)"
for so in build/variants/librvk_*.so; do
  v=$(basename $so .so)
  case $v in *trace*) continue;; esac
  RAVEST_AMD_LIB=$so timeout -k 10 100 python tools/gp_bench.py > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
  echo "$v $(cut -c80-150 $O/${v}_$rep.json)"
done
done
if [ -f build/variants/librvk_trace.so ]; then
  RAVEST_AMD_LIB=build/variants/librvk_trace.so timeout -k 10 100 python tools/gp_trace.py > $O/trace.txt 2>&1
  RVK_GP_WGPCU=1 RAVEST_AMD_LIB=build/variants/librvk_trace.so timeout -k 10 100 python tools/gp_trace.py > $O/trace_wg1.txt 2>&1
fi
echo done
