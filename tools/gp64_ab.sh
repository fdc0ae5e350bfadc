#!/bin/bash
# fp64 GP kernel A/B: GP parity tests on the in-tree library, then config-5 fp64 timings of the
# in-tree library ("main") against every varlib/librvk_*.so, interleaved.  Usage: tools/gp64_ab.sh TAG [prec]
O=gpurun_out/${1:-g64ab}
PREC=${2:-fp64}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIPTEST" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gp.log 2>&1 || { tail -40 $O/pytest_gp.log; exit 1; }
echo "gp tests: $(tail -1 $O/pytest_gp.log)"
fi
for rep in $(seq 1 ${REPS:-2}); do
  timeout -k 10 120 python tools/gp_bench.py 4096 512 $PREC > $O/main_$rep.json 2>/dev/null || { echo "fail main"; exit 1; }
  echo "main $(cut -c1-300 $O/main_$rep.json)"
  for so in ${VARDIR:-varlib}/librvk_*.so; do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 120 python tools/gp_bench.py 4096 512 $PREC > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$v $(cut -c1-300 $O/${v}_$rep.json)"
  done
done
echo done
