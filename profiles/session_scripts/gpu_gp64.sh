#!/bin/bash
# GPU session: GP tests (fp32 + fp64 + posterior + predictive), then config-5 timing per precision
# and a rocprof kernel-stats pass.  Every GPU step has its own time limit; the first failure ends it.
# Usage: bash profiles/session_scripts/gpu_gp64.sh TAG
TAG=${1:-gp64}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py -x -v --timeout 120 --timeout-method thread > $O/pytest_gp.log 2>&1 \
  || { echo "pytest failed"; tail -60 $O/pytest_gp.log; exit 1; }
tail -3 $O/pytest_gp.log
for P in fp32+fp64 fp64; do
  timeout -k 10 180 python tools/gp_bench.py 4096 512 $P > $O/gp_bench_$P.json 2>&1 || { cat $O/gp_bench_$P.json; exit 1; }
  cat $O/gp_bench_$P.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/gp_bench.py 4096 512 fp64 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
