#!/bin/bash
# One GPU-box session (round 2): GPU tests, smoke, bench, lanes-per-walker A/B, rocprof stats.
# Every GPU step has its own time limit; the first failure ends the script.
# Usage: bash profiles/session_scripts/gpu_r2.sh TAG [quick]
TAG=${1:-r2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
[ "$2" = "quick" ] && { echo done; exit 0; }
for L in 64 32; do
  KB_LPW=$L timeout -k 10 180 python tools/kbench.py > $O/kbench_lpw$L.json 2>&1 || { cat $O/kbench_lpw$L.json; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
