#!/bin/bash
# Session check on a GPU box: GPU tests, smoke, bench, GP bench, rocprof kernel stats of both.
# Usage: bash profiles/session_scripts/gpu_check.sh TAG
TAG=${1:-r}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 120 python tools/gp_bench.py > $O/gp_bench.json 2> $O/gp_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/profgp -o run --output-format csv -- python tools/gp_bench.py > $O/profgp.log 2>&1 || exit 1
cat $O/bench.json $O/gp_bench.json
echo done
