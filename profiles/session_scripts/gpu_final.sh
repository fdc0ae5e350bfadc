#!/bin/bash
# Round-end evidence on one fresh box: GPU tests, smoke, bench, rocprof kernel stats of the bench
# command, then PMC passes over config 5 (GP).  Each GPU step has its own limit; the first failure ends it.
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
timeout -k 10 600 bash tools/pmc_gp.sh $O/pmc_gp > $O/pmc_config5.json 2> $O/pmc_gp.err || { tail -20 $O/pmc_gp.err; exit 1; }
echo done
