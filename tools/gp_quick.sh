#!/bin/bash
# GP kernel check: parity tests, then config-5 timing (tools/gp_bench.py).
O=gpurun_out/${1:-gpq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gp.log 2>&1 || { tail -40 $O/pytest_gp.log; exit 1; }
tail -2 $O/pytest_gp.log
timeout -k 10 120 python tools/gp_bench.py > $O/gp_bench.json 2> $O/gp_bench.err || { tail $O/gp_bench.err; exit 1; }
cat $O/gp_bench.json
