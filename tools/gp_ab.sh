#!/bin/bash
# GP kernel: parity tests once, then config-5 timings under the launch-shape experiment hooks.
O=gpurun_out/${1:-gpab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gp.log 2>&1 || { tail -40 $O/pytest_gp.log; exit 1; }
tail -1 $O/pytest_gp.log
for cfg in "4 2" "8 1" "8 2"; do
  set -- $cfg
  RVK_GP_NW=$1 RVK_GP_WGPCU=$2 timeout -k 10 100 python tools/gp_bench.py > $O/nw$1_wg$2.json 2>&1 || { echo "fail $cfg"; exit 1; }
  echo "nw=$1 wgpcu=$2 $(cat $O/nw$1_wg$2.json)"
done
