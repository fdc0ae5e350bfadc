#!/bin/bash
# Full GPU suite + kernel timings (kbench x3, gp_bench fp64 / fp32+fp64) on the working tree.
TAG=${1:-r4h}
O=gpurun_out/$TAG; mkdir -p $O/kb
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do timeout -k 10 200 python tools/kbench.py > $O/kb/kb_librvk_main_$rep.log 2>&1 || exit 1; done
python tools/ab_summary.py $O/kb
timeout -k 10 300 python tools/gp_bench.py 4096 512 fp64 > $O/gp64.json 2>&1 && timeout -k 10 300 python tools/gp_bench.py 4096 512 fp32+fp64 > $O/gp32.json 2>&1 || exit 1
tail -1 $O/gp64.json | cut -c1-200; tail -1 $O/gp32.json | cut -c1-200
SKIPTEST=1 bash tools/gp64_ab.sh ${TAG}_abl fp64 || exit 1
