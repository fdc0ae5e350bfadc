#!/bin/bash
# Parity of the GP fp64 and likelihood kernels, then GP fp64 variant A/B (3 reps) and kbench (3 reps).
TAG=${1:-r4j}
O=gpurun_out/$TAG; mkdir -p $O/kb
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_parity.py tests/test_gpu_layout.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
REPS=3 SKIPTEST=1 bash tools/gp64_ab.sh ${TAG}_g64 fp64 || exit 1
for rep in 1 2 3; do timeout -k 10 200 python tools/kbench.py > $O/kb/kb_librvk_main_$rep.log 2>&1 || exit 1; done
python tools/ab_summary.py $O/kb
