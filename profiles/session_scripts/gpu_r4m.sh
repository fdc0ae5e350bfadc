#!/bin/bash
TAG=${1:-r4m}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
REPS=3 SKIPTEST=1 bash tools/gp64_ab.sh ${TAG}_g64 fp64 || exit 1
SKIPTEST=1 VARDIR=varlib/f32 bash tools/gp64_ab.sh ${TAG}_g32 fp32+fp64 || exit 1
