#!/bin/bash
# GP fp64 parity + A/B of the fp64 kernel variants (varlib/) and a likelihood kbench A/B (varlib/ll/).
TAG=${1:-r4i}
O=gpurun_out/$TAG; mkdir -p $O/kb
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_hostpath.py tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
SKIPTEST=1 bash tools/gp64_ab.sh ${TAG}_g64 fp64 || exit 1
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/ll/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=librvk_main
    RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/kbench.py > $O/kb/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; exit 1; }
  done
done
python tools/ab_summary.py $O/kb
