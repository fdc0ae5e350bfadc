#!/bin/bash
# config-2 kernel A/B vs the round-2 / round-3 final libraries (kbench, 3 interleaved reps) and the
# predictive WRITE_SIZE calibration probe.
TAG=${1:-r4e}
export TMPDIR=/tmp
O=gpurun_out/${TAG}_kb
mkdir -p $O
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/ab/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=librvk_main
    RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -5 $O/kb_${v}_$rep.log; }
  done
done
python tools/ab_summary.py $O || ls $O
bash tools/pmc_write_probe.sh gpurun_out/${TAG}_wp || exit 1
echo done
