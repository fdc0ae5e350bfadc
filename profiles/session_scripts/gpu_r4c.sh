#!/bin/bash
# Round-4 session, part B: config-2 kernel A/B of the round-2 / round-3 final libraries against the
# working tree (kbench, 3 interleaved reps), the fp32 GP variants, and the predictive WRITE_SIZE probe.
TAG=${1:-r4c}
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
SKIPTEST=1 VARDIR=varlib/f32 bash tools/gp64_ab.sh ${TAG}_gp32 fp32+fp64 || exit 1
bash tools/pmc_write_probe.sh gpurun_out/${TAG}_wp || exit 1
echo done
