#!/bin/bash
# Round-4 session: the r4a checks, the fp64 GP A/B, and a config-2 kernel A/B of round 2 / round 3
# final libraries against the working tree (kbench, 3 interleaved reps).  Usage: tools/gpu_r4b.sh TAG
TAG=${1:-r4b}
bash tools/gpu_r4.sh $TAG || exit 1
bash tools/gp64_ab.sh ${TAG}_gp || exit 1
SKIPTEST=1 VARDIR=varlib/f32 bash tools/gp64_ab.sh ${TAG}_gp32 fp32+fp64 || exit 1
O=gpurun_out/${TAG}_kb
mkdir -p $O
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/ab/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=librvk_main
    RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -5 $O/kb_${v}_$rep.log; }
  done
done
python tools/ab_summary.py $O 2>/dev/null || ls $O
echo done
