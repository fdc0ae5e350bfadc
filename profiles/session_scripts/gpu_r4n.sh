#!/bin/bash
# kbench A/B of the likelihood variants in varlib/ll (3 interleaved reps)
O=gpurun_out/r4n; mkdir -p $O/kb
export TMPDIR=/tmp
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/ll/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=librvk_main
    RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/kbench.py > $O/kb/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $O/kb/kb_${v}_$rep.log; exit 1; }
  done
done
python tools/ab_summary.py $O/kb
RAVEST_AMD_LIB=$(realpath varlib/trace/librvk_lltrace.so) timeout -k 10 120 python tools/sampler_trace.py 4096 > $O/sampler_trace.txt 2>&1 || { tail -5 $O/sampler_trace.txt; exit 1; }
RAVEST_AMD_LIB=$(realpath varlib/trace/librvk_lltrace.so) timeout -k 10 120 python tools/ll_trace.py 4096 > $O/ll_trace.txt 2>&1 || { tail -5 $O/ll_trace.txt; exit 1; }
cat $O/sampler_trace.txt $O/ll_trace.txt
