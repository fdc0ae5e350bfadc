#!/bin/bash
# A/B the variant builds in build/variants (tools/variants.sh): kbench (graph-replay us per launch)
# per variant, interleaved over 3 repetitions in one session.
O=gpurun_out/${1:-ab}
mkdir -p $O
for rep in 1 2 3; do
for so in ${VARDIR:-build/variants}/librvk_*.so; do
  v=$(basename $so .so)
  RAVEST_AMD_LIB=$so timeout -k 10 200 python tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || echo "fail $v"
done
done
echo done
