#!/bin/bash
# A/B the variant builds (kbench + scaling per variant), then the default bench with 1 and 4 streams.
O=gpurun_out/${1:-ab}
mkdir -p $O
for rep in 1 2; do
for so in build/variants/librvk_*.so; do
  v=$(basename $so .so)
  RAVEST_AMD_LIB=$so timeout -k 10 200 python tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || echo "fail $v"
done
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_s1.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 > $O/bench_s4.json 2>&1 || exit 1
echo done
