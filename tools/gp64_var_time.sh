#!/bin/bash
# Timing-only fp64 config-5 A/B of prebuilt variant libraries (varlib/librvk_<name>.so), base and variants
# interleaved, 3 reps.  Only for variants whose config-5 shape already passed its parity tests.
O=gpurun_out/${1:-g64t}; shift
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
  echo "base $(cut -c1-300 $O/base_$rep.json)"
  for v in "$@"; do
    RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/${v}_$rep.json 2>/dev/null || { echo "fail $v"; exit 1; }
    echo "$v $(cut -c1-300 $O/${v}_$rep.json)"
  done
  if [ -n "$GP32_NW8" ]; then   # the fp32 kernel's 8-wave x 2-row shape against its 4-wave default
    timeout -k 10 120 python tools/gp_bench.py 4096 512 > $O/f32_$rep.json 2>/dev/null || { echo "fail f32"; exit 1; }
    echo "f32 $(cut -c1-200 $O/f32_$rep.json)"
    RVK_GP_NW=8 timeout -k 10 120 python tools/gp_bench.py 4096 512 > $O/f32nw8_$rep.json 2>/dev/null || { echo "fail f32nw8"; exit 1; }
    echo "f32nw8 $(cut -c1-200 $O/f32nw8_$rep.json)"
  fi
done
echo done
