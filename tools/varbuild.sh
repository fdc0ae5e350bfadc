#!/bin/bash
# Build A/B variants of librvk.so into varlib/ (travels to the GPU box; git-ignored):
#   TUS="rvk" VAROUT=varlib/x tools/varbuild.sh name1:"-DFOO=1" name2:"..."  -> $VAROUT/librvk_<name>.so
# The translation units in TUS (default: all four) are rebuilt with the flags (objects under
# build/var/<name>/); the others are linked from the in-tree build (build/obj, make first).
# Variants build in parallel.
set -e
cd "$(dirname "$0")/.."
OUT=${VAROUT:-varlib}
mkdir -p $OUT
ALL="rvk rvk_sample rvk_sample1 rvk_post rvk_gp rvk_gp64"
TUS=${TUS:-$ALL}
for t in $TUS; do [[ " $ALL " == *" $t "* ]] || ALL="$ALL $t"; done   # a unit only the variant has
one() {
  local name=$1 flags=$2 o=build/var/$1 objs=""
  mkdir -p $o
  for s in $ALL; do
    if [[ " $TUS " == *" $s "* ]]; then
      local tuf=""
      if [[ "$flags" != *sched-strategy* ]]; then   # as the Makefile
        [ $s = rvk_sample ] && tuf="-mllvm -amdgpu-sched-strategy=iterative-ilp"
        [ $s = rvk_sample1 ] && tuf="-mllvm -amdgpu-sched-strategy=max-ilp"
      fi
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result $tuf $flags -c \
        -o $o/$s.o ravest_amd/csrc/$s.hip -Rpass-analysis=kernel-resource-usage 2> $o/$s.res &
      objs="$objs $o/$s.o"
    else
      objs="$objs build/obj/$s.o"
    fi
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/librvk_$name.so $objs
  cat $o/*.res > $o/resource.txt 2>/dev/null || true
  echo "built $OUT/librvk_$name.so"
}
for spec in "$@"; do
  one "${spec%%:*}" "${spec#*:}" &
done
wait
