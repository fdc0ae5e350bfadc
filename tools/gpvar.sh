#!/bin/bash
# A/B variants of librvk.so that differ only in one translation unit (default rvk_gp64.hip):
#   tools/gpvar.sh [-u rvk_gp.hip] name1:"-DFOO=1" name2:"-DBAR=0" ...  -> varlib/librvk_<name>.so
# The other objects come from the in-tree build (build/obj, `make -C ravest_amd` first).
set -e
cd "$(dirname "$0")/.."
TU=rvk_gp64.hip
if [ "$1" = "-u" ]; then TU=$2; shift 2; fi
OUT=${VAROUT:-varlib}
mkdir -p $OUT build/varobj
OTHERS=$(ls build/obj/*.o | grep -v "/${TU%.hip}.o$")
one() {
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c \
    -o build/varobj/${TU%.hip}_$name.o ravest_amd/csrc/$TU -Rpass-analysis=kernel-resource-usage 2> build/varobj/$name.res
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/librvk_$name.so build/varobj/${TU%.hip}_$name.o $OTHERS
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  one $name $flags &
done
wait
ls -la $OUT
