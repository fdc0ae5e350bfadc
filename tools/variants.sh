#!/bin/bash
# Build A/B variants of librvk.so from the working tree with different -D knobs:
#   tools/variants.sh name1:"-DFOO=1" name2:"-DBAR=0" ...   -> build/variants/librvk_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
build() { name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
  -o build/variants/librvk_$name.so ravest_amd/csrc/rvk.hip ravest_amd/csrc/rvk_post.hip ravest_amd/csrc/rvk_gp.hip \
  ravest_amd/csrc/rvk_gp64.hip 2>/dev/null & }
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags
done
wait
ls build/variants
