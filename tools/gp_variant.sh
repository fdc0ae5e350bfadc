#!/bin/bash
# Build librvk_<name>.so with extra -D flags on rvk_gp.hip only (reuses the built rvk.o, rvk_post.o).
# usage: tools/gp_variant.sh name -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c -o build/variants/rvk_gp_$name.o ravest_amd/csrc/rvk_gp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/librvk_$name.so build/obj/rvk.o build/obj/rvk_post.o build/obj/rvk_gp64.o build/variants/rvk_gp_$name.o
