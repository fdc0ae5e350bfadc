#!/bin/bash
# Build librvk_gp64trace.so with -DRVK_GP64_TRACE=1 on rvk_gp64.hip (reuses the other objects).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DRVK_GP64_TRACE=1 -c -o build/variants/rvk_gp64trace.o ravest_amd/csrc/rvk_gp64.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/librvk_gp64trace.so build/obj/rvk.o build/obj/rvk_post.o build/obj/rvk_gp.o build/variants/rvk_gp64trace.o
