#!/bin/bash
# Build librvk_lltrace.so with -DRVK_LL_TRACE=1 on rvk.hip (reuses rvk_post.o, rvk_gp.o).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DRVK_LL_TRACE=1 -c -o build/variants/rvk_lltrace.o ravest_amd/csrc/rvk.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/librvk_lltrace.so build/variants/rvk_lltrace.o build/obj/rvk_post.o build/obj/rvk_gp.o build/obj/rvk_gp64.o
