#!/bin/bash
# Build a traced librvk (RVK_GP_TRACE=1) from the built objects + a traced rvk_gp.o (run here, on the CPU).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DRVK_GP_TRACE=1 $@ -c -o build/variants/rvk_gp_trace.o ravest_amd/csrc/rvk_gp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/librvk_trace.so build/obj/rvk.o build/obj/rvk_post.o build/variants/rvk_gp_trace.o build/obj/rvk_gp64.o
