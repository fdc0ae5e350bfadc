#!/bin/bash
# Build A/B variants of librvk.so from the same source (different -D knobs).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
build() { name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
  -o build/variants/librvk_$name.so ravest_amd/csrc/rvk.hip 2>/dev/null & }
build base
build oldseed -DRVK_SEED_START=0 -DRVK_SEED_THR=2e-5f
build thr1e3 -DRVK_SEED_THR=1e-3f
build start0 -DRVK_SEED_START=0
wait
ls build/variants
