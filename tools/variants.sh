#!/bin/bash
# Build A/B variants of librvk.so from the same source (different -D knobs).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
build() { name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
  -o build/variants/librvk_$name.so ravest_amd/csrc/rvk.hip 2>/dev/null & }
build base
build abl1 -DRVK_ABLATE=1
build abl2 -DRVK_ABLATE=2
build abl3 -DRVK_ABLATE=3
wait
ls build/variants
