#!/bin/bash
# Build the committed tree (git REV, default HEAD) as build/variants/librvk_<name>.so so a GPU run can
# A/B the working tree's librvk.so against it on the same box (tools/sampler_ab.sh, tools/ab.sh).
# Usage: tools/ab_head.sh [REV] [name]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-head}
WT=$(mktemp -d /tmp/rvk_ab.XXXX)
git worktree add -q --detach "$WT" "$REV"
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o build/variants/librvk_$NAME.so \
  "$WT"/ravest_amd/csrc/rvk.hip "$WT"/ravest_amd/csrc/rvk_post.hip "$WT"/ravest_amd/csrc/rvk_gp.hip \
  "$WT"/ravest_amd/csrc/rvk_gp64.hip
git worktree remove --force "$WT"
ls -la build/variants/librvk_$NAME.so
