#!/bin/bash
# Build a committed tree (git REV) as varlib/librvk_<name>.so, so a GPU run can A/B the working
# tree's library against it in one session (tools/ab.sh VARDIR=varlib; kbench / bench).
# Usage: tools/ab_rev.sh REV name
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
WT=$(mktemp -d /tmp/rvk_ab.XXXX)
git worktree add -q --detach "$WT" "$REV"
mkdir -p varlib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o varlib/librvk_$NAME.so \
  "$WT"/ravest_amd/csrc/rvk.hip "$WT"/ravest_amd/csrc/rvk_post.hip "$WT"/ravest_amd/csrc/rvk_gp.hip \
  "$WT"/ravest_amd/csrc/rvk_gp64.hip
git worktree remove --force "$WT"
ls -la varlib/librvk_$NAME.so
