#!/bin/bash
# Build a committed tree (git REV) as varlib/librvk_<name>.so, so a GPU run can A/B the working
# tree's library against it in one session (tools/gpu_session.sh kbench / sampler / gp64 ...).
# The revision is built by its OWN Makefile (its translation units and per-unit scheduler
# flags), so a revision with more units than rvk.hip..rvk_gp64.hip links completely.
# Usage: tools/ab_rev.sh REV name
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
WT=$(mktemp -d /tmp/rvk_ab.XXXX)
git worktree add -q --detach "$WT" "$REV"
make -s -j8 -C "$WT"/ravest_amd
mkdir -p varlib
cp "$WT"/ravest_amd/lib/librvk.so varlib/librvk_$NAME.so
git worktree remove --force "$WT"
python -c "import ctypes, sys; ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL | 2)" varlib/librvk_$NAME.so  # RTLD_NOW: no undefined symbol
ls -la varlib/librvk_$NAME.so
