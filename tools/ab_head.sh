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
make -s -j4 -C "$WT"/ravest_amd > /dev/null   # the committed Makefile (its translation units and flags)
cp "$WT"/ravest_amd/lib/librvk.so build/variants/librvk_$NAME.so
git worktree remove --force "$WT"
ls -la build/variants/librvk_$NAME.so
