#!/bin/bash
# Build the phase-trace library varlib/trace/librvk_lltrace.so (-DRVK_LL_TRACE=1) from the working tree:
# the likelihood unit (rvk.hip) and the config-2 sampler unit (rvk_sample1.hip) with the stamps, the
# other units from the in-tree build (make first).  tools/ll_trace.py / tools/sampler_trace.py read it.
set -e
cd "$(dirname "$0")/.."
TUS="rvk rvk_sample1" VAROUT=varlib/trace bash tools/varbuild.sh lltrace:"-DRVK_LL_TRACE=1"
