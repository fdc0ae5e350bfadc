#!/bin/bash
# Round-4 session, part A: GPU tests + smoke + host probe + group bench + bench line (profiles/session_scripts/gpu_r4.sh),
# then the fp64 GP kernel A/B.  Usage: profiles/session_scripts/gpu_r4b.sh TAG
TAG=${1:-r4b}
bash profiles/session_scripts/gpu_r4.sh $TAG || exit 1
bash tools/gp64_ab.sh ${TAG}_gp || exit 1
echo done
