#!/bin/bash
# PMC passes (tools/pmc.sh) for the config-2, config-3 and config-4-shard likelihood launches;
# summaries land in gpurun_out/pmcN/pmc_configN.json.  Usage: bash profiles/session_scripts/gpu_pmc_all.sh
set -e
declare -A KF=([2]="loglike_kernel<1, false, 0, true, 0, 1024>" [3]="loglike_seg_kernel<3, true, true, 32>" [4]="loglike_seg_kernel<2, false, true, 32>")
for C in 2 3 4; do
  timeout -k 10 900 bash tools/pmc.sh gpurun_out/pmc$C $C "${KF[$C]}" > gpurun_out/pmc$C.log 2>&1 || { tail -30 gpurun_out/pmc$C.log; exit 1; }
  echo "config $C: $(python -c "import json; d=json.load(open('gpurun_out/pmc$C/pmc_config$C.json')); print(d['kernel'][:70], d.get('valu_insts_per_launch'), d.get('fabric_bytes_per_launch'))")"
done
