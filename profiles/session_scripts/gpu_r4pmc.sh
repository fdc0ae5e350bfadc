#!/bin/bash
# PMC refresh: likelihood configs 2/3/4, the predictive, GP fp32 (config 5) and GP fp64 -- each counter
# group its own rocprofv3 --pmc pass (tools/pmc.sh, pmc_pred.sh, pmc_gp.sh).  Summaries -> gpurun_out/pmc*/.
export TMPDIR=/tmp
bash profiles/session_scripts/gpu_pmc_all.sh || exit 1
timeout -k 10 600 bash tools/pmc_pred.sh gpurun_out/pmc_pred > gpurun_out/pmc_pred.log 2>&1 || { tail -20 gpurun_out/pmc_pred.log; exit 1; }
echo "pred done"
timeout -k 10 600 bash tools/pmc_gp.sh gpurun_out/pmc_gp32 fp32+fp64 5 gp_loglike_kernel > gpurun_out/pmc_gp32.log 2>&1 || { tail -20 gpurun_out/pmc_gp32.log; exit 1; }
echo "gp32 done"
timeout -k 10 600 bash tools/pmc_gp.sh gpurun_out/pmc_gp64 fp64 5_fp64 gp64_kernel > gpurun_out/pmc_gp64.log 2>&1 || { tail -20 gpurun_out/pmc_gp64.log; exit 1; }
echo "gp64 done"
