bash profiles/session_scripts/gpu_check.sh s2b || exit 1
timeout -k 10 600 bash tools/pmc_gp.sh gpurun_out/s2b/pmc_gp > gpurun_out/s2b/pmc_gp.log 2>&1 || echo "pmc_gp failed"
tail -30 gpurun_out/s2b/pmc_gp.log
