#!/bin/bash
# PMC passes for the GP kernel (config 5, tools/gp_bench.py), one counter group per rocprofv3 pass.
set -e
OUT=${1:-gpurun_out/pmc_gp}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python tools/gp_bench.py"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F32"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT 5 gp_loglike_kernel
