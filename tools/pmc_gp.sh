#!/bin/bash
# PMC passes for a GP kernel (config 5, tools/gp_bench.py), one counter group per rocprofv3 pass.
# usage: tools/pmc_gp.sh OUT [precision=fp32+fp64] [label=config5] [kernel filter=gp_loglike_kernel]
set -e
OUT=${1:-gpurun_out/pmc_gp}
PREC=${2:-fp32+fp64}
LABEL=${3:-5}
KF=${4:-gp_loglike_kernel}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python tools/gp_bench.py 4096 512 $PREC"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
done
# the fp64 MFMA op counter in a pass of its own (optional: skipped if this ROCm lacks it)
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 --output-format csv -d $OUT/p9 -o run -- $CMD > $OUT/p9.log 2>&1 || true
python tools/pmc_summary.py $OUT $LABEL $KF "$CMD"
rm -rf $OUT/p[0-9]*/
