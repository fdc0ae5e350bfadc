#!/bin/bash
# PMC passes for the posterior-predictive kernel (bench.py's predictive line: predict_kernel),
# one counter group per rocprofv3 --pmc pass (no trace domains); summary -> OUT/pmc_predictive.json.
set -e
OUT=${1:-gpurun_out/pmc_pred}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline --no-sampler --no-gp --no-configs --no-host-path"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FLOPS_FP32 SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT predictive predict_kernel "$CMD"
rm -rf $OUT/p[0-9]*/
