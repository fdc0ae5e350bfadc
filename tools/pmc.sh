#!/bin/bash
# PMC passes for the bench workload (run on the GPU box from the repo root).
# Each counter group in its own rocprofv3 pass, --pmc only (no trace domains),
# as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes.
set -e
OUT=${1:-gpurun_out/pmc}
CFG=${2:-2}
KF=${3:-}          # kernel-name filter (default: the plain loglike launch with the most dispatches)
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-sampler --no-gp --no-predictive --no-configs --no-host-path"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FLOPS_FP32 SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
done
python tools/pmc_summary.py $OUT $CFG "$KF" "$CMD"
rm -rf $OUT/p[0-9]*/   # raw per-dispatch CSVs (tens of MB): the summary is what is kept
