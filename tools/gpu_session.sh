#!/bin/bash
# One GPU-box session, steps chosen on the command line (replaces the per-round gpu_r*.sh scripts):
#   bash tools/gpu_session.sh TAG step [step ...]
# steps:
#   tests      pytest -m gpu (whole suite; PYTEST_K narrows it with -k)
#   vartests   VARTESTS (default: the parity and layout GPU tests) on every varlib/librvk_*.so
#   smoke      __graft_entry__.smoke()
#   bench      the driver's command: bench.py --steps 20 --warmup 5
#   prof       the same command under rocprofv3 --kernel-trace --stats (stats kept)
#   profnh     bench.py --no-host-path under rocprofv3 (the device-resident launches only)
#   kbench     tools/kbench.py: the in-tree library, then every $VARDIR/librvk_*.so (default varlib/), interleaved (REPS)
#   hostphase  tools/host_phase_probe.py 4096 (the blocking rvk_loglike call by phase): in-tree, then variants
#   decomp     tools/decomp.py (trivial / 1-epoch / N, W sweeps) on the in-tree library
#   lltrace    tools/ll_trace.py on varlib/trace/librvk_lltrace.so (tools/ll_trace.sh builds it)
#   sampler    tools/sampler_variants.py (raw device stretch move, 3 posteriors + config 3): in-tree, then variants
#   gp64       tools/gp_bench.py 4096 512 fp64: in-tree library, then varlib/librvk_*.so
#   gp32       tools/gp_bench.py 4096 512 fp32: in-tree library, then varlib/librvk_*.so
#   group      bench.py --group on a world-size-1 RCCL group
#   pmc2|pmc3|pmc4|pmc5|pmc5d|pmcpred   the PMC passes of tools/pmc*.sh (one counter group per pass)
# Every GPU step runs under its own timeout; the script stops at the first failing step.
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
REPS=${REPS:-3}
VARS=$(ls ${VARDIR:-varlib}/librvk_*.so 2>/dev/null)
fail() { echo "FAILED: $1"; tail -30 "$2" 2>/dev/null; exit 1; }
ab() {   # ab NAME TIMEOUT cmd...: in-tree library then each variant, REPS interleaved rounds
  local name=$1 to=$2; shift 2
  for rep in $(seq 1 $REPS); do
    timeout -k 10 $to "$@" > $O/${name}_main_$rep.log 2>&1 || fail "$name main" $O/${name}_main_$rep.log
    for so in $VARS; do
      v=$(basename $so .so)
      RAVEST_AMD_LIB=$so timeout -k 10 $to "$@" > $O/${name}_${v}_$rep.log 2>&1 || fail "$name $v" $O/${name}_${v}_$rep.log
    done
  done
  echo "$name: done ($REPS reps, variants: $VARS)"
}
for step in "$@"; do
  case $step in
  tests)
    K=${PYTEST_K:+-k "$PYTEST_K"}
    eval timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 \
      || fail tests $O/pytest_gpu.log
    echo "tests: $(tail -1 $O/pytest_gpu.log)" ;;
  vartests)   # VARTESTS (default: parity + layout) on every varlib/librvk_*.so
    for so in $VARS; do
      v=$(basename $so .so)
      RAVEST_AMD_LIB=$so timeout -k 10 600 python -u -m pytest ${VARTESTS:-tests/test_gpu_parity.py tests/test_gpu_layout.py} \
        -m gpu -x -q --timeout 120 --timeout-method thread > $O/vartests_$v.log 2>&1 || fail "vartests $v" $O/vartests_$v.log
      echo "vartests $v: $(tail -1 $O/vartests_$v.log)"
    done ;;
  smoke)
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
    tail -1 $O/smoke.log ;;
  bench)
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
    python tools/bench_summary.py $O/bench.json ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 \
      > $O/bench_under_rocprof.json 2> $O/rocprof.err || fail prof $O/rocprof.err
    find $O/prof -type f ! -name "*stats*" -delete; echo "prof: done" ;;
  profnh)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profnh -o run -- python bench.py --steps 20 --warmup 5 --no-host-path \
      > $O/bench_under_rocprof_nh.json 2> $O/rocprof_nh.err || fail profnh $O/rocprof_nh.err
    find $O/profnh -type f ! -name "*stats*" -delete; echo "profnh: done" ;;
  kbench)  ab kbench 200 python tools/kbench.py ;;
  hostphase) ab hostphase 150 python tools/host_phase_probe.py 4096 ;;
  sampler) ab sampler 300 python tools/sampler_variants.py uniform beta vaneylen cfg3 ;;
  gp64)    ab gp64 150 python tools/gp_bench.py 4096 512 fp64 ;;
  gp32)    ab gp32 150 python tools/gp_bench.py 4096 512 fp32 ;;
  decomp)
    timeout -k 10 200 python tools/decomp.py > $O/decomp.log 2>&1 || fail decomp $O/decomp.log
    echo "decomp: done" ;;
  lltrace)
    for W in 4096 2048; do
      RAVEST_AMD_LIB=varlib/trace/librvk_lltrace.so timeout -k 10 120 python tools/ll_trace.py $W > $O/lltrace_$W.log 2>&1 \
        || fail lltrace $O/lltrace_$W.log
    done; echo "lltrace: done" ;;
  group)
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29561 \
      bench.py --group --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive --no-host-path > $O/bench_group.out 2> $O/bench_group.err \
      || fail group $O/bench_group.err
    echo "group: done" ;;
  pmc2|pmc3|pmc4) bash tools/pmc.sh $O/$step ${step#pmc} || fail $step /dev/null ;;
  pmc5)    bash tools/pmc_gp.sh $O/$step || fail $step /dev/null ;;
  pmc5d)   bash tools/pmc_gp.sh $O/$step fp64 5_fp64 gp64_kernel || fail $step /dev/null ;;
  pmcpred) bash tools/pmc_pred.sh $O/$step || fail $step /dev/null ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG: all steps done"
