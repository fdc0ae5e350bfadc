#!/bin/bash
# Round-3 evidence for profiles/: kernel-trace stats of the driver's bench command, then the PMC
# passes (configs 2/3/4, config-5 GP fp32 and fp64, predictive).  usage: profiles/session_scripts/prof_round3.sh OUT [part]
O=${1:-gpurun_out/prof3}
PART=${2:-all}
mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" = all ] || [ "$PART" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/trace.log || { tail $O/trace.log; exit 1; }
fi
if [ "$PART" = all ] || [ "$PART" = ll ]; then
  for C in 2 3 4; do
    timeout -k 10 600 bash tools/pmc.sh $O/pmc$C $C > $O/pmc$C.log 2>&1 || { tail -20 $O/pmc$C.log; exit 1; }
  done
fi
if [ "$PART" = all ] || [ "$PART" = gp ]; then
  timeout -k 10 600 bash tools/pmc_gp.sh $O/pmc5 fp32+fp64 5 gp_loglike_kernel > $O/pmc5.log 2>&1 || { tail -20 $O/pmc5.log; exit 1; }
  timeout -k 10 600 bash tools/pmc_gp.sh $O/pmc5f64 fp64 config5_fp64 gp64_kernel > $O/pmc5f64.log 2>&1 || { tail -20 $O/pmc5f64.log; exit 1; }
  timeout -k 10 600 bash tools/pmc_pred.sh $O/pmcpred > $O/pmcpred.log 2>&1 || { tail -20 $O/pmcpred.log; exit 1; }
fi
echo done
