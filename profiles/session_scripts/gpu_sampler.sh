#!/bin/bash
# Sampler session: device-posterior / sampler GPU tests, then bench.py's device stretch-move line
# (HIP events) with the fused half-step and the two-kernel path (RVK_SAMPLER_FUSE=0), and a
# rocprof kernel-stats pass of the sampler bench.  Usage: bash profiles/session_scripts/gpu_sampler.sh TAG
O=gpurun_out/${1:-samp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_device_posterior.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive --no-configs"
ext() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['sampler']['ms_per_step']*1e3,2), 'us/step', round(d['sampler']['acceptance'],4))" $1; }
for rep in 1 2; do
  timeout -k 10 120 $B > $O/fused_$rep.json 2>/dev/null || { echo fail; exit 1; }
  echo "fused $(ext $O/fused_$rep.json)"
  RVK_SAMPLER_FUSE=0 timeout -k 10 120 $B > $O/unfused_$rep.json 2>/dev/null || { echo fail; exit 1; }
  echo "unfused $(ext $O/unfused_$rep.json)"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $B > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
