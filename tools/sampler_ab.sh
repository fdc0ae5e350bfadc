#!/bin/bash
# Sampler: GPU tests (device sampler parity), then bench.py's device stretch-move line (HIP events), base vs variants.
O=gpurun_out/${1:-samp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_device_posterior.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive --no-configs"
ext() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['sampler']['ms_per_step']*1e3,2), 'us/step')" $1; }
for rep in 1 2 3; do
  timeout -k 10 120 $B > $O/base_$rep.json 2>/dev/null || { echo fail; exit 1; }
  echo "base $(ext $O/base_$rep.json)"
  for so in build/variants/librvk_*.so; do
    v=$(basename $so .so)
    RAVEST_AMD_LIB=$so timeout -k 10 120 $B > $O/${v}_$rep.json 2>/dev/null || { echo fail $v; exit 1; }
    echo "$v $(ext $O/${v}_$rep.json)"
  done
done
