#!/bin/bash
# graph size at the driver's K = 20: steps per graph G = 20 / 10 / 5 / 4, 3 interleaved reps
O=gpurun_out/r4g; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for G in 20 10 5 4; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph-steps $G --no-cpu-baseline --no-sampler --no-gp --no-predictive --no-configs --no-host-path > $O/b_${G}_$rep.json 2>/dev/null || { echo "fail $G"; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${G}_$rep.json').read().strip().splitlines()[-1]); print('G=$G', round(d['ms_per_step']*1e3,3), round(d['kernel_ms']*1e3,3), d['config'].get('launch', d.get('launch')))"
  done
done
