#!/bin/bash
# Round-3 session check on a GPU box: GPU tests, smoke, bench line.  Usage: bash profiles/session_scripts/gpu_r3.sh TAG [pytest args]
TAG=${1:-r3}
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step']*1e3, 'kernel us', d['kernel_ms']*1e3)
print('sampler', {k: v for k, v in d.get('sampler', {}).items() if 'ms' in k or 'over' in k})
print('config4_sampler', d.get('config4_sampler'))
print('gp', d['gp_config5']['ms_per_eval'], d['gp_config5']['fp64']['ms_per_eval'])
"
echo done
