#!/bin/bash
# Final check of the committed tree: every GPU test, smoke, the default bench line.
O=gpurun_out/r4check; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step']*1e3, 'kernel us', d['kernel_ms']*1e3, 'steps', d['steps'], d['warmup'])
print('sampler', d['sampler']['ms_per_step']*1e3, 'host stretch', d['sampler']['host_stretch_move_ms_per_step'], 'gp', d['gp_config5']['ms_per_eval'], d['gp_config5']['fp64']['ms_per_eval'])
"
