#!/bin/bash
# Round-4 session check on a GPU box.  Usage: bash profiles/session_scripts/gpu_r4.sh TAG [pytest selection...]
# Steps (each under its own time limit, stop at the first failure): the GPU tests given (default:
# all), smoke, the host-path probe, the N>1 bench path on a world-size-1 RCCL group, the bench line.
TAG=${1:-r4}
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu --maxfail=8 -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR|Error:" $O/pytest_gpu.log | head -30
  [ $rc -eq 1 ] || exit 1          # only ordinary test failures go on to the measurements
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 180 python tools/host_step_probe.py > $O/host_probe.json 2> $O/host_probe.err || { tail -20 $O/host_probe.err; exit 1; }
cat $O/host_probe.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29561 --log-dir $O/tr_logs --redirects 3 --tee 3 bench.py --group --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive > $O/bench_group.json 2> $O/bench_group.err || { tail -30 $O/bench_group.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_group.json'))
print('group', d.get('process_group'), 'value', d['value'], 'ranks_same', d['logprob_agreement']['ranks_bitwise_identical'])
print('c4 sharded', d.get('config4_sharded')); print('c4 sampler', d.get('config4_sampler'))
"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step']*1e3, 'kernel us', d['kernel_ms']*1e3, 'host call us', d['host_path_ms_per_call']*1e3)
print('sampler', {k: v for k, v in d.get('sampler', {}).items() if 'ms' in k or 'over' in k})
print('host_path', json.dumps(d.get('host_path'), indent=1))
print('gp', d['gp_config5']['ms_per_eval'], d['gp_config5']['fp64']['ms_per_eval'])
"
echo done
