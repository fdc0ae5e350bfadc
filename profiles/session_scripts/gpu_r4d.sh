#!/bin/bash
# Targeted re-check: the sharded/RCCL/GP tests and GP parity on the balanced row map, the --group
# bench with torchrun's logs, then session part B (profiles/session_scripts/gpu_r4c.sh).
TAG=${1:-r4d}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_sampler.py tests/test_gpu_gp64.py tests/test_gpu_hostpath.py -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29561 --log-dir $O/tr_logs --redirects 3 --tee 3 bench.py --group --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive > $O/bench_group.json 2> $O/bench_group.err
echo "group bench rc=$?"; find $O/tr_logs -type f | head; tail -c 2000 $O/bench_group.json
bash profiles/session_scripts/gpu_r4c.sh $TAG
