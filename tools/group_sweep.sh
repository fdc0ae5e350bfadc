#!/bin/bash
# N>1 bench path at RCCL world 1: sweep of gather mode x steps per gather (probe), then one
# rocprofv3 kernel trace of the default grouped run.   bash tools/group_sweep.sh TAG
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
OFF="--no-cpu-baseline --no-gp --no-predictive --no-host-path --no-sampler --no-configs"
port=29600
run() {  # name args...
  local name=$1; shift
  port=$((port + 1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
    --master-port=$port bench.py --group --steps 20 --warmup 5 $OFF "$@" > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', 'us/step=%.3f' % (d['ms_per_step']*1e3), 'kernel=%.3f' % (d['kernel_ms']*1e3), d['logprob_agreement']['ranks_bitwise_identical'])"
}
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 $OFF > $O/n1_$rep.json 2> $O/n1_$rep.err || exit 1
  python -c "import json; d=json.loads(open('$O/n1_$rep.json').read().strip().splitlines()[-1]); print('n1', 'us/step=%.3f' % (d['ms_per_step']*1e3))"
  for G in 20 10 5 2; do
    run graph_G${G}_$rep --gather graph --gather-steps $G
    run none_G${G}_$rep --gather none --gather-steps $G
  done
  run stream_G20_$rep --gather stream --gather-steps 20
  run stream_G10_$rep --gather stream --gather-steps 10
done
port=$((port + 1))
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$port bench.py --group --steps 20 --warmup 5 $OFF \
  > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
echo "group_sweep: done"
