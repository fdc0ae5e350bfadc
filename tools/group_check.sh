#!/bin/bash
# The N > 1 bench path on one GPU: RCCL world 1 (graph form), RCCL world 1 with the capture refused on
# rank 0 (the agreed host-issued fallback), and the gloo 2-rank rehearsal (ranks share the card).
O=gpurun_out/${1:-groupchk}; mkdir -p $O
export TMPDIR=/tmp
OFF="--no-cpu-baseline --no-gp --no-predictive --no-host-path"
run() {  # name env... -- args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $O/$name.json 2> $O/$name.err || { echo "FAILED $name"; tail -30 $O/$name.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); pg=d.get('process_group',{}); print('$name', round(d['ms_per_step']*1e3,3), 'us/step', pg.get('gather'), 'bitwise', d['logprob_agreement']['ranks_bitwise_identical'])"
}
run rccl1 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29571 bench.py --group --steps 20 --warmup 5 $OFF
run rccl1_fallback RVK_BENCH_NO_CAPTURE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29572 bench.py --group --steps 20 --warmup 5 $OFF
run gloo2 RVK_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29573 bench.py --steps 20 --warmup 5 --gpus 2 $OFF
