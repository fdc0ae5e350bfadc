#!/bin/bash
# N>1 bench path at RCCL world 1 against the N=1 line, interleaved on one box:
#   bash tools/group_ab.sh TAG [REPS]
# n1: the driver's command (bench.py --steps 20 --warmup 5, sub-lines off)
# graph / stream: bench.py --group under torch.distributed.run, --gather graph | stream
TAG=${1:?tag}; REPS=${2:-3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
OFF="--no-cpu-baseline --no-gp --no-predictive --no-host-path --no-sampler --no-configs"
port=29570
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 $OFF > $O/n1_$rep.json 2> $O/n1_$rep.err || { tail -20 $O/n1_$rep.err; exit 1; }
  for mode in graph stream; do
    port=$((port + 1))
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
      --master-port=$port bench.py --group --gather $mode --steps 20 --warmup 5 $OFF \
      > $O/${mode}_$rep.json 2> $O/${mode}_$rep.err || { tail -30 $O/${mode}_$rep.err; exit 1; }
  done
  python - $O $rep <<'EOF'
import json, sys
o, rep = sys.argv[1], sys.argv[2]
for m in ("n1", "graph", "stream"):
    d = json.loads(open(f"{o}/{m}_{rep}.json").read().strip().splitlines()[-1])
    print(rep, m, "ms_per_step_us=%.3f" % (d["ms_per_step"] * 1e3), "kernel_us=%.3f" % (d["kernel_ms"] * 1e3),
          "bitwise=%s" % d["logprob_agreement"]["ranks_bitwise_identical"], flush=True)
EOF
done

# gloo rehearsal of the N>1 path, 2 ranks sharing the card (bitwise check only)
RVK_BENCH_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29599 bench.py --steps 20 --warmup 5 --gpus 2 $OFF > $O/gloo2.json 2> $O/gloo2.err || { tail -30 $O/gloo2.err; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/gloo2.json').read().strip().splitlines()[-1]); print('gloo2 bitwise', d['logprob_agreement']['ranks_bitwise_identical'])"
echo "group_ab: done"
