#!/bin/bash
# One GPU-box session: tests, smoke, bench (+ variants), rocprof kernel trace of the bench command.
# Usage: bash profiles/session_scripts/gpu_round.sh TAG
TAG=${1:-r}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 120 python bench.py --streams 1 --no-cpu-baseline > $O/bench_s1.json 2>&1 || exit 1
RVK_BENCH_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --no-cpu-baseline > $O/bench_gloo2.json 2> $O/bench_gloo2.err || echo "gloo2 failed"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
echo done
