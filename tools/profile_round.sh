#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench command, then PMC passes.
O=gpurun_out/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py > $O/bench_under_rocprof.json 2> $O/trace.log || exit 1
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 800 bash tools/pmc.sh $O/pmc 2 > $O/pmc.log 2>&1 || exit 1
echo done
