#!/bin/bash
# The driver's bench command under rocprofv3 --kernel-trace --stats (csv; the stats kept, raw traces dropped)
O=gpurun_out/${1:-r4prof}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
find $O/prof -type f ! -name "*stats*" -delete
find $O/prof -type f
