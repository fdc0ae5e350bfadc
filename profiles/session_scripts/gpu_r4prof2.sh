#!/bin/bash
# The bench command without the host-path lines (whose zero-copy rvk_loglike calls launch the same
# kernel reading host memory) under rocprofv3 --kernel-trace --stats: the hot kernel's average is then
# the timed launches' (plus warmup), comparable with the line's live kernel_ms.
O=gpurun_out/${1:-r4prof2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-host-path > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
find $O/prof -type f ! -name "*stats*" -delete
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
