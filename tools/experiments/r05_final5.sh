#!/bin/bash
# the default bench (every line) under rocprofv3 --kernel-trace --stats; only the stats come back (the trace of a
# whole bench is too large to pull)
set -u
O=gpurun_out/${1:-r05final5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 11; }
rm -f $O/prof/prof_kernel_trace.csv
ls -la $O/prof
