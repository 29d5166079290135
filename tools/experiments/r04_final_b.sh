#!/bin/bash
# Round-end evidence, part 2: the default bench under rocprofv3 --kernel-trace --stats
set -u
O=gpurun_out/r04final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 -u bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 12; }
tail -1 $O/bench_prof.log | cut -c1-300
ls $O/prof
