#!/bin/bash
# round-5 final evidence, part 1: the default bench exactly as the driver runs it, then the same under
# rocprofv3 --kernel-trace --stats
set -u
O=gpurun_out/${1:-r05final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 11; }
grep "^\[" $O/bench.log | tail -40
timeout -k 10 700 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 12; }
ls $O/prof
