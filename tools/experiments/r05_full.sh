#!/bin/bash
# the -m gpu suite, then the default bench exactly as the driver runs it (every side line)
set -u
O=gpurun_out/${1:-r05full}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05full} || exit 11
timeout -k 10 900 python3 -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 12; }
grep "^\[" $O/bench.log | tail -40
