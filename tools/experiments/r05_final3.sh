#!/bin/bash
# the -m gpu suite on the final tree, then the default bench exactly as the driver runs it
set -u
O=gpurun_out/${1:-r05final3}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05final3} || exit 11
timeout -k 10 700 python3 -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 12; }
grep "^\[" $O/bench.log | tail -40
