#!/bin/bash
# round 5: the -m gpu suite, then the default bench's main line with the side lines that changed (latency, build
# roofline, CPU baseline)
set -u
O=gpurun_out/${1:-r05c}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05c} || exit 11
timeout -k 10 600 python3 -u bench.py --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --sweep "" \
  --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 12; }
grep "^\[" $O/bench.log | tail -20
