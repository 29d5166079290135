#!/bin/bash
# K10 (pre-pass) phase clocks on the default bench shape, and the build roofline
set -u
O=gpurun_out/${1:-r05k10}
mkdir -p $O
export TMPDIR=/tmp
MIVS_PF_FLAGS=32 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" \
  --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $O/b.json > $O/b.log 2>&1 || exit 11
grep "k10 phases" $O/b.log | tail -3
python3 -c "
import json
b=json.load(open('$O/b.json'))
for k,v in b['build_roofline'].items():
    if isinstance(v,dict): print(k, v['ms_per_launch'], v['frac'])
"
