#!/bin/bash
# the default bench's main line only, twice (no side lines)
set -u
O=gpurun_out/r04bq
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --json-out $O/b$r.json > $O/b$r.log 2>&1 || { tail -20 $O/b$r.log; exit 12; }
  python3 -c "import json;b=json.load(open('$O/b$r.json'));print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['launch_ms'])"
done
