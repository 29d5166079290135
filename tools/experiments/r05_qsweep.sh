#!/bin/bash
# default bench shape at several query batch sizes (QPS vs batch)
set -u
O=gpurun_out/${1:-r05q}
mkdir -p $O
export TMPDIR=/tmp
for nq in 20000 5000 32768; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gt-queries 100 --sweep "" --queries $nq \
    --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" > $O/q$nq.log 2>&1 || exit 11
  python3 -c "
import json,sys
for ln in open('$O/q$nq.log'):
    if ln.startswith('{'):
        b=json.loads(ln); print($nq, b['value'], b['ms_per_step'], b['roofline']['launch_ms'], b['recall_at_10'])
"
done
