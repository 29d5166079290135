#!/bin/bash
# K13's probe map + tile images on a side stream beside the pre-pass (MIVS_RS_FORK): every -m gpu test, then the
# default bench's main line alternating fork on / off
set -u
O=gpurun_out/r04fk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for r in 1 0 1 0; do
  MIVS_RS_FORK=$r timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --json-out $O/b$r.json > $O/b$r.log 2>&1 || { tail -20 $O/b$r.log; exit 12; }
  python3 -c "import json;b=json.load(open('$O/b$r.json'));print('fork $r', b['value'], b['ms_per_step'], b['roofline']['launch_ms'], b['recall_at_10'])"
done
