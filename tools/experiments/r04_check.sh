#!/bin/bash
# the committed tree: every -m gpu test, then the bench's main line
set -u
O=gpurun_out/r04chk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --json-out $O/b.json > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 12; }
python3 -c "import json;b=json.load(open('$O/b.json'));print(b['value'], b['ms_per_step'], b['roofline']['frac'])"
