#!/bin/bash
# aggregator GPU tests, then the bench's one-process aggregator side line (with the main line)
set -u
O=gpurun_out/${1:-r05agg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_exchange.py tests/test_gpu_multidevice.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 \
  --pq-rows 0 --large-k "" --latency "" --batch-sweep "" --json-out $O/b.json > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 12; }
grep "^\[search\]\|^\[single" $O/b.log
