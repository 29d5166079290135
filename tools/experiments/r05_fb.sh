#!/bin/bash
# device-sized fallback: switch/oracle tests, then the default bench with it and with the host-sized one (A/B, twice)
set -u
O=gpurun_out/${1:-r05fb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/k13_probe 3000 > $O/probe.log 2>&1 || exit 10
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine_switches.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
for r in 1 2; do
  for m in 0 1; do
    MIVS_FALLBACK_SYNC=$m timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 100 \
      --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" > $O/b$m-$r.log 2>&1 || exit 12
    python3 -c "
import json
for ln in open('$O/b$m-$r.log'):
    if ln.startswith('{'):
        b=json.loads(ln); print('sync=$m run $r', b['value'], b['ms_per_step'], b['roofline']['launch_ms'], b['search_stats']['overflow_queries'])
"
  done
done
cat $O/probe.log
bash tools/experiments/r05_qsweep.sh ${1:-r05fb}_q
