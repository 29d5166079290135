#!/bin/bash
# One GPU round trip: the -m gpu suite (optional selection), then a quick default bench (IVF-Flat line only) and
# the same bench with K13 phase clocks. Each step under its own time limit; the script stops at the first failure.
# Usage: bash tools/gpu_check.sh TAG [pytest selection...]   (TESTS=0: skip the suite; PHASE=0: skip the clocks)
set -u
TAG=${1:-chk}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread "${@:-tests}" > $OUT/tests.log 2>&1
  rc=$?
  tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
QB="--steps 10 --warmup 2 --no-cpu-baseline --sweep '' --flat-rows 0 --pq-rows 0 --large-k '' --single-process 0 --gt-queries 500"
eval timeout -k 10 300 python -u bench.py $QB --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 3; }
python3 -c "import json;j=json.load(open('$OUT/bench.json'));r=j['roofline'];print('value',j['value'],'ms',j['ms_per_step'],'recall',j['recall_at_10'],'k13_ms',r['launch_ms'],'frac',r['frac'],'cand',j['search_stats']['candidates'])"
if [ "${PHASE:-1}" = "1" ]; then
  eval MIVS_RS_FLAGS=24 timeout -k 10 300 python -u bench.py $QB > $OUT/phase.log 2>&1 || { echo "phase run failed"; exit 4; }
  grep "k13" $OUT/phase.log | tail -3
fi
