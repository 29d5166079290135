#!/bin/bash
# K13 A/B: wave priority (MIVS_RS_PRIO) off / on, alternated, plain and with phase clocks; parity tests first.
set -u
OUT=gpurun_out/${1:-k13prio}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for p in ${PRIOS:-0 1}; do
    MIVS_RS_PRIO=$p timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/p${p}_$r.json > $OUT/p${p}_$r.log 2>&1 || exit $?
    python3 -c "import json;j=json.load(open('$OUT/p${p}_$r.json'));print('prio=$p run $r', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['roofline']['frac'], j['recall_at_10'])"
  done
done
for p in ${PRIOS:-0 1}; do
  MIVS_RS_PRIO=$p MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/ph$p.json > $OUT/ph$p.log 2>&1 || exit $?
  echo "prio=$p phases:"; grep "k13 " $OUT/ph$p.log | tail -3
done
