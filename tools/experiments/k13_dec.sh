#!/bin/bash
# K13 A/B: lock-step tile protocol (MIVS_RS_DEC=0) vs decoupled (=1); parity suites through both first.
set -u
OUT=gpurun_out/${1:-k13dec}
mkdir -p $OUT
export TMPDIR=/tmp
for dv in 1 0; do
  MIVS_RS_DEC=$dv timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_engine_switches.py tests/test_gpu_cosine.py > $OUT/tests$dv.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/tests$dv.log; echo "dec=$dv"; tail -2 $OUT/tests$dv.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for dv in 0 1; do
    MIVS_RS_DEC=$dv timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/d${dv}_$r.json > $OUT/d${dv}_$r.log 2>&1 || exit $?
    python3 -c "import json;j=json.load(open('$OUT/d${dv}_$r.json'));s=j['search_stats'];print('dec=$dv run $r', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['roofline']['frac'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['overflow_queries'])"
  done
done
for dv in 0 1; do
  MIVS_RS_DEC=$dv MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/ph$dv.log 2>&1 || exit $?
  echo "dec=$dv phases:"; grep "k13 " $OUT/ph$dv.log | tail -3
done
