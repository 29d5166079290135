#!/bin/bash
# K13 A/B: v_mfma 32x32x16 (default) vs 16x16x32 (MIVS_RS_SHAPE=16): parity suites through the S16 path
# first, then alternating benches and phase clocks; then the pre-pass sample A/B (MIVS_RS_PRE_DIV).
set -u
OUT=gpurun_out/${1:-k13s16}
mkdir -p $OUT
export TMPDIR=/tmp
MIVS_RS_SHAPE=16 timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_engine_switches.py tests/test_gpu_cosine.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sh in 0 16; do
    MIVS_RS_SHAPE=$sh timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/s${sh}_$r.json > $OUT/s${sh}_$r.log 2>&1 || exit $?
    python3 -c "import json;j=json.load(open('$OUT/s${sh}_$r.json'));s=j['search_stats'];print('shape=$sh run $r', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['roofline']['frac'], j['recall_at_10'], 'cand', s['candidates'])"
  done
done
for sh in 0 16; do
  MIVS_RS_SHAPE=$sh MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/ph$sh.log 2>&1 || exit $?
  echo "shape=$sh phases:"; grep "k13 " $OUT/ph$sh.log | tail -3
done
for dv in 2 1; do
  MIVS_RS_SHAPE=16 MIVS_RS_PRE_DIV=$dv timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/d$dv.json > $OUT/d$dv.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/d$dv.json'));s=j['search_stats'];print('s16 div=$dv', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
done
