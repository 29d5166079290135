#!/bin/bash
# K13 A/B over the pre-pass sample (MIVS_RS_PRE_DIV) with per-block clocks (MIVS_RS_FLAGS=8), after the
# pre-filter parity tests.
set -u
OUT=gpurun_out/${1:-k13div}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B='--steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0'
for dv in ${DIVS:-1 4 8 16}; do
  MIVS_RS_FLAGS=${RSF:-24} MIVS_RS_PRE_DIV=$dv timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/d$dv.json > $OUT/d$dv.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/d$dv.json'));s=j['search_stats'];print('div=$dv', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['cand_overflow'], s['overflow_queries'])"
  grep "k13 " $OUT/d$dv.log | tail -2
done
MIVS_PF_ROWSTAT=0 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/b10.json > $OUT/b10.log 2>&1 || exit $?
python3 -c "import json;j=json.load(open('$OUT/b10.json'));print('k10', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'])"
