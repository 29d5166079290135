#!/bin/bash
# PQ parity (DUMP / register paths), K13 dual-variant parity, then the bench for both K13 variants
set -u
OUT=gpurun_out/${1:-k13dual}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pq" > $OUT/pq_tests.log 2>&1
rc=$?; echo "pytest(pq) rc=$rc" >> $OUT/pq_tests.log; tail -2 $OUT/pq_tests.log
[ $rc -eq 0 ] || exit $rc
MIVS_RS_DUAL=1 timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py -k "not pq" > $OUT/dual_tests.log 2>&1
rc=$?; echo "pytest(dual) rc=$rc" >> $OUT/dual_tests.log; tail -2 $OUT/dual_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MIVS_RS_DUAL=$v MIVS_RS_FLAGS=8 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/dual$v.json > $OUT/dual$v.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/dual$v.json'));s=j['search_stats'];print('dual=$v', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['cand_overflow'], s['overflow_queries'])"
  grep "k13 " $OUT/dual$v.log | tail -1
done
