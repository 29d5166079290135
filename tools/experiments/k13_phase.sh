#!/bin/bash
# K13 phase clocks (MIVS_RS_FLAGS 24 = block clocks + per-phase wave-cycles; 25 also skips the epilogue)
set -u
OUT=gpurun_out/${1:-k13ph}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_prefilter.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for f in ${FLAGS:-24 25}; do
  MIVS_RS_FLAGS=$f timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --json-out $OUT/f$f.json > $OUT/f$f.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/f$f.json'));s=j['search_stats'];print('flags=$f', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
  grep "k13 " $OUT/f$f.log | tail -2
done
