#!/bin/bash
# K13 dual vs single: parity tests for both variants, then the bench over pre-pass samples.
set -u
OUT=gpurun_out/${1:-k13ab2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MIVS_RS_DUAL=0 timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_prefilter.py > $OUT/tests_single.log 2>&1
rc=$?; echo "pytest(single) rc=$rc" >> $OUT/tests_single.log; tail -2 $OUT/tests_single.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local nm=$1; shift
  env "$@" MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/$nm.json > $OUT/$nm.log 2>&1 || return $?
  python3 -c "import json;j=json.load(open('$OUT/$nm.json'));s=j['search_stats'];print('$nm', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['cand_overflow'], s['overflow_queries'])"
  grep "k13 " $OUT/$nm.log | tail -2
}
run dual_d1 MIVS_RS_PRE_DIV=1 || exit 1
run dual_d4 MIVS_RS_PRE_DIV=4 || exit 1
run dual_d8 MIVS_RS_PRE_DIV=8 || exit 1
run single_d4 MIVS_RS_PRE_DIV=4 MIVS_RS_DUAL=0 || exit 1
