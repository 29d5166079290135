#!/bin/bash
# K13 dynamic vs static item deal (MIVS_RS_STATIC_DEAL=1), alternating on one box, then phase clocks of each
set -u
OUT=gpurun_out/${1:-dynab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for st in 0 1; do
    MIVS_RS_STATIC_DEAL=$st timeout -k 10 300 python3 bench.py --steps 30 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/b${r}_$st.json > $OUT/b${r}_$st.log 2>&1 || exit $?
    python3 -c "import json;j=json.load(open('$OUT/b${r}_$st.json'));print('run $r static=$st', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'])"
  done
done
for st in 0 1; do
  MIVS_RS_STATIC_DEAL=$st MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/phase$st.json > $OUT/phase$st.log 2>&1 || exit $?
  echo "static=$st"; grep "k13 " $OUT/phase$st.log | tail -3
done
