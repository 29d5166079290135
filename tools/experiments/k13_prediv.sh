#!/bin/bash
# K13 A/B over the pre-pass sample (MIVS_RS_PRE_DIV: the nearest list's first 1/div groups) with phase clocks:
# a larger sample tightens T_q (fewer filter hits, fewer hit-path epilogues) at a longer pre-pass.
set -u
OUT=gpurun_out/${1:-k13prediv}
mkdir -p $OUT
export TMPDIR=/tmp
for dv in ${DIVS:-4 2 1}; do
  MIVS_RS_PRE_DIV=$dv timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/d$dv.json > $OUT/d$dv.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/d$dv.json'));s=j['search_stats'];print('div=$dv', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
  MIVS_RS_PRE_DIV=$dv MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/ph$dv.log 2>&1 || exit $?
  grep "k13 " $OUT/ph$dv.log | tail -3
done
