#!/bin/bash
# K13 step breakdown: bench + rocprofv3 kernel-trace per pre-pass sample (MIVS_RS_PRE_DIV)
set -u
OUT=gpurun_out/${1:-k13kt}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_exchange.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for dv in ${DIVS:-4 8}; do
  MIVS_RS_FLAGS=24 MIVS_RS_PRE_DIV=$dv timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/d$dv.json > $OUT/d$dv.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/d$dv.json'));s=j['search_stats'];print('div=$dv', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['cand_overflow'], s['overflow_queries'])"
  grep "k13 " $OUT/d$dv.log | tail -2
  [ "$dv" = "${KTDIV:-4}" ] || continue
  MIVS_RS_PRE_DIV=$dv timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt$dv -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 > $OUT/kt$dv.log 2>&1 || exit $?
  python3 tools/kt_top.py $OUT/kt$dv/kt_kernel_stats.csv 28 | tee $OUT/kt_top$dv.txt
done
MIVS_PF_ROWSTAT=0 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/k10.json > $OUT/k10.log 2>&1 || exit $?
python3 -c "import json;j=json.load(open('$OUT/k10.json'));print('k10', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'])"
