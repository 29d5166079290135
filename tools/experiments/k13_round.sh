#!/bin/bash
# K13 bring-up: parity tests that exercise the IVF pre-filter path, then a short bench (K13 default) and
# the same bench with K10 (MIVS_PF_ROWSTAT=0) for an A/B.
set -u
OUT=gpurun_out/${1:-k13}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_refine.py tests/test_gpu_baseline_configs.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/b13.json > $OUT/b13.log 2>&1 || exit $?
MIVS_RS_PRE_DIV=1 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/b13d1.json > $OUT/b13d1.log 2>&1 || exit $?
MIVS_RS_PRE_DIV=8 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/b13d8.json > $OUT/b13d8.log 2>&1 || exit $?
MIVS_PF_ROWSTAT=0 timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --json-out $OUT/b10.json > $OUT/b10.log 2>&1 || exit $?
for t in b13 b13d1 b13d8 b10; do python3 -c "import json;j=json.load(open('$OUT/$t.json'));print('$t', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], j['search_stats'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 > $OUT/kt.log 2>&1 || exit $?
python3 tools/kt_top.py $OUT/kt/kt_kernel_stats.csv | tee $OUT/kt_top.txt
