#!/bin/bash
# parity suites that exercise the IVF pre-filter path, then a short bench + step breakdown
set -u
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_engine_switches.py tests/test_gpu_cosine.py tests/test_gpu_dropin.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/b$r.json > $OUT/b$r.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/b$r.json'));s=j['search_stats'];print('run $r', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['roofline']['frac'], j['recall_at_10'], 'cand', s['candidates'], 'ovf', s['overflow_queries'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/kt.log 2>&1 || exit $?
python3 tools/step_breakdown.py $OUT/kt/kt_kernel_trace.csv 3 20 | head -14
