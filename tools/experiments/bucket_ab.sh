#!/bin/bash
# K13 stream bucketing A/B: parity suites through the pre-filter, then alternating benches with the
# grouped LDS-histogram bucketing (default) and the flat atomics (MIVS_RS_BUCKET_FLAT=1), then a kernel
# trace of the default for the step breakdown.
set -u
OUT=gpurun_out/${1:-bucket}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py tests/test_gpu_baseline_configs.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    MIVS_RS_BUCKET_FLAT=$f timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/b${r}_f$f.json > $OUT/b${r}_f$f.log 2>&1 || exit $?
    python3 -c "import json;j=json.load(open('$OUT/b${r}_f$f.json'));s=j['search_stats'];print('run $r flat=$f', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/kt.log 2>&1 || exit $?
python3 tools/step_breakdown.py $OUT/kt/kt_kernel_trace.csv 3 20 | head -16
