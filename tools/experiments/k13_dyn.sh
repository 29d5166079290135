#!/bin/bash
# K13 item dealing: parity suites through K13, two benches, then the phase / block clocks (MIVS_RS_FLAGS=24)
set -u
OUT=gpurun_out/${1:-dyn}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_engine_switches.py tests/test_gpu_baseline_configs.py tests/test_gpu_cosine.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/b$r.json > $OUT/b$r.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/b$r.json'));s=j['search_stats'];print('run $r', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
done
MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/phase.json > $OUT/phase.log 2>&1 || exit $?
grep "k13 " $OUT/phase.log | tail -3
