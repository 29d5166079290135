#!/bin/bash
set -u
OUT=gpurun_out/pqrt
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pq" > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine_switches.py -k "pq" > $OUT/sw.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/sw.log; tail -3 $OUT/sw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/bench_ivf_pq.py --sweep 16,32 --refine-ratios 10 > $OUT/bench.log 2>&1 || exit $?
grep -E "build|search|refine" $OUT/bench.log
