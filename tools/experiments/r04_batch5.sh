#!/bin/bash
# PQ: parity suites, then the IVF-PQ bench
set -u
O=gpurun_out/r04b5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_engine_switches.py tests/test_gpu_dropin.py tests/test_gpu_refine.py tests/test_gpu_streaming.py \
  tests/test_gpu_baseline_configs.py -k pq > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/bench_ivf_pq.py --sweep 16 --refine-ratios 10 --gt-queries 200 > $O/pq.log 2>&1 || exit 12
grep -v "^W2026" $O/pq.log | head -4
