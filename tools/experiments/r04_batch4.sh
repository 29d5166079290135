#!/bin/bash
# PQ: parity suites, then the IVF-PQ bench with K9r QL=4 (default) and QL=16
set -u
O=gpurun_out/r04b4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_engine_switches.py tests/test_gpu_dropin.py tests/test_gpu_refine.py tests/test_gpu_streaming.py \
  tests/test_gpu_baseline_configs.py -k pq > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/bench_ivf_pq.py --sweep 16 --refine-ratios 10 --gt-queries 200 > $O/pq_ql4.log 2>&1 || exit 12
grep -v "^W2026" $O/pq_ql4.log | head -3
MIVS_PQ_RT_QL=16 timeout -k 10 300 python3 -u tools/bench_ivf_pq.py --sweep 16 --refine-ratios 10 --gt-queries 200 > $O/pq_ql16.log 2>&1 || exit 13
grep -v "^W2026" $O/pq_ql16.log | head -3
