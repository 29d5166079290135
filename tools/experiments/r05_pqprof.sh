#!/bin/bash
# the -m gpu engine-switch tests (back-to-back searches), then the IVF-PQ refined operating point (n_probes 10,
# 120 candidates) under the kernel trace: where the refined batch's time goes
set -u
O=gpurun_out/${1:-r05pq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine_switches.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 11; }
tail -2 $O/tests.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 -u tools/bench_ivf_pq.py --sweep 10 --refine-ratios 12 --gt-queries 64 > $O/b.log 2>&1 || exit 12
head -16 $O/kt/kt_kernel_stats.csv | cut -d, -f1-4
grep -v "^\s*$" $O/b.log | tail -8
