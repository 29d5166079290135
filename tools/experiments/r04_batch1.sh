#!/bin/bash
# One GPU call: parity of the changed paths, the IVF-PQ bench, and the step breakdown A/B of the K11 gather.
set -u
O=gpurun_out/r04b1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_dropin.py \
  tests/test_gpu_refine.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/bench_ivf_pq.py --sweep 16 --refine-ratios 10 --gt-queries 200 > $O/pq_bench.log 2>&1 || exit 12
grep -v "^W2026" $O/pq_bench.log | head -4
bash tools/step_prof.sh r04b1/step_gather > /dev/null || exit 13
MIVS_K11_GATHER=0 bash tools/step_prof.sh r04b1/step_nogather > /dev/null || exit 14
head -16 $O/step_gather/breakdown.txt
grep "k_pf_refine\|window" $O/step_nogather/breakdown.txt
