#!/bin/bash
# One GPU call: parity of the split K11 (switch, prefilter, parity, baseline-config suites), then the step breakdown
set -u
O=gpurun_out/r04b2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_large_k.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
bash tools/step_prof.sh r04b2/step > /dev/null || exit 13
MIVS_K11_SPLIT=0 bash tools/step_prof.sh r04b2/step_nosplit > /dev/null || exit 14
head -22 $O/step/breakdown.txt
grep "k_pf_r\|window" $O/step_nosplit/breakdown.txt
