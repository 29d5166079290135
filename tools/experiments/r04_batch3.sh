#!/bin/bash
# One GPU call: the K13 / pre-filter / switch / large-k / config suites, then the step breakdown
set -u
O=gpurun_out/r04b3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py tests/test_gpu_parity.py tests/test_gpu_large_k.py \
  tests/test_gpu_baseline_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
bash tools/step_prof.sh r04b3/step > /dev/null || exit 13
head -26 $O/step/breakdown.txt
