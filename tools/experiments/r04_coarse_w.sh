#!/bin/bash
# coarse probe on K3w DUMP (64-query tiles): every -m gpu test, then the step breakdown
set -u
O=gpurun_out/r04cw2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for r in a b; do
  d=r04cw2/$r
  bash tools/step_prof.sh $d > /dev/null || exit 12
  echo "$r: $(head -1 gpurun_out/$d/breakdown.txt)"
  grep "k_scan\|k_select_small" gpurun_out/$d/breakdown.txt
done
