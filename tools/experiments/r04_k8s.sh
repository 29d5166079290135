#!/bin/bash
# K8s lane exchanges by DPP / ds_swizzle: every -m gpu test, then the step breakdown twice
set -u
O=gpurun_out/r04k8s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for r in a b; do
  bash tools/step_prof.sh r04k8s/$r > /dev/null || exit 12
  echo "$r: $(head -1 gpurun_out/r04k8s/$r/breakdown.txt)"
  grep "k_select_small\|k_scan_wide" gpurun_out/r04k8s/$r/breakdown.txt
done
