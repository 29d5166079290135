#!/bin/bash
# coarse probe work-item size A/B (MIVS_COARSE_G groups per K3 item; default: >= 4 items per CU)
set -u
for g in ${GS:-0 16 32 0 16}; do
  if [ $g = 0 ]; then unset MIVS_COARSE_G; else export MIVS_COARSE_G=$g; fi
  d=r04cg/g$g$RANDOM
  bash tools/step_prof.sh $d > /dev/null || exit 12
  echo "G $g: $(head -1 gpurun_out/$d/breakdown.txt)"
  grep "k_scan<\|k_select_small" gpurun_out/$d/breakdown.txt
done
