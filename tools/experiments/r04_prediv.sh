#!/bin/bash
# K13 pre-pass sample fraction A/B (fp8 nomination): step time and the main kernels per MIVS_RS_PRE_DIV
set -u
for dv in ${DIVS:-4 3 6 8}; do
  MIVS_RS_PRE_DIV=$dv bash tools/step_prof.sh r04prediv/d$dv > /dev/null || exit 1
  echo "div $dv: $(head -1 gpurun_out/r04prediv/d$dv/breakdown.txt) | $(grep -o '"candidates": [0-9]*' gpurun_out/r04prediv/d$dv/b.json)"
  grep "k_rs_scan\|k_pf_scan\|k_pf_verify\|scatter\|count_lds" gpurun_out/r04prediv/d$dv/breakdown.txt
done
