#!/bin/bash
# K11 (final refine) phase ablation at the bench shape: kernel time per flag set (timing-only flags)
set -u
O=gpurun_out/r04k11${1:-}
mkdir -p $O
for f in ${FLAGSETS:-0 2 6}; do
  MIVS_K11_FLAGS=$f bash tools/step_prof.sh r04k11${1:-}/f$f > /dev/null || exit 1
  echo "flags $f: $(grep 'k_pf_refine' $O/f$f/breakdown.txt)"
done
