#!/bin/bash
# pre-pass merge early exit (MIVS_PF_SLOT_OUT) + launch trims: every -m gpu test, then the step breakdown with and
# without the early exit
set -u
O=gpurun_out/r04so
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for v in 1 0 1; do
  MIVS_PF_SLOT_OUT=$v bash tools/step_prof.sh r04so/s$v$RANDOM > /dev/null || exit 12
done
for d in gpurun_out/r04so/s*; do
  echo "$d: $(head -1 $d/breakdown.txt) | $(grep -o '"candidates": [0-9]*' $d/b.json)"
  grep "k_rs_scan\|k_pf_scan\|k_pf_verify\|k_rs_tiles" $d/breakdown.txt
done
