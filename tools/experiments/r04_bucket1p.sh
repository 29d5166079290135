#!/bin/bash
# K13 one-pass bucketing: every -m gpu test, then the step breakdown with it and with the two-pass form
set -u
O=gpurun_out/r04b1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for v in 1 1; do
  MIVS_RS_BUCKET_1P=$v bash tools/step_prof.sh r04b1/s$v$RANDOM > /dev/null || exit 12
done
for d in gpurun_out/r04b1/s*; do
  echo "$d: $(head -1 $d/breakdown.txt) | $(grep -o '"candidates": [0-9]*' $d/b.json) $(grep -o '"overflow_queries": [0-9]*' $d/b.json)"
  grep "bucket\|count_lds\|scatter\|k_pf_refine\|stream_off\|k_scan_small\|k_rs_headers" $d/breakdown.txt
done
