#!/bin/bash
# K13 timing experiments: the short bench under MIVS_RS_FLAGS variants (1 no epilogue, 2 no staging, 3 both)
set -u
OUT=gpurun_out/${1:-k13ab}
mkdir -p $OUT
export TMPDIR=/tmp
for f in 0 1 2 3; do
  MIVS_RS_FLAGS=$f timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --json-out $OUT/f$f.json > $OUT/f$f.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/f$f.json'));s=j['search_stats'];print('flags=$f', 'step_ms', j['ms_per_step'], 'scan_ms', j['roofline']['launch_ms'], 'rec', j['recall_at_10'], 'ovf', s['overflow_queries'], 'cand', s['candidates'], 'cand_ovf', s['cand_overflow'])" | tee -a $OUT/summary.txt
done
