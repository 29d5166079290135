#!/bin/bash
# K13 phase ablation (timing experiments only; results are not valid with flags 1/2):
# MIVS_RS_FLAGS 16 = phase clocks; +1 skip the epilogue; +2 skip the tile staging (stale LDS tiles).
set -u
OUT=gpurun_out/${1:-k13abl}
mkdir -p $OUT
export TMPDIR=/tmp
for f in ${FLAGS:-0 1 3 16 17 19}; do
  MIVS_RS_FLAGS=$f timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/f$f.json > $OUT/f$f.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/f$f.json'));print('flags=$f', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'])"
  grep "k13 phases" $OUT/f$f.log | tail -2
done
