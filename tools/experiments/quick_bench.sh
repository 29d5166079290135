#!/bin/bash
# quick A/B: bench (short) for each env assignment given as args, e.g. "MIVS_PF_DEPTH=8" "MIVS_PF_DEPTH=16"
OUT=gpurun_out/${QTAG:-quick}
mkdir -p $OUT
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 || exit 1
  python3 -c "import json;j=json.load(open('$OUT/b$i.json'));print('$e', round(j['value']), j['roofline']['launch_ms'], j['ms_per_step'], j['recall_at_10'], j['search_stats']['overflow_queries'])" | tee -a $OUT/summary.txt
  i=$((i+1))
done
