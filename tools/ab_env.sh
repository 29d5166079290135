#!/bin/bash
# Alternating A/B of environment settings on the default quick bench (IVF-Flat line only).
# Usage: bash tools/ab_env.sh TAG REPS "ENV_A" "ENV_B" ...   (ENV "" = defaults); prints value / K13 ms per run
set -u
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
QB="--steps 10 --warmup 2 --no-cpu-baseline --sweep '' --flat-rows 0 --pq-rows 0 --large-k '' --single-process 0 --gt-queries 200 --latency '' --batch-sweep ''"
for r in $(seq 1 $REPS); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    eval env $e timeout -k 10 300 python -u bench.py $QB --json-out $OUT/v${i}_$r.json > $OUT/v${i}_$r.log 2>&1 || { echo "run v$i failed"; tail -3 $OUT/v${i}_$r.log; exit 3; }
    python3 -c "import json;j=json.load(open('$OUT/v${i}_$r.json'));r=j['roofline'];print('v$i [$e] rep $r: value',j['value'],'ms',j['ms_per_step'],'k13',r['launch_ms'],'frac',r['frac'],'cand',j['search_stats']['candidates'],'ovf',j['search_stats']['overflow_queries'])"
  done
done
