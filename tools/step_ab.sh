#!/bin/bash
# A/B of two libmivs builds on the default search step alone (MIVS_LIB selects the library), alternated; each run
# under rocprofv3 --kernel-trace --stats. Prints ms_per_step and the per-kernel averages matching PATTERN.
# Usage: bash tools/step_ab.sh TAG LIB_A LIB_B [REPS] [PATTERN]
set -u
TAG=$1; A=$2; B=$3; REPS=${4:-2}; PAT=${5:-k_pf_scan}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $REPS); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MIVS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/${v}$r -o kt -- python3 bench.py \
      --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" \
      --single-process 0 --latency "" --batch-sweep "" --json-out $OUT/${v}$r.json > $OUT/${v}$r.log 2>&1 \
      || { echo "run $v$r failed"; tail -3 $OUT/${v}$r.log; exit 2; }
    echo "== $v rep $r ($lib): $(python3 -c "import json;d=json.load(open('$OUT/${v}$r.json'));print(d['ms_per_step'], 'ms/step', d['recall_at_10'])")"
    find $OUT/${v}$r -name "*kernel_stats.csv" -exec grep -h "$PAT" {} \; | cut -d, -f1,2,4 || true
  done
done
