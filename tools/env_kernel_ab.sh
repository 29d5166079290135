#!/bin/bash
# Alternating runs of one environment variable's values on the default search step, each under rocprofv3
# --kernel-trace --stats; prints ms_per_step and the average duration of the kernels matching PATTERN.
# Usage: bash tools/env_kernel_ab.sh TAG REPS PATTERN VAR VALUE...
set -u
TAG=$1; REPS=$2; PAT=$3; VAR=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $REPS); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/v${v}_$r -o kt -- python3 bench.py \
      --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" \
      --single-process 0 --latency "" --batch-sweep "" --json-out $OUT/v${v}_$r.json > $OUT/v${v}_$r.log 2>&1 \
      || { echo "run $VAR=$v rep $r failed"; tail -3 $OUT/v${v}_$r.log; exit 2; }
    python3 - "$OUT/v${v}_$r" "$PAT" "$VAR=$v" <<'PY'
import csv, glob, json, sys
d, pat, lab = sys.argv[1], sys.argv[2], sys.argv[3]
ms = json.load(open(d + '.json'))['ms_per_step']
ks = []
for r in csv.DictReader(open(glob.glob(d + '/*kernel_stats.csv')[0])):
    if pat in r['Name']:
        ks.append('%s %.1f us' % (r['Name'].split('(')[0].split('::')[-1], float(r['AverageNs']) / 1e3))
print('%s rep %s: %.4f ms/step | %s' % (lab, d.rsplit('_', 1)[-1], ms, '; '.join(ks)))
PY
  done
done
