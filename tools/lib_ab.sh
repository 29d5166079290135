#!/bin/bash
# Alternating runs of several libmivs builds (MIVS_LIB) on the default search step, each under rocprofv3
# --kernel-trace --stats; prints ms_per_step and the average duration of the kernels matching PATTERN.
# Usage: bash tools/lib_ab.sh TAG REPS PATTERN LIB...
set -u
TAG=$1; REPS=$2; PAT=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $REPS); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    MIVS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/v${i}_$r -o kt -- python3 bench.py \
      --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" \
      --single-process 0 --latency "" --batch-sweep "" --json-out $OUT/v${i}_$r.json > $OUT/v${i}_$r.log 2>&1 \
      || { echo "run v$i rep $r failed"; tail -3 $OUT/v${i}_$r.log; exit 2; }
    python3 - "$OUT/v${i}_$r" "$PAT" "$lib" <<'PY'
import csv, glob, json, sys
d, pat, lib = sys.argv[1], sys.argv[2], sys.argv[3]
ms = json.load(open(d + '.json'))['ms_per_step']
ks = []
for r in csv.DictReader(open(glob.glob(d + '/*kernel_stats.csv')[0])):
    if pat in r['Name']:
        ks.append('%s %.1f us' % (r['Name'].split('(')[0].split('::')[-1], float(r['AverageNs']) / 1e3))
print('%s %s: %.4f ms/step | %s' % (d.split('/')[-1], lib.split('/')[-1], ms, '; '.join(ks)))
PY
  done
done
