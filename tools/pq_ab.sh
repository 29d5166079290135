#!/bin/bash
# A/B of two libmivs builds on the IVF-PQ side line alone (MIVS_LIB selects the library), alternated, each run under
# rocprofv3 --kernel-trace --stats; prints the [pq] lines and the K9r averages per run.
# Usage: bash tools/pq_ab.sh TAG LIB_A LIB_B [REPS]
set -u
TAG=$1; A=$2; B=$3; REPS=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $REPS); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MIVS_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/${v}$r -o kt -- python3 bench.py --rows 1000000 \
      --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --large-k "" --single-process 0 \
      --latency "" --batch-sweep "" --build-warmup 0 > $OUT/${v}$r.log 2>&1 || { echo "run $v$r failed"; tail -3 $OUT/${v}$r.log; exit 2; }
    echo "== $v rep $r ($lib)"; grep "\[pq\]" $OUT/${v}$r.log
    find $OUT/${v}$r -name "*kernel_stats.csv" -exec grep -h "pq_scan_rt" {} \; | cut -d, -f1,2,4
  done
done
