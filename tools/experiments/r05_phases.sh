#!/bin/bash
# K13 block spans (MIVS_RS_FLAGS=8) and phase clocks (16) on the default bench shape
set -u
O=gpurun_out/${1:-r05ph}
mkdir -p $O
export TMPDIR=/tmp
for f in 8 16; do
  MIVS_RS_FLAGS=$f timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" \
    --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" > $O/f$f.log 2>&1 || exit 11
  grep "k13" $O/f$f.log | tail -4
done
