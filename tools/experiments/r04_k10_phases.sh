#!/bin/bash
# K10 phase clocks of the fp8 pre-pass at the bench shape (MIVS_PF_FLAGS=32; stderr lines "[k10 phases]")
set -u
O=gpurun_out/r04k10
mkdir -p $O
MIVS_PF_FLAGS=32 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 > $O/b.log 2>&1 || exit 1
grep "k10 phases" $O/b.log | tail -4
