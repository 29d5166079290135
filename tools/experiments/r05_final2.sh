#!/bin/bash
# round-5 final evidence, part 2: rocprofv3 --kernel-trace --stats of the main line alone (side lines off, so
# K13's average is the timed launches' own), then the K13 PMC passes (FETCH_SIZE / WRITE_SIZE / DRAM / SQ)
set -u
O=gpurun_out/${1:-r05final2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 bench.py --steps 20 --warmup 3 \
  --no-cpu-baseline --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" \
  --json-out $O/bench_main.json > $O/bench_main.log 2>&1 || { tail -20 $O/bench_main.log; exit 11; }
grep -E "k_rs_scan|k_as_scan" $O/prof/prof_kernel_stats.csv | cut -d, -f1-4
bash tools/pmc_k13_passes.sh ${1:-r05final2}_pmc || exit 12
