#!/bin/bash
# final-tree profiles: the default bench under rocprofv3 --kernel-trace --stats (every line), the main line alone
# under the same, then the K13 PMC passes
set -u
O=gpurun_out/${1:-r05final4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o prof -- python3 bench.py --json-out $O/bench_prof.json > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 11; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/profm -o prof -- python3 bench.py --steps 20 --warmup 3 \
  --no-cpu-baseline --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" \
  --json-out $O/bench_main.json > $O/bench_main.log 2>&1 || { tail -20 $O/bench_main.log; exit 12; }
bash tools/pmc_k13_passes.sh ${1:-r05final4}_pmc || exit 13
