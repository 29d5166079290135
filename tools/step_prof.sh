#!/bin/bash
# kernel trace of the search step only (no side lines) -> per-step kernel breakdown
set -u
OUT=gpurun_out/${1:-stepprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $OUT/b.json > $OUT/b.log 2>&1 || exit $?
python3 tools/step_breakdown.py $OUT/kt/kt_kernel_trace.csv 3 20 | tee $OUT/breakdown.txt
