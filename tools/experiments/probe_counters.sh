#!/bin/bash
# List the PMC counters this box's rocprofv3 offers (looking for DRAM-side TCC/EA counters), then
# run the -m gpu tests once.
set -u
OUT=gpurun_out/${1:-probe}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "rocprofv3 -L rc=$?" >> $OUT/counters.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo "pytest rc=$?" >> $OUT/tests.log
