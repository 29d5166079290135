#!/bin/bash
# the IVF-PQ side line (fp32 and opt-in fp16 LUT) under rocprofv3 --kernel-trace --stats: K9r's fp32
# (k_pq_scan_rt<.., false>) and fp16 (<.., true>) launches average separately
set -u
O=gpurun_out/${1:-r05pq16}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 -u bench.py --sweep "" --latency "" \
  --batch-sweep "" --large-k "" --flat-rows 0 --no-cpu-baseline --single-process 0 --json-out $O/b.json > $O/b.log 2>&1 || exit 12
rm -f $O/kt/kt_kernel_trace.csv
grep "k_pq_scan_rt" $O/kt/kt_kernel_stats.csv | cut -d, -f1-4
grep "\[pq\]" $O/b.log
