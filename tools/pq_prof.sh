#!/bin/bash
# kernel stats of the IVF-PQ bench (plain + refined at n_probes 16, 100 candidates)
set -u
O=gpurun_out/${1:-pqprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 -u tools/bench_ivf_pq.py --sweep 16 --refine-ratios 10 --gt-queries 64 > $O/b.log 2>&1 || exit 1
head -25 $O/kt/kt_kernel_stats.csv | cut -d, -f1-4
