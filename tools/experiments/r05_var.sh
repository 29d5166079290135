#!/bin/bash
# K11v variants (variants/libmivs_*.so via MIVS_LIB) under the kernel trace, alternated: per-step kernel times
set -u
O=gpurun_out/${1:-r05var}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name lib
  local nm=$1 lib=$2
  MIVS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/$nm -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $O/$nm.json > $O/$nm.log 2>&1 || return 1
  python3 tools/step_breakdown.py $O/$nm/kt_kernel_trace.csv 3 20 > $O/$nm.txt
  echo "$nm $(grep -E 'k_pf_verify|k_pf_refine' $O/$nm.txt | awk '{print $1, $(NF-1)}' | tr '\n' ' ') $(head -1 $O/$nm.txt)"
}
run v1a variants/libmivs_k11v1.so && run v6a variants/libmivs_k11v6.so && run v8a variants/libmivs_k11v8.so && \
run v1b variants/libmivs_k11v1.so && run v6b variants/libmivs_k11v6.so && run v8b variants/libmivs_k11v8.so
