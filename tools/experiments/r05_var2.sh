#!/bin/bash
# variants (variants/libmivs_*.so via MIVS_LIB) under the kernel trace, alternated: per-step kernel times
set -u
O=gpurun_out/${1:-r05var2}
shift
mkdir -p $O
export TMPDIR=/tmp
run() {  # name lib
  local nm=$1 lib=$2
  MIVS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/$nm -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $O/$nm.json > $O/$nm.log 2>&1 || return 1
  python3 tools/step_breakdown.py $O/$nm/kt_kernel_trace.csv 3 20 > $O/$nm.txt
  echo "$nm $(grep -E "$KRE" $O/$nm.txt | awk '{print $1, $(NF-1)}' | tr '\n' ' ') $(head -1 $O/$nm.txt)"
}
for r in a b; do
  for v in "$@"; do run $v$r variants/libmivs_$v.so || exit 1; done
done
