#!/bin/bash
# build variants (variants/libmivs_*.so via MIVS_LIB), alternated: build time and build_roofline per kernel
set -u
O=gpurun_out/${1:-r05varb}
shift
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  for v in "$@"; do
    MIVS_LIB=variants/libmivs_$v.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gt-queries 16 \
      --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" \
      --json-out $O/$v$r.json > $O/$v$r.log 2>&1 || exit 1
    python3 -c "
import json
b=json.load(open('$O/$v$r.json'))
print('$v$r', 'build_s', b['build_s'], 'step', b['ms_per_step'], ' '.join(f\"{k}={v['ms_per_launch']}\" for k,v in b['build_roofline'].items() if isinstance(v,dict)))
"
  done
done
