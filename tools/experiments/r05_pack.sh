#!/bin/bash
# the -m gpu suite, then the default bench's main line (build roofline: the pack kernel)
set -u
O=gpurun_out/${1:-r05pk}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05pk} || exit 11
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --sweep "" --flat-rows 0 --pq-rows 0 \
  --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $O/bench.json > $O/bench.log 2>&1 || exit 12
python3 -c "
import json
b=json.load(open('$O/bench.json'))
print(b['value'], b['ms_per_step'], b['build_s'], b['build_vectors_per_s'])
for k,v in b['build_roofline'].items():
    if isinstance(v,dict): print(k, v['ms_per_launch'], v['frac'])
"
