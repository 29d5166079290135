#!/bin/bash
# the -m gpu suite with the device block cache, then three bench main lines (build time, phases, index footprint)
set -u
O=gpurun_out/${1:-r05cache}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests.sh ${1:-r05cache} || exit 11
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 \
    --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" --json-out $O/b$r.json > $O/b$r.log 2>&1 || exit 12
  python3 -c "
import json
b=json.load(open('$O/b$r.json'))
print('run $r build_s', b['build_s'], b['build_phases_s'], 'index', b['index_memory']['total_bytes'], 'step', b['ms_per_step'])
"
done
