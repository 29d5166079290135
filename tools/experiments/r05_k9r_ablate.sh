#!/bin/bash
# K9r ablation at the configs[4] share: MIVS_PQ_FLAGS 1 = skip the LUT builds, 2 = skip the LUT reads (scan),
# 3 = both; the launch times of the plain search (fp32 and fp16 LUT) from bench.py's PQ side line
set -u
O=gpurun_out/k9r_ablate
mkdir -p $O
for f in 0 1 2 3; do
  MIVS_PQ_FLAGS=$f timeout -k 10 300 python3 -u bench.py --sweep "" --latency "" --batch-sweep "" --large-k "" \
    --flat-rows 0 --no-cpu-baseline --single-process 0 --json-out $O/f$f.json > $O/f$f.log 2>&1 || exit 1
  python3 -c "
import json; d = json.load(open('$O/f$f.json'))['ivf_pq_12m5']
print('flags $f', 'fp32 K9r', d['roofline']['launch_ms'], 'ms; fp16 K9r', d['lut_fp16']['roofline']['launch_ms'], 'ms')"
done
