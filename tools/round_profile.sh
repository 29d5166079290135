#!/bin/bash
# The round's profiles of the bench's main line, each step under its own time limit, stopping at the first failure:
#   1. rocprofv3 --kernel-trace --stats of the IVF-Flat main line (the per-kernel averages behind `roofline.launch_ms`)
#   2. K13 effective-clock PMC passes (tools/pmc_k13_clock.sh) -> profiles-ready JSON with clock_mhz_held
# Usage: bash tools/round_profile.sh TAG     (outputs under gpurun_out/TAG; copy what is judged into profiles/)
set -u
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MAIN="--steps 20 --warmup 3 --no-cpu-baseline --flat-rows 0 --pq-rows 0 --large-k '' --single-process 0 --sweep '' --batch-sweep '' --latency '' --gt-queries 200"
eval timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o main -- python3 bench.py $MAIN \
  --json-out $OUT/main_bench.json > $OUT/trace.log 2>&1 || { echo "trace run failed"; tail -5 $OUT/trace.log; exit 2; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/main_kernel_stats.csv \;
head -6 $OUT/main_kernel_stats.csv
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep '' --flat-rows 0 --pq-rows 0 --large-k '' --single-process 0 --batch-sweep '' --latency ''" bash tools/pmc_k13_clock.sh $TAG/pmc || { echo "pmc passes failed"; exit 3; }
KEY=$(python3 -c "import json;j=json.load(open('$OUT/main_bench.json'));s=j['search_stats'];c=j['config'];print(f\"ivf_flat_n{c['rows_per_gpu']}_d{c['dim']}_q{c['queries']}_l{c['n_lists']}_p{c['n_probes']}_k{c['k']}_t{s['query_tile']}\" + ('_pf' if s['prefilter'] else ''))")
python3 tools/pmc_clock_summary.py $OUT/pmc $OUT/k13_clock.json k_rs_scan "$KEY" > /dev/null
python3 -c "import json;j=json.load(open('$OUT/k13_clock.json'));print('clock MHz', round(j['clock_mhz_held'],1), j['config_key'])"
