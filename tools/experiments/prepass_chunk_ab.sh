#!/bin/bash
# K13 pre-pass work-item size: MIVS_PF_CHUNK_ROWS (K10 rows per item; the pre-pass samples are ~2.4k rows, so
# the default 16384 gives one item per list) -- step time and the pre-pass kernels per value.
set -u
OUT=gpurun_out/${1:-pcab}
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VALUES:-16384 2048 1024 512}; do
  MIVS_PF_CHUNK_ROWS=$v timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --gt-queries 500 --sweep "" --flat-rows 0 --pq-rows 0 --json-out $OUT/b$v.json > $OUT/b$v.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/b$v.json'));s=j['search_stats'];print('rows $v', round(j['value']), j['ms_per_step'], j['roofline']['launch_ms'], j['recall_at_10'], 'cand', s['candidates'])"
  MIVS_PF_CHUNK_ROWS=$v timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/kt$v -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/kt$v.log 2>&1 || exit $?
  python3 tools/step_breakdown.py $OUT/kt$v/kt_kernel_trace.csv 3 10 > $OUT/bd$v.txt || exit $?
  grep -E "window|k_pf_scan|k_pf_refine|k_rs_scan" $OUT/bd$v.txt
done
