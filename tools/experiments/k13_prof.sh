#!/bin/bash
# K13 profile: timing experiments (MIVS_RS_FLAGS), a kernel-trace --stats pass of the short bench, and SQ PMC
set -u
OUT=gpurun_out/${1:-k13prof}
mkdir -p $OUT
export TMPDIR=/tmp
for f in 0 1 3; do
  MIVS_RS_FLAGS=$f timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --json-out $OUT/f$f.json > $OUT/f$f.log 2>&1 || exit $?
  python3 -c "import json;j=json.load(open('$OUT/f$f.json'));s=j['search_stats'];print('flags=$f', 'step_ms', j['ms_per_step'], 'scan_ms', j['roofline']['launch_ms'], 'rec', j['recall_at_10'], 'ovf', s['overflow_queries'], 'cand', s['candidates'], 'cand_ovf', s['cand_overflow'])" | tee -a $OUT/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 bench.py --steps 10 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 > $OUT/kt.log 2>&1 || exit $?
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep '' --flat-rows 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex k_rs_scan -f csv -d $OUT/sq -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 > $OUT/sq.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum --kernel-include-regex k_rs_scan -f csv -d $OUT/ta -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 > $OUT/ta.log 2>&1 || exit 15
python3 tools/pmc_print.py ${1:-k13prof} | tee -a $OUT/summary.txt
