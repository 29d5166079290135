#!/bin/bash
# Round-2 evidence for the default search path (K13): PMC passes over k_rs_scan (FETCH_SIZE, WRITE_SIZE,
# DRAM-side read requests, SQ), the default bench under --kernel-trace --stats, and the default bench.
set -u
OUT=gpurun_out/${1:-pmc13}
KRE=${KRE:-k_rs_scan}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep '' --flat-rows 0"
run_pmc() {  # name, counters...
  local nm=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d $OUT/$nm -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 > $OUT/$nm.log 2>&1
}
run_pmc fetch FETCH_SIZE || exit 11
run_pmc write WRITE_SIZE || exit 12
run_pmc dram TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || exit 13
run_pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit 14
run_pmc mf SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE GRBM_COUNT || exit 15
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 bench.py --no-cpu-baseline --json-out $OUT/bench_kt.json > $OUT/kt.log 2>&1 || exit 16
timeout -k 10 600 python3 bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || exit 17
tail -1 $OUT/bench.log
