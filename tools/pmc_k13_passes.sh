#!/bin/bash
# PMC passes over K13 (k_rs_scan) at the default bench shape, one counter group per run (each its own
# time limit); summarised on the CPU by tools/pmc_k13_summary.py
set -u
OUT=gpurun_out/${1:-pmc13}
KRE=${KRE:-k_rs_scan}
mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() {  # name, counters...
  local nm=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d $OUT/$nm -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" --batch-sweep "" > $OUT/$nm.log 2>&1
}
run_pmc fetch FETCH_SIZE || exit 11
run_pmc write WRITE_SIZE || exit 12
run_pmc dram TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || exit 13
run_pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit 14
echo "pmc passes done"
