#!/bin/bash
# K13 (k_rs_scan) issue/wait/clock counters at the default bench shape, one counter group per run (each
# its own time limit): effective clock (GRBM_GUI_ACTIVE), MFMA pipe busy, and the wave-cycle split
# WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES. Summarised by tools/pmc_clock_summary.py.
set -u
OUT=gpurun_out/${1:-pmc13c}
KRE=${KRE:-k_rs_scan}
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep '' --flat-rows 0 --pq-rows 0 --large-k '' --single-process 0 --batch-sweep '' --latency ''"}
mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() {  # name, counters...
  local nm=$1; shift
  eval timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d $OUT/$nm -o pmc -- \
    python3 bench.py $BENCH_ARGS > $OUT/$nm.log 2>&1
}
run_pmc clk SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 11
run_pmc ins SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA || exit 12
echo "pmc clock passes done"
