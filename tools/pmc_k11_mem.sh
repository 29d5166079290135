#!/bin/bash
# memory-side PMC of the final K11 (k_pf_refine) at the bench shape: L2 hits / misses, L1 -> L2 reads, HBM fetch
set -u
OUT=gpurun_out/${1:-pmck11}
KRE=${KRE:-k_pf_refine}
mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() {  # name, counters...
  local nm=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d $OUT/$nm -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 > $OUT/$nm.log 2>&1
}
run_pmc tcc TCC_HIT_sum TCC_MISS_sum || exit 11
run_pmc tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 12
run_pmc fetch FETCH_SIZE || exit 13
run_pmc clk SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 14
echo done
