#!/bin/bash
# PMC passes over one kernel (KRE regex) at the default bench shape (no side lines): wave-cycle split and
# instruction mix. Usage: KRE=k_pf_refine bash tools/pmc_kernel.sh <out name>
set -u
OUT=gpurun_out/${1:-pmck}
KRE=${KRE:-k_pf_refine}
mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() {  # name, counters...
  local nm=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d $OUT/$nm -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 > $OUT/$nm.log 2>&1
}
run_pmc clk SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 11
run_pmc ins SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU || exit 12
echo "pmc kernel passes done"
