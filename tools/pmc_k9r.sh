#!/bin/bash
# PMC passes over K9r (k_pq_scan_rt) on the IVF-PQ bench shape (12.5M x 768 fp16, n_probes 16, k 10)
# Usage: bash tools/pmc_k9r.sh TAG [float32|float16]   (the LUT dtype)
set -u
OUT=gpurun_out/${1:-pmck9r}
LUT=${2:-float32}
mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() {  # name, counters...
  local nm=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "k_pq_scan_rt" -f csv -d $OUT/$nm -o pmc -- python3 tools/bench_ivf_pq.py --sweep 16 --refine-ratios "" --gt-queries 16 --lut-dtype $LUT > $OUT/$nm.log 2>&1
}
run_pmc clk SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 11
run_pmc lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH || exit 12
echo "pmc k9r passes done"
