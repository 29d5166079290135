#!/bin/bash
# PMC passes over the K10 pre-filter scan (one rocprofv3 run per counter group)
set -u
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_pf_scan -f csv -d $OUT/fetch -o pmc -- $B > $OUT/fetch.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_pf_scan -f csv -d $OUT/write -o pmc -- $B > $OUT/write.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_pf_scan -f csv -d $OUT/tcc -o pmc -- $B > $OUT/tcc.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex k_pf_scan -f csv -d $OUT/sq -o pmc -- $B > $OUT/sq.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex k_pf_scan -f csv -d $OUT/sq2 -o pmc -- $B > $OUT/sq2.log 2>&1 || exit 15
exit 0
