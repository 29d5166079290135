#!/bin/bash
# PMC passes over the pre-filter scan kernel (one rocprofv3 run per counter group); KRE = kernel regex
set -u
OUT=gpurun_out/${1:-pmc}
KRE=${KRE:-k_pf_scan}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex "$KRE" -f csv -d $OUT/sq -o pmc -- $B > $OUT/sq.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex "$KRE" -f csv -d $OUT/sq2 -o pmc -- $B > $OUT/sq2.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "$KRE" -f csv -d $OUT/ta -o pmc -- $B > $OUT/ta.log 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY --kernel-include-regex "$KRE" -f csv -d $OUT/mf -o pmc -- $B > $OUT/mf.log 2>&1 || echo "mf pass failed"
exit 0
