#!/bin/bash
# One GPU-box session: parity tests, then the default bench under rocprofv3 kernel-trace,
# then two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the fine-scan kernel and their summary.
# Usage: [PF=0|1] [WIDE=0|1] [PMC=0|1] [MICRO=0|1] [TESTS=0|1] bash tools/gpu_round.sh TAG
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export MIVS_SCAN_WIDE=${WIDE:-1}
export MIVS_PREFILTER=${PF:-1}
if [ "$MIVS_PREFILTER" = "1" ]; then KSUB="k_pf_scan<0"; KRE="k_pf_scan<"; T=64_pf;
elif [ "$MIVS_SCAN_WIDE" = "1" ]; then KSUB="k_scan_wide<12, 0, 4>"; KRE='k_scan_wide<12'; T=64; else KSUB="k_scan<12, 0, 8>"; KRE='k_scan<12'; T=32; fi
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/tests.log
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python3 bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 > $OUT/pmc_fetch.log 2>&1 || exit $?
  timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 > $OUT/pmc_write.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/pmc_fetch/pmc_counter_collection.csv $OUT/pmc_write/pmc_counter_collection.csv "$KSUB" ivf_flat_n10000000_d768_q10000_l1024_p32_k10_t$T $OUT/pmc_summary.json > /dev/null || exit $?
fi
if [ "${MICRO:-0}" = "1" ]; then
  timeout -k 10 400 python3 tools/scan_microbench.py > $OUT/micro.log 2>&1 || exit $?
fi
exit 0
