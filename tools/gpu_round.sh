#!/bin/bash
# One GPU-box session: parity tests, then the default bench under rocprofv3 kernel-trace,
# then two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the fine-scan kernel.
# Usage: bash tools/gpu_round.sh TAG
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python3 bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_scan<16' -f csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 > $OUT/pmc_fetch.log 2>&1 || exit $?
  timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_scan<16' -f csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 > $OUT/pmc_write.log 2>&1 || exit $?
fi
[ "${MICRO:-0}" = "1" ] && { timeout -k 10 300 python3 tools/scan_microbench.py > $OUT/micro.log 2>&1 || exit $?; }
exit $rc
