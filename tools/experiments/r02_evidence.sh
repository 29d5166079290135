#!/bin/bash
# Round-2 evidence run on one GPU box: the full -m gpu suite, then the default bench under
# rocprofv3 --kernel-trace --stats (kernel averages for profiles/), then the K9r IVF-PQ bench.
# Usage: [TESTS=0|1] [PQ=0|1] bash tools/r02_evidence.sh TAG
set -u
OUT=gpurun_out/${1:-r02ev}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -v -x --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
python3 tools/kt_top.py $OUT/kt/kt_kernel_stats.csv > $OUT/kt_top.txt || exit $?
head -12 $OUT/kt_top.txt
if [ "${PQ:-1}" = "1" ]; then
  timeout -k 10 400 python3 tools/bench_ivf_pq.py --sweep 16,32,64 --refine-ratios 10,20 > $OUT/pq.json 2> $OUT/pq.log || exit $?
  grep -E "build|search|refine" $OUT/pq.log
fi
if [ "${PHASE:-1}" = "1" ]; then
  MIVS_RS_FLAGS=24 timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --gt-queries 200 --sweep "" --flat-rows 0 --json-out $OUT/phase.json > $OUT/phase.log 2>&1 || exit $?
  grep "k13 " $OUT/phase.log | tail -3
fi
exit 0
