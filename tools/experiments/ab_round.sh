#!/bin/bash
# GPU tests, then a quick A/B bench over env assignments (tools/quick_bench.sh). Usage: QTAG=x bash tools/ab_round.sh "ENV=1" ...
set -u
OUT=gpurun_out/${QTAG:-quick}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/quick_bench.sh "$@"
