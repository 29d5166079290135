#!/bin/bash
# -m gpu tests on the box, one pytest process, per-test timeout; log under gpurun_out/TAG.
# Usage: bash tools/gpu_tests.sh TAG [pytest selection args...]
set -u
TAG=${1:-gpu}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu -v -x --timeout 400 --timeout-method thread "${@:-tests}" > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
tail -5 $OUT/tests.log
exit $rc
