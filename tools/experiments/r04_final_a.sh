#!/bin/bash
# Round-end evidence, part 1: every -m gpu test, then the default bench unprofiled
set -u
O=gpurun_out/r04final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 11; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 12; }
tail -1 $O/bench.log | cut -c1-600
