#!/bin/bash
# round 5: staggered K13 -- the stagger parity suite, the engine switches, then an alternating A/B of the bench
set -u
O=gpurun_out/${1:-r05k13}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_k13_stagger.py \
  tests/test_gpu_engine_switches.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -3 $O/tests.log
bash tools/ab_env.sh ${1:-r05k13}/ab ${2:-2} "MIVS_RS_STAGGER=0" "" || exit 12
