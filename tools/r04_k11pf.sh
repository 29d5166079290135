#!/bin/bash
# K11 window-row prefetch (MIVS_PF_REFINE_PREFETCH) and the probe map's chunk (MIVS_PM_CHUNK): the switch tests, then
# step breakdowns
set -u
O=gpurun_out/r04k11pf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine_switches.py tests/test_gpu_prefilter.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
run() {  # label, env...
  local d=r04k11pf/$1
  env "${@:2}" bash tools/step_prof.sh $d > /dev/null || exit 12
  echo "$1: $(head -1 gpurun_out/$d/breakdown.txt) | $(grep 'k_pf_refine<0>' gpurun_out/$d/breakdown.txt | awk '{print $NF, $(NF-1)}') | bucket $(grep 'bucket_fused' gpurun_out/$d/breakdown.txt | awk '{print $(NF-1)}') fill $(grep 'k_probe_fill_lds' gpurun_out/$d/breakdown.txt | awk '{print $(NF-1)}') count $(grep 'k_probe_count_lds' gpurun_out/$d/breakdown.txt | awk '{print $(NF-1)}')"
}
run pf1 MIVS_PF_REFINE_PREFETCH=1
run pf0 MIVS_PF_REFINE_PREFETCH=0
run pf1b MIVS_PF_REFINE_PREFETCH=1
run pf0b MIVS_PF_REFINE_PREFETCH=0
run pmc2k MIVS_PM_CHUNK=2048
run pmc1k MIVS_PM_CHUNK=1024
run bs2 MIVS_RS_BUCKET_SPLIT=2
run bs4 MIVS_RS_BUCKET_SPLIT=4
