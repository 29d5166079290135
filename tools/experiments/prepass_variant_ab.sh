#!/bin/bash
# K13 pre-pass (K10 over the nearest-list samples): K10 variants by engine switch, step breakdown of each
set -u
OUT=gpurun_out/${1:-ppv}
mkdir -p $OUT
export TMPDIR=/tmp
for v in default MIVS_PF_PAIR=0 MIVS_PF_CONVOY=0 MIVS_PF_DEPTH=8; do
  if [ "$v" = default ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/kt_$v -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 > $OUT/kt_$v.log 2>&1 || exit $?
  python3 tools/step_breakdown.py $OUT/kt_$v/kt_kernel_trace.csv 3 10 > $OUT/bd_$v.txt || exit $?
  echo "$v"; grep -E "window|k_pf_scan|k_pf_refine" $OUT/bd_$v.txt
done
