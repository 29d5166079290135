#!/bin/bash
# Brute force (configs[1], 1M x 768, 10k queries, k 10): K10 variants by engine switch, alternating
set -u
OUT=gpurun_out/${1:-flatv}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in default MIVS_PF_PAIR=0 MIVS_PF_REG=1; do
    if [ "$v" = default ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 300 python3 tools/bench_flat.py --reps 10 > $OUT/f_${v}_$r.json 2> $OUT/f_${v}_$r.log || exit $?
    echo "$r $v $(tail -1 $OUT/f_${v}_$r.json | cut -c1-300)"
  done
done
