#!/bin/bash
# round 5: staggered K13 A/B (round-4 kernel, staggered default, staggered with one-item segments, round-4 kernel with
# the reloads skipped), the K10 path's small-batch latency, and K13's fabric traffic with the staggered kernel
set -u
O=gpurun_out/${1:-r05k13b}
mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_env.sh ${1:-r05k13b}/ab 1 "MIVS_RS_STAGGER=0" "" "MIVS_RS_STAGGER=2" "MIVS_RS_STAGGER=0 MIVS_RS_FLAGS=4" \
  "MIVS_PF_ROWSTAT=0" || exit 12
for v in 1 2 3 4 5; do grep "\[latency\]" $O/ab/v${v}_1.log | sed "s/^/v$v /"; done
KRE=k_rs_scan timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rs_scan -f csv -d $O/fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --pq-rows 0 --large-k "" --single-process 0 --latency "" > $O/fetch.log 2>&1 || exit 13
echo pmc done
