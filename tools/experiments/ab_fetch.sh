#!/bin/bash
# A/B of env assignments: quick bench each, then a FETCH_SIZE pass over the K10 launches of each.
# Usage: QTAG=x bash tools/ab_fetch.sh "ENV=1" "ENV=0" ...
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${QTAG:-abf}
mkdir -p $OUT
bash tools/quick_bench.sh "$@" || exit $?
i=0
for e in "$@"; do
  env $e timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_pf_scan<" -f csv -d $OUT/f$i -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gt-queries 16 > $OUT/f$i.log 2>&1 || exit $?
  python3 - "$e" $OUT/f$i/pmc_counter_collection.csv <<'PY' | tee -a $OUT/summary.txt
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[2])) if r.get("Counter_Name") == "FETCH_SIZE" and "k_pf_scan<" in r.get("Kernel_Name", "")]
by = {}
for r in rows: by.setdefault(r["Dispatch_Id"], 0.0); by[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = sorted(by.values())
print(sys.argv[1], "fetch GB/launch (x2 corrected):", [round(x * 1024 * 2 / 1e9, 2) for x in v])
PY
  i=$((i+1))
done
