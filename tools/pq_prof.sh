#!/bin/bash
# rocprofv3 kernel trace of the IVF-PQ side line alone (configs[4] per-GPU share; the IVF-Flat line on a 1M-row
# corpus so it costs little) -> per-kernel totals of the PQ searches (plain k and refined 12 k)
set -u
OUT=gpurun_out/${1:-pqprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 bench.py --rows 1000000 --steps 2 \
  --warmup 1 --no-cpu-baseline --gt-queries 16 --sweep "" --flat-rows 0 --large-k "" --single-process 0 --latency "" \
  --batch-sweep "" --build-warmup 0 --json-out $OUT/b.json > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 2; }
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:10.1f} us avg {float(r["TotalDurationNs"])/1e6:9.2f} ms total')
PY
grep "\[pq\]" $OUT/b.log
