"""Per-search kernel time of tools/lk_bench.py's timed searches from a rocprofv3 kernel trace: the window from the
end of the warm search's k_lk_sort to the end of the last one, kernel durations summed by name / reps.
Usage: python tools/lk_breakdown.py kt_kernel_trace.csv [reps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [r for r in rows if "k_lk_sort" in r["Kernel_Name"]]
t0 = int(ends[-R - 1]["End_Timestamp"])
t1 = int(ends[-1]["End_Timestamp"])
acc = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and e <= t1:
        n = r["Kernel_Name"].replace("void ", "").replace("mivs::(anonymous namespace)::", "").split("(")[0]
        acc[n] += (e - s) / 1e6
        cnt[n] += 1
busy = sum(acc.values())
print(f"window {(t1 - t0) / 1e6 / R:.3f} ms per search, kernels busy {busy / R:.3f} ms per search")
for n, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {n[:70]:70s} {cnt[n] / R:5.1f} launches {v / R * 1e3:9.1f} us")
