"""Per-step kernel time of the timed search steps from a rocprofv3 kernel trace of
`bench.py --warmup W --steps K ...`: the window from the end of the W-th K13 (fine scan) launch to the end
of the (W+K)-th, kernel durations summed by name and divided by K.
Usage: python tools/step_breakdown.py kt_kernel_trace.csv [W K]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
scan = [r for r in rows if "k_rs_scan" in r["Kernel_Name"]]
t0 = int(scan[W - 1]["End_Timestamp"])
t1 = int(scan[W + K - 1]["End_Timestamp"])
acc = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and e <= t1:
        n = r["Kernel_Name"].replace("void ", "").replace("mivs::(anonymous namespace)::", "").split("(")[0]
        acc[n] += (e - s) / 1e6
        cnt[n] += 1
busy = sum(acc.values())
print(f"window {(t1 - t0) / 1e6 / K:.3f} ms per step, kernels busy {busy / K:.3f} ms per step")
for n, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {n[:60]:60s} {cnt[n] / K:5.1f} launches {v / K * 1e3:9.1f} us")
