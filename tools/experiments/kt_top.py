"""Top kernels of a rocprofv3 --kernel-trace --stats csv: calls, average and total duration."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:n]:
    print(f"{x['Name'][:72]:72s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:10.1f} us {float(x['TotalDurationNs']) / 1e6:9.2f} ms")
