#!/usr/bin/env python3
"""Print per-dispatch means of every counter under gpurun_out/<tag>/*/pmc_counter_collection.csv."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
for path in sorted(glob.glob(f"gpurun_out/{tag}/*/pmc_counter_collection.csv")):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(path)):
        vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ms = sum(dur.values()) / len(dur)
    print(f"{path.split('/')[-2]:6s} ({len(dur)} dispatches, {ms:.2f} ms):",
          ", ".join(f"{k}={sum(v.values()) / len(v):.4g}" for k, v in sorted(vals.items())))
