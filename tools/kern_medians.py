"""Median / sum of durations per kernel name in a rocprofv3 kernel trace (last N dispatches of each).
usage: python tools/kern_medians.py <trace dir> [substr]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
key = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if key in n:
        short = n.split("::")[1].split("(")[0] if "::" in n else n[:40]
        d[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:40s} n={len(v):6d} sum={sum(v):10.1f} us median={statistics.median(v):8.1f} min={min(v):7.1f} max={max(v):8.1f}")
