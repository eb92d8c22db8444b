"""Summarise a rocprofv3 kernel-trace CSV: per-kernel count/avg/min/max (us) for
the engine's kernels, plus per-call timeline of the last N dispatches."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows = list(csv.DictReader(open(path)))
ours = [r for r in rows if "anonymous namespace)::" in r["Kernel_Name"] and "at::" not in r["Kernel_Name"]]
agg = defaultdict(list)
for r in ours:
    name = r["Kernel_Name"].split("::")[1].split("(")[0].split("<")[0]
    agg[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in agg.items():
    print(f"{k:28s} n={len(v):4d} avg={sum(v)/len(v):8.1f} min={min(v):8.1f} max={max(v):8.1f} us")
tl = ours[-last:]
t0 = int(tl[0]["Start_Timestamp"])
for r in tl:
    name = r["Kernel_Name"].split("::")[1].split("(")[0].split("<")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {name:24s} start={(s-t0)/1000:9.1f} dur={(e-s)/1000:7.1f}")
