"""Per-layer hole counts (OFD_IP_DEBUG stderr of the last call) next to the
hole-layer kernel durations of a rocprofv3 kernel trace of tools/ip_time.py.
usage: python tools/ip_layers.py <stderr log> <trace dir>"""
import csv
import sys

lines = [l.split() for l in open(sys.argv[1]) if l.startswith("ip layer")]
# the last call's layers: the layer index restarts at 1 per call
starts = [i for i, l in enumerate(lines) if l[2] == "1"]
last = lines[starts[-1]:]
tr = list(csv.DictReader(open(f"{sys.argv[2]}/run_kernel_trace.csv")))
hl = [r for r in tr if "hole_" in r["Kernel_Name"]]
hl = hl[-len(last):]
rows = []
for l, r in zip(last, hl):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows.append((int(l[2]), int(l[4]), int(l[6]), d, r["Kernel_Name"].split("(")[0][-24:]))
tot = sum(r[3] for r in rows)
print(f"{len(rows)} layers, {tot:.0f} us")
for r in rows[:12] + rows[12::20]:
    print(f"L={r[0]:4d} interior={r[1]:8d} other={r[2]:7d} dur={r[3]:8.1f} us {r[4]}")
import statistics
for lo, hi in ((0, 1000), (1000, 5000), (5000, 20000), (20000, 50000), (50000, 10**9)):
    ds = [r[3] for r in rows if lo <= r[1] + r[2] < hi]
    if ds:
        print(f"holes in [{lo},{hi}): {len(ds)} layers, median {statistics.median(ds):.1f} us, sum {sum(ds):.0f} us")
