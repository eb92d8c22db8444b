"""Summarise a rocprofv3 kernel trace of tools/ip_time.py: hole-fill kernels of the last call.

usage: python tools/ip_prof_summary.py <rocprof output dir>
"""
import csv
import sys

d = sys.argv[1]
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
ip = [r for r in tr if "ip_" in r["Kernel_Name"]]
calls = [i for i, r in enumerate(ip) if "ip_prep" in r["Kernel_Name"]]
last = ip[calls[-1]:]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
busy = sum(dur(r) for r in last)
print(f"last call: span {span:.0f} us over {len(last)} launches, kernels {busy:.0f} us, gaps {span - busy:.0f} us")
for name in ("prep", "cols", "rows", "hist", "scan", "scatter", "ring_layer", "negate", "hole_layer", "hole_tail"):
    t = [dur(r) for r in last if any(f"ip_{name}{suf}_kernel" in r["Kernel_Name"] for suf in ("", "4", "_reg"))]
    if t:
        print(f"  {name:10s} {sum(t):8.1f} us ({len(t)} launches, median {sorted(t)[len(t) // 2]:.1f})")
hl = [dur(r) for r in last if "hole_layer" in r["Kernel_Name"]]
if hl:
    print("  hole layers in order (us): " + " ".join(f"{x:.0f}" for x in hl[:12]) + " ... " +
          " ".join(f"{x:.0f}" for x in hl[-8:]))
    for lo, hi in ((0, 10), (10, 20), (20, 40), (40, 100), (100, 1e9)):
        sel = [x for x in hl if lo <= x < hi]
        print(f"    {lo:>5}-{hi:<5} us: {len(sel):4d} layers, {sum(sel):8.1f} us")
