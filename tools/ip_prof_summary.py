"""Summarise a rocprofv3 kernel trace of tools/ip_time.py: hole-fill kernels of the last call."""
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} n={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:9.1f} us")
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
ip = [r for r in tr if "ip_" in r["Kernel_Name"]]
calls = [i for i, r in enumerate(ip) if "ip_prep" in r["Kernel_Name"]]
last = ip[calls[-1]:]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
hl = [dur(r) for r in last if "hole_layer" in r["Kernel_Name"]]
print(f"last call: span {span:.0f} us, {len(last)} launches, hole layers {len(hl)}: sum {sum(hl):.0f} us, "
      f"first {[round(x) for x in hl[:6]]}, median {sorted(hl)[len(hl) // 2]:.1f} us")
for name in ("prep", "cols", "rows", "hist", "scan", "scatter", "ring_layer", "negate"):
    t = [dur(r) for r in last if f"ip_{name}_kernel" in r["Kernel_Name"] or f"ip_{name}4_kernel" in r["Kernel_Name"]
         or f"ip_{name}_reg_kernel" in r["Kernel_Name"]]
    if t:
        print(f"  {name:10s} {sum(t):8.1f} us ({len(t)} launches)")
