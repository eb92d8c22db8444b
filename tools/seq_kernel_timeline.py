"""Kernel timeline of the last sequential fill in a rocprofv3 kernel trace of
tools/seq_time.py (or any run whose last FMM launch is the fill's):
  rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/seq_time.py 64
  python tools/seq_kernel_timeline.py DIR/.../run_kernel_trace.csv
Prints every kernel from the last sq_prep_tile_kernel on, relative to its start
(us), with its duration."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "sq_prep_tile_kernel" in r["Kernel_Name"]]
i0 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
end = 0
for r in rows[i0:]:
    n = r["Kernel_Name"]
    if not n.split("(")[0].split("::")[-1].startswith(("sq_", "void (anonymous namespace)::sq_")) and "sq_" not in n:
        continue
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    end = max(end, e)
    short = n.split("(")[0].replace("(anonymous namespace)::", "").replace("void ", "")
    if "sq_colour3df" in n:
        short = "sq_colour3df"
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {short}")
print(f"fill: {end / 1e3:.1f} us from PREP's start")
