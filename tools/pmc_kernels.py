"""Per-kernel table from a rocprofv3 kernel trace plus FETCH_SIZE / WRITE_SIZE passes.

usage: python tools/pmc_kernels.py <trace dir> <fetch dir> <write dir>
       python tools/pmc_kernels.py --counters <run_counter_collection.csv> substr [substr ...]

One row per kernel instantiation (full demangled name, shortened): dispatches,
median duration, registers / scratch / LDS from the trace, and per-dispatch
medians of FETCH_SIZE x 2 (the gfx950 half-count of wide reads,
MI355X_MICROARCH.md HBM section) and WRITE_SIZE, in MB, with the implied GB/s.
"""
import collections
import csv
import re
import statistics
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]
    n = n.replace("unsigned short", "bf16").replace("float", "f32").replace("double", "f64")
    return n[:110]


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))  # (name, dispatch) -> counter -> value
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (name, _), v in agg.items():
        for c, x in v.items():
            per[(name, c)].append(x)
    return per


def main_table(trace, fetch, write):
    rows = list(csv.DictReader(open(f"{trace}/run_kernel_trace.csv")))
    dur = collections.defaultdict(list)
    info = {}
    for r in rows:
        n = r["Kernel_Name"]
        dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        info[n] = (r.get("Arch_VGPR_Count", r.get("VGPR_Count", "?")), r.get("Accum_VGPR_Count", "?"),
                   r.get("Scratch_Size", "?"), r.get("LDS_Block_Size", r.get("LDS_Size", "?")))
    fc = counters(f"{fetch}/run_counter_collection.csv")
    wc = counters(f"{write}/run_counter_collection.csv")
    print(f"{'kernel':110s} {'n':>4s} {'med us':>8s} {'vgpr':>5s} {'agpr':>5s} {'scr':>4s} {'lds':>6s} "
          f"{'fetch MB':>9s} {'write MB':>9s} {'GB/s':>7s}")
    for n, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if sum(d) < 50:
            continue
        f = fc.get((n, "FETCH_SIZE"))
        w = wc.get((n, "WRITE_SIZE"))
        fm = 2 * statistics.median(f) * 1024 / 1e6 if f else float("nan")  # counters in KiB
        wm = statistics.median(w) * 1024 / 1e6 if w else float("nan")
        md = statistics.median(d)
        gbs = (fm + wm) * 1e6 / (md * 1e3) if f and w else float("nan")
        v, a, s, l = info[n]
        print(f"{short(n):110s} {len(d):4d} {md:8.1f} {v:>5s} {a:>5s} {s:>4s} {l:>6s} {fm:9.1f} {wm:9.1f} {gbs:7.0f}")


def main_counters(path, keys):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        for k in keys:
            if k in r["Kernel_Name"]:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    for k in keys:
        print(f"{k}: {len(disp[k])} dispatches")
        for c, x in sorted(agg[k].items()):
            print(f"   {c:24s} {x:16.0f}")


if __name__ == "__main__":
    if sys.argv[1] == "--counters":
        main_counters(sys.argv[2], sys.argv[3:])
    else:
        main_table(*sys.argv[1:4])
