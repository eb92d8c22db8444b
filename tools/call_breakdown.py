"""Per-call breakdown of a rocprofv3 kernel trace of repeated warp calls.

usage: python tools/call_breakdown.py <kernel_trace.csv>

Groups consecutive bin_kernel -> splat launches into calls, splits the trace
into runs of similar calls (a pause of > 1 ms between calls starts a new
group) and prints per group the median BIN and SPLAT durations, the gap
BIN end -> SPLAT start, the gap SPLAT end -> next BIN start, and the call
period (BIN start to next BIN start).
"""
import csv
import statistics as st
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        if "bin_kernel" in n or "splat" in n or "row_kernel" in n:
            kind = "bin" if "bin_kernel" in n else "splat"
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, n))
    ks.sort()
    calls = []
    i = 0
    while i + 1 < len(ks):
        if ks[i][2] == "bin" and ks[i + 1][2] == "splat":
            calls.append((ks[i], ks[i + 1]))
            i += 2
        else:
            i += 1
    groups, cur = [], []
    for c in calls:
        if cur and c[0][0] - cur[-1][1][1] > 1_000_000:
            groups.append(cur)
            cur = []
        cur.append(c)
    if cur:
        groups.append(cur)
    for g in groups:
        binu = [(b[1] - b[0]) / 1e3 for b, s in g]
        spl = [(s[1] - s[0]) / 1e3 for b, s in g]
        gap1 = [(s[0] - b[1]) / 1e3 for b, s in g]
        gap2 = [(g[k + 1][0][0] - g[k][1][1]) / 1e3 for k in range(len(g) - 1)]
        per = [(g[k + 1][0][0] - g[k][0][0]) / 1e3 for k in range(len(g) - 1)]
        name = g[0][1][3].split("(")[0][-60:]
        print(f"{len(g):4d} calls  BIN {st.median(binu):7.1f}  BIN->SPLAT gap {st.median(gap1):5.1f}  "
              f"SPLAT {st.median(spl):7.1f}  SPLAT->next BIN {st.median(gap2) if gap2 else 0:5.1f}  "
              f"period {st.median(per) if per else 0:7.1f} us   [{name}]")


if __name__ == "__main__":
    main()
