"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) for the engine's kernels.

Usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <trace_dir> <B> <C> <H> <W> [out.json]

Takes the LAST step's dispatches (BIN, SPLAT, RESOLVE of one call), applies the
gfx950 correction from MI355X_MICROARCH.md ("FETCH_SIZE reports exactly half of
the bytes of a wide coalesced streaming read": x2), reports per-kernel and
per-step HBM bytes, and writes the JSON bench.py folds into its roofline line.
"""
import csv
import json
import sys
from collections import OrderedDict


WARP_KERNELS = ("bin_kernel", "splat_persist_kernel", "splat_kernel", "resolve2d_kernel", "splat_atomic_kernel",
                "resolve_atomic_kernel")


def per_dispatch(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    out = OrderedDict()
    for r in rows:
        name = r["Kernel_Name"]
        if "anonymous namespace)::" not in name or "at::" in name:
            continue
        if not any(k in name for k in WARP_KERNELS):  # the warp's kernels only
            continue
        k = r["Dispatch_Id"]
        short = name.split("::")[1].split("(")[0].split("<")[0]
        if k not in out:
            out[k] = [short, 0.0, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3]
        out[k][1] += float(r["Counter_Value"])
    return list(out.values())


def main():
    fd, wd, td = sys.argv[1:4]
    B, C, H, W = (int(x) for x in sys.argv[4:8])
    dst = sys.argv[8] if len(sys.argv) > 8 else None
    f = per_dispatch(fd)
    w = per_dispatch(wd)
    names = [x[0] for x in f]
    # launches per call: BIN + SPLAT (tile), + RESOLVE (split), or the atomic pair
    per_call = len(set(names))
    f, w = f[-per_call:], w[-per_call:]
    engine = ("split" if "resolve2d_kernel" in names else "tile" if "bin_kernel" in names else "atomic")
    rep = {"config": [B, C, H, W], "engine": engine, "kernels": []}
    tot_r = tot_w = 0.0
    for (n, fk, t), (_, wk, _) in zip(f, w):
        rb, wb = fk * 1024 * 2, wk * 1024   # KiB; FETCH x2 on gfx950
        tot_r += rb
        tot_w += wb
        rep["kernels"].append({"kernel": n, "fetch_bytes_x2": rb, "write_bytes": wb, "dur_us_profiled": t})
    px = B * H * W
    rep["hbm_bytes_per_step"] = tot_r + tot_w
    rep["hbm_bytes_per_px"] = (tot_r + tot_w) / px
    rep["algorithmic_bytes_per_px"] = (2 * C + 5) * 4
    # the library these counters came from: bench.py uses the file only for a
    # run of the same build (the hash of the sources, as _native checks it)
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from opticalflowfromdepth_amd import build as _b
    rep["build_id"] = _b.built_id() or _b.source_hash()
    rep["source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, last call of a bench.py run; "
                     "FETCH_SIZE x2 per MI355X_MICROARCH.md (gfx950 half-count of wide reads)")
    print(json.dumps(rep, indent=1))
    if dst:
        json.dump(rep, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
