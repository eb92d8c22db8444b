"""Anatomy of the persistent fused SPLAT at the headline workload (diagnostic, GPU only).

Uses tools/probe_tile.hip (the product TU + per-tile wall-clock stamps):
case 0 = BIN, 8 = stamped persistent fused SPLAT, 9 = unstamped.  Prints the
per-tile phase medians split by flow kind (disparity images 0..B/2-1,
ego-motion images B/2..), the launch span, how many workgroups are busy over
time (the drain tail), and the slowest tiles.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import probe_tile as pt  # noqa: E402
from opticalflowfromdepth_amd import synth  # noqa: E402


def band_major(lin, nimg, tilesX=8, tilesY=24):
    start = 0
    for k in range(8):
        r0, r1 = k * tilesY // 8, (k + 1) * tilesY // 8
        per_img = (r1 - r0) * tilesX
        cnt = per_img * nimg
        if lin < start + cnt or k == 7:
            idx = lin - start
            bl = idx // per_img
            return bl, r0 * tilesX + idx - bl * per_img
        start += cnt


def main():
    import ctypes
    pt.build()
    lib = ctypes.CDLL(pt.SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), int(os.environ.get("H", "768")), int(os.environ.get("W", "1024"))
    TW, TH = int(os.environ.get("TW", "128")), int(os.environ.get("TH", "32"))
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev)
    C = obj.shape[1]
    out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
    slab = torch.full((lib.probe_slab_bytes(B, H, W),), 255, dtype=torch.uint8, device=dev)
    ntiles = B * ((H + TH - 1) // TH) * ((W + TW - 1) // TW)
    stamps = torch.zeros(8 * (ntiles + 64), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(), coll.data_ptr(),
            C, H, W, slab.data_ptr(), 0, B, stamps.data_ptr(), st)

    def run(whichs):
        ev = []
        for w in whichs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert lib.probe_launch(w, *base) == 0
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        return [a.elapsed_time(b) * 1e3 for a, b in ev]

    for _ in range(3):
        run([0, 9])
    t = np.median(np.array([run([0, 9]) for _ in range(10)]), axis=0)
    print(f"BIN {t[0]:.1f} us, persistent SPLAT {t[1]:.1f} us (unstamped, medians of 10)")
    from opticalflowfromdepth_amd import forward_warp_flow
    ref = forward_warp_flow(obj, flow, depth)
    print("probe result == product:", all(torch.equal(x, y) for x, y in zip((out, valid, coll), ref)))
    stamps.zero_()
    ts = run([0, 8])
    print(f"stamped persistent SPLAT {ts[1]:.1f} us")
    s = stamps.view(-1, 8).cpu().numpy()
    s = s[s[:, 1] > 0].astype(np.int64)
    t0 = s[:, 0].min()
    seg = (s[:, 4] - s[:, 0]) / 100.0
    spl = (s[:, 5] - s[:, 4]) / 100.0
    mrg = (s[:, 6] - s[:, 5]) / 100.0
    pub = (s[:, 1] - s[:, 6]) / 100.0
    tot = (s[:, 1] - s[:, 0]) / 100.0
    bl = np.array([band_major(int(l), B, (W + TW - 1) // TW, (H + TH - 1) // TH)[0] for l in s[:, 3]])
    tile = np.array([band_major(int(l), B, (W + TW - 1) // TW, (H + TH - 1) // TH)[1] for l in s[:, 3]])
    for name, m in (("disparity", bl < B // 2), ("ego", bl >= B // 2)):
        print(f"{name:9s} tiles {m.sum():5d}: median seg {np.median(seg[m]):5.2f} splat {np.median(spl[m]):5.2f} "
              f"merge {np.median(mrg[m]):5.2f} publish {np.median(pub[m]):5.2f} total {np.median(tot[m]):5.2f} "
              f"p90 {np.percentile(tot[m], 90):6.2f} max {tot[m].max():7.2f} sum {tot[m].sum():9.1f} us; "
              f"nseg median {np.median(s[m, 7]):.0f} max {s[m, 7].max()}")
    span = (s[:, 1].max() - t0) / 100.0
    print(f"span {span:.1f} us; sum of tile times {tot.sum():.0f} us = {tot.sum() / span:.0f} busy workgroups on average")
    t1 = (s[:, 1] - t0) / 100.0
    ta = (s[:, 0] - t0) / 100.0
    pts = np.linspace(0, span, 21)[:-1]
    print("busy workgroups at 5% steps: " + " ".join(str(int(((ta <= p) & (t1 > p)).sum())) for p in pts))
    print("tiles finishing in the last 10% of the span:", int((t1 > 0.9 * span).sum()))
    slow = np.argsort(-tot)[:12]
    print("slowest tiles (image, tile, total us, segs, publish us, splat us):")
    for i in slow:
        print(f"   img {bl[i]:3d} tile {tile[i]:3d}  {tot[i]:7.2f}  nseg {s[i, 7]:5d}  pub {pub[i]:6.2f}  splat {spl[i]:6.2f}")
    # per tile-row: where do heavy tiles sit
    ty = tile // ((W + TW - 1) // TW)
    tx = tile % ((W + TW - 1) // TW)
    for name, m in (("disparity", bl < B // 2), ("ego", bl >= B // 2)):
        grid = np.zeros(((H + TH - 1) // TH, (W + TW - 1) // TW))
        for a, b_, v in zip(ty[m], tx[m], tot[m]):
            grid[a, b_] += v / (B // 2)
        print(f"{name} mean tile time by tile position (rows 0,1,2 ... last):")
        for r in list(range(3)) + [grid.shape[0] // 2] + list(range(grid.shape[0] - 2, grid.shape[0])):
            print(f"   row {r:2d}: " + " ".join(f"{v:5.1f}" for v in grid[r]))


if __name__ == "__main__":
    main()
