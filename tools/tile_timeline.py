"""Per-tile timeline of the persistent fused SPLAT on the headline batch (diagnostic, GPU only).

Runs BIN + the stamped persistent SPLAT of tools/probe_tile.hip (cases 15 + 16,
packed targets; PACK=0: cases 0 + 8) on the
headline workload (64 x 768x1024, C = 6, half disparity / half ego-motion) and
prints where the kernel's span goes:
  - per-tile duration by kind (disparity / ego image, border / interior tile)
    and its candidate-block count;
  - the drain: when the last tile was dequeued vs the span's end, how many
    workgroups are still resident over the last 100 us, and which tiles run
    last.
Writes the raw stamps to gpurun_out/tile_timeline.npz.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import probe_tile  # noqa: E402
from opticalflowfromdepth_amd import synth  # noqa: E402


def main():
    probe_tile.build()
    import ctypes
    lib = ctypes.CDLL(probe_tile.SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), int(os.environ.get("H", "768")), int(os.environ.get("W", "1024"))
    ego = float(os.environ.get("EGO", "0.5"))
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev, ego_fraction=ego)
    n_disp = B - int(round(B * ego))
    C = obj.shape[1]
    out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
    slab = torch.full((lib.probe_slab_bytes(B, H, W),), 255, dtype=torch.uint8, device=dev)
    tx, ty = (W + 127) // 128, (H + 31) // 32
    ntiles = B * tx * ty
    stamps = torch.zeros(8 * (ntiles + 64), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(), coll.data_ptr(),
            C, H, W, slab.data_ptr(), 0, B, stamps.data_ptr(), st)
    runs = []
    for rep in range(int(os.environ.get("REPS", "6"))):
        stamps.zero_()
        for w in ((15, 16) if os.environ.get("PACK", "1") != "0" else (0, 8)):
            assert lib.probe_launch(w, *base) == 0
        torch.cuda.synchronize()
        runs.append(stamps.view(-1, 8)[:ntiles].cpu().numpy().copy())
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(REPO, "gpurun_out", "tile_timeline.npz"), *runs)

    spans = []
    for r, s in enumerate(runs):
        s = s[s[:, 1] > 0]
        t0 = s[:, 0].min()
        start, end = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0
        dur = end - start
        lin = s[:, 3]
        nblk = s[:, 2]
        # band-major: recover (image, tile) like band_major_tile
        img = np.zeros_like(lin)
        tile = np.zeros_like(lin)
        startk = 0
        for k in range(8):
            r0, r1 = k * ty // 8, (k + 1) * ty // 8
            per_img = (r1 - r0) * tx
            cnt = per_img * B
            sel = (lin >= startk) & ((lin < startk + cnt) | (k == 7))
            idx = lin[sel] - startk
            img[sel] = idx // per_img
            tile[sel] = r0 * tx + idx % per_img
            startk += cnt
        trow, tcol = tile // tx, tile % tx
        border = (trow == 0) | (trow == ty - 1) | (tcol == 0) | (tcol == tx - 1)
        isego = img >= n_disp
        span = end.max()
        spans.append(span)
        if r < len(runs) - 2:
            continue
        print(f"run {r}: span {span:.1f} us over {len(s)} tiles; last dequeue (start) at {start.max():.1f} us; "
              f"sum of tile time / span = {dur.sum() / span:.0f} resident wgs")
        for nm, m in (("disp interior", ~isego & ~border), ("disp border", ~isego & border),
                      ("ego interior", isego & ~border), ("ego border", isego & border)):
            if m.sum():
                print(f"  {nm:14s} n={m.sum():5d} dur med {np.median(dur[m]):6.1f} p90 {np.percentile(dur[m], 90):6.1f} "
                      f"max {dur[m].max():6.1f} us   nblk med {np.median(nblk[m]):6.0f} max {nblk[m].max():6.0f}  "
                      f"total {dur[m].sum() / 1e3:7.1f} ms-wg")
        for q in (0.90, 0.95, 0.98):
            t = span * q
            print(f"  resident at {q:.2f} of span ({t:.0f} us): {int(((start <= t) & (end > t)).sum())}")
        pts = np.arange(0.0, span, 20.0)
        act = [int(((start <= t) & (end > t)).sum()) for t in pts]
        print("  resident every 20 us: " + " ".join(map(str, act)))
        last = np.argsort(end)[-12:]
        print("  last 12 tiles to finish (img kind row col start dur nblk):")
        for i in last:
            print(f"    img {img[i]:2d} {'ego ' if isego[i] else 'disp'} r{trow[i]:2d} c{tcol[i]} "
                  f"start {start[i]:6.1f} dur {dur[i]:6.1f} nblk {nblk[i]}")
        heavy = np.argsort(dur)[::-1][:20]
        print("  20 heaviest tiles (img kind row col dur nblk): " +
              "; ".join(f"{img[i]}{'e' if isego[i] else 'd'} r{trow[i]}c{tcol[i]} {dur[i]:.0f}us {nblk[i]}" for i in heavy))
    print(f"spans (us): {' '.join(f'{x:.1f}' for x in spans)}")


if __name__ == "__main__":
    main()
