"""Time the hole-fill orders on the headline batch (64 warped 768x1024 RGB) and
report the sequential fill's per-image march statistics (buckets, pushes,
Kahn levels) read from its workspace.  Usage: python tools/seq_time.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflowfromdepth_amd import forward_warp_flow, ops, synth  # noqa: E402


def a256(x):
    return (x + 255) & ~255


def seq_meta(ws, B, H, W):
    eh, ew = H + 2, W + 2
    en = eh * ew
    pi = (a256(en * 4) * 6 + a256(en * 8) * 2 + a256(eh * 4) + 32 * 4 + en * 160 + H * W * 4 + en * 8 + 768
          + en * 8 + en * 24 + en * 8 + en * 4 + en * 8 + 64 * 4 + 6 * 256)
    G = min(B, (ws.numel() - 2048) // pi)
    off = 6 * a256(G * en * 4) + 2 * a256(G * en * 8) + a256(G * eh * 4)
    return ws[off:off + G * 32 * 4].view(torch.int32).view(G, 32).cpu().numpy()


def seq_pipe(ws, B, H, W):
    """The pipelined fill's per-image control / timeline words (kPipe = 64 per
    image, after the ready queue and the carry buffer; csrc/ofd_inpaint_seq.hip carve())."""
    eh, ew = H + 2, W + 2
    en, hw = eh * ew, H * W
    G = B
    off = (6 * a256(G * en * 4) + 2 * a256(G * en * 8) + a256(G * eh * 4) + a256(G * 32 * 4) + a256(G * en * 160)
           + a256(G * hw * 4) + 2 * a256(G * en * 8) + a256(G * en * 24) + a256(G * en * 8) + a256(G * en * 4)
           + a256(G * en * 8) + a256(G * en * 8))
    return ws[off:off + G * 64 * 4].view(torch.int32).view(G, 64).cpu().numpy().astype(np.int64) & 0xFFFFFFFF


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda:0")
    seeds = [12345 + i for i in range(B)]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    for order in ("layered", "sequential"):
        r = ops.inpaint(rgb, valid, coll, order=order)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        n = 3
        for _ in range(n):
            r = ops.inpaint(rgb, valid, coll, order=order)
        ev[1].record()
        torch.cuda.synchronize()
        print(f"{order}: {ev[0].elapsed_time(ev[1]) / n:.3f} ms per {B} images", flush=True)
    key = (dev.index, torch.cuda.current_stream().cuda_stream)
    ws = ops._ip_workspaces[key]
    m = seq_meta(ws, B, 768, 1024)
    print("meta columns: band, pushes, level0, levels, buckets, error, colour3 rounds, levels <= 64 holes")
    if not m[:, 8:24].any():  # non-probe build: each march's wall-clock duration (100 MHz ticks)
        o, i = m[:, 24].astype(np.float64) / 100.0, m[:, 25].astype(np.float64) / 100.0
        print(f"marches (us, 100 MHz wall clock): outer max {o.max():.0f} (image {int(o.argmax())}), "
              f"inner max {i.max():.0f} (image {int(i.argmax())}); images whose outer march is the longer: "
              f"{int((o > i).sum())} of {len(o)}")
        for k in np.argsort(-np.maximum(o, i))[:6]:
            print(f"  image {int(k)}: outer {o[k]:.0f} us, inner {i[k]:.0f} us, levels {int(m[k, 3])}")
    for k in np.argsort(-m[:, 3])[:8]:
        print(k, m[k, :8].tolist())
    try:
        pp = seq_pipe(ws, B, 768, 1024)
    except RuntimeError:  # a probe build with an older workspace layout
        pp = np.zeros((B, 64), np.int64)
    t = lambda c: (pp[:, c] | (pp[:, c + 1] << 32)).astype(np.float64)  # noqa: E731
    t0 = t(8).min()
    if t0 > 0:  # pipelined-fill timeline of the last call (us from the first march's start)
        rel = lambda c: np.where(t(c) > 0, (t(c) - t0) / 100.0, np.nan)  # noqa: E731
        fo, fi, c0, c1 = rel(10), rel(12), rel(40), rel(42)
        print(f"timeline (us): outer end max {np.nanmax(fo):.0f}, inner end max {np.nanmax(fi):.0f}, "
              f"colour end max {np.nanmax(c1):.0f} (image {int(np.nanargmax(c1))})")
        for k in np.argsort(-np.nan_to_num(c1))[:6]:
            print(f"  image {int(k)}: outer end {fo[k]:.0f}, inner end {fi[k]:.0f}, colour {c0[k]:.0f} .. {c1[k]:.0f}"
                  f" in {int(pp[k, 44])} rounds, levels {int(m[k, 3])}")
    eh, ew = 770, 1026
    en = eh * ew
    pi_ = a256(en * 4) * 6 + a256(en * 8) * 2 + a256(eh * 4) + 32 * 4 + en * 160 + 768 * 1024 * 4 + en * 8 + 768
    G = min(B, (ws.numel() - 2048) // pi_)
    k1 = 6 * a256(G * en * 4) + a256(G * en * 8)
    kdeep = int(np.argmax(m[:, 3])) if m[:, 3].any() else int(np.argmax(m[:, 7]))  # levels-free pass: most batches
    L = int(m[kdeep, 3])
    if not os.environ.get("OFD_SEQ_COLOUR", "").startswith("g"):  # level sizes: the g16 colour kernel only
        print(f"deepest image {kdeep}: {L} levels")
        if m[:, 8:24].any():
            r = m[kdeep]
            print("FMM   gather/sort/claim/push/dist/log (Mclk):", [round(x * 256 / 1e6, 2) for x in r[8:14]],
                  "sweeps", int(r[14]))
            print("FMM (buckets > 4096 keys) -/sort/claim/push/dist/log (Mclk):",
                  [round(x * 256 / 1e6, 2) for x in r[24:30]], "sweeps", int(r[30]))
            print("COLOUR3 level work/barrier, per-round loads/terms/chains/final+append/atomics (Mclk;"
                  " levels-free pass: publish/append/loads/terms/chains/final/wait/atomic return):",
                  [round(x * 256 / 1e6, 2) for x in r[16:24]])
        print("max levels", m[:, 3].max(), "max buckets", m[:, 4].max(), "errors", int((m[:, 5] != 0).sum()))
        if m[:, 8:24].any():  # per image: FMM phase sum vs COLOUR3 level work + barrier (Mclk)
            f = m[:, 8:14].astype(np.float64).sum(1) * 256 / 1e6
            c = m[:, 16:18].astype(np.float64).sum(1) * 256 / 1e6
            print("per image (Mclk): max FMM", round(f.max(), 2), "max COLOUR3", round(c.max(), 2),
                  "max FMM+COLOUR3", round((f + c).max(), 2))
            for k in np.argsort(-(f + c))[:6]:
                print("  image", int(k), "FMM", round(f[k], 2), "COLOUR3", round(c[k], 2), "levels", int(m[k, 3]),
                      "buckets", int(m[k, 4]), "pushes", int(m[k, 1]))
        return
    lsz = ws[k1 + kdeep * en * 8: k1 + kdeep * en * 8 + L * 4].view(torch.int32).cpu().numpy()
    q = np.percentile(lsz, [0, 10, 50, 90, 99, 100])
    print(f"deepest image {kdeep}: {L} levels, level sizes p0/10/50/90/99/100 {q.tolist()}, "
          f"levels with <=16 holes {(lsz <= 16).mean():.2f}, <=64 {(lsz <= 64).mean():.2f}; "
          f"sum ceil(n/16) {int(np.ceil(lsz / 16).sum())}, sum ceil(n/256) {int(np.ceil(lsz / 256).sum())}")
    if m[:, 8:24].any():  # probe build (tools/seq_probe.sh): clocks >> 8, deepest image
        r = m[kdeep]
        print("FMM   gather/sort/claim/push/dist/log (Mclk):", [round(x * 256 / 1e6, 2) for x in r[8:14]],
              "sweeps", int(r[14]))
        print("COLOUR level work/barrier, per-pixel [value loads], load/weights/channels/release, [terms] (Mclk):",
              [round(x * 256 / 1e6, 2) for x in r[16:24]])
    print("max levels", m[:, 3].max(), "max buckets", m[:, 4].max(), "errors", int((m[:, 5] != 0).sum()))


if __name__ == "__main__":
    main()
