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
    pi = a256(en * 4) * 6 + a256(en * 8) * 2 + a256(eh * 4) + 256
    G = min(B, (ws.numel() - 2048) // pi)
    off = 6 * a256(G * en * 4) + 2 * a256(G * en * 8) + a256(G * eh * 4)
    return ws[off:off + G * 8 * 4].view(torch.int32).view(G, 8).cpu().numpy()


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
    print("meta columns: band, pushes, level0, levels, buckets, error")
    for k in np.argsort(-m[:, 3])[:8]:
        print(k, m[k, :6].tolist())
    print("max levels", m[:, 3].max(), "max buckets", m[:, 4].max(), "errors", int((m[:, 5] != 0).sum()))


if __name__ == "__main__":
    main()
