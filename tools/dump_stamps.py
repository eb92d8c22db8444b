"""Dump the sequential fill's final inner-march stamps (sI) of a few warped
768x1024 images for offline Kahn-depth studies (diagnostic, GPU only):
    python tools/dump_stamps.py gpurun_out/stamps.npz SEED [SEED ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflowfromdepth_amd import forward_warp_flow, ops, synth  # noqa: E402


def main():
    out = sys.argv[1]
    seeds = [int(x) for x in sys.argv[2:]]
    dev = torch.device("cuda:0")
    H, W = 768, 1024
    obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev)
    o, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (o[:, 0:3] * valid).contiguous()
    ops.inpaint(rgb, valid, coll, order="sequential")
    torch.cuda.synchronize()
    ws = ops._ip_workspaces[(dev.index, torch.cuda.current_stream().cuda_stream)]
    B = len(seeds)
    eh, ew = H + 2, W + 2
    en = eh * ew
    a256 = lambda x: (x + 255) & ~255  # noqa: E731
    off = a256(B * en * 4)  # sO, then sI
    sI = ws[off:off + B * en * 4].view(torch.int32).view(B, eh, ew).cpu().numpy()
    np.savez_compressed(out, sI=sI, seeds=np.array(seeds))
    print("stamps", sI.shape, "holes", [(int(((s != 0) & (s != -1)).sum())) for s in sI])


if __name__ == "__main__":
    main()
