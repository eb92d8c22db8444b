"""Time the layered fill's deep-tail cliff: at one shape, a deep
call (ego-motion border bands) after a history of shallow calls (disparity
holes) runs the layers beyond the history's depth in the one-workgroup tail
kernel; the same deep call with deep calls in the history does not.
Usage: python tools/tail_cliff.py [B H W]  -> one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, shard, synth  # noqa: E402


def main():
    B, H, W = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (16, 768, 1024)
    dev = torch.device("cuda:0")
    lib = _native.lib()
    seeds = [shard.image_seed(i) for i in range(B)]

    def inputs(ego):
        out, valid, coll = forward_warp_flow(*synth.stage_one_batch(seeds, H, W, dev, ego_fraction=ego))
        return (out[:, 0:3] * valid).contiguous(), valid, coll

    s_in, d_in = inputs(0.0), inputs(1.0)

    def timed(x):
        torch.cuda.synchronize()
        lib.ofd_inpaint_tail_layers(1)
        t0 = time.perf_counter()
        ops.inpaint(*x, order="layered")
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, lib.ofd_inpaint_tail_layers(1)

    for _ in range(10):
        ops.inpaint(*s_in, order="layered")
    torch.cuda.synchronize()
    time.sleep(0.1)
    shallow_ms, _ = timed(s_in)
    time.sleep(0.1)
    cliff_ms, cliff_layers = timed(d_in)  # deep after 8+ shallow calls: the tail runs the extra layers
    for _ in range(3):
        ops.inpaint(*d_in, order="layered")
        torch.cuda.synchronize()
        time.sleep(0.05)
    deep_ms, deep_layers = timed(d_in)
    print(json.dumps({"images": B, "height": H, "width": W, "shallow_ms": round(shallow_ms, 3),
                      "deep_after_shallow_history_ms": round(cliff_ms, 3), "tail_layers": cliff_layers,
                      "deep_after_deep_history_ms": round(deep_ms, 3), "tail_layers_warm": deep_layers}))


if __name__ == "__main__":
    main()
