"""Run the fused first-stage warps at the headline size (for rocprofv3 kernel traces).

    rocprofv3 --kernel-trace --stats -d gpurun_out/fz -- python3 tools/fused_time.py
Runs warp_disparity (float32 and float64 depth) and warp_ego (float64 depth)
over 64 images of 768x1024, 10 calls each, plus the plain FW call on the
materialised inputs for comparison.
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import forward_warp_flow, synth, warp_disparity, warp_ego  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), 768, 1024
    seeds = [12345 + i for i in range(B)]
    d64 = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64))
    d32 = d64.float()
    rgb = synth.synthetic_rgb(seeds, H, W, dev)
    s, T = synth.batch_camera_params(seeds)
    P, ik = synth.projection(H, W, T.to(dev), dev)
    s = s.to(dev)
    runs = {"disp_f32": lambda: warp_disparity(rgb, d32, s), "disp_f64": lambda: warp_disparity(rgb, d64, s),
            "ego_f64": lambda: warp_ego(rgb, d64, P, ik), "ego_f32": lambda: warp_ego(rgb, d32, P, ik)}
    obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev)
    runs["fw_plain"] = lambda: forward_warp_flow(obj, flow, depth)
    for name, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        print(f"{name:10s} {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call", flush=True)


if __name__ == "__main__":
    main()
