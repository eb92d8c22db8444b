"""Run the fused first-stage warps at the headline size (for rocprofv3 kernel traces).

    rocprofv3 --kernel-trace --stats -d gpurun_out/fz -- python3 tools/fused_time.py
Runs warp_disparity (float32 and float64 depth) and warp_ego (float64 depth)
over 64 images of 768x1024, 10 calls each, plus the plain FW call on the
materialised inputs for comparison, and warp_flow_cat on the ego-motion plane
(float64 / float32 depth) beside the plain FW on the same all-ego flows
(RUNS=name,name selects).
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, synth, warp_disparity, warp_ego, warp_flow_cat  # noqa: E402


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
    # warp_flow_cat on the ego plane (the pipeline's ego-motion warp), and the
    # plain FW on the same all-ego flows materialised (the comparator)
    plane = ego_flow(d64, P, ik)
    runs["flowcat_ego_f64"] = lambda: warp_flow_cat(rgb, plane, d64)
    runs["flowcat_ego_f32"] = lambda: warp_flow_cat(rgb, plane, d32)
    cat = torch.cat((rgb, d32, plane * -1.0), 1)
    runs["fw_ego_cat"] = lambda: forward_warp_flow(cat, plane, d32)
    only = os.environ.get("RUNS")
    if only:
        runs = {k: v for k, v in runs.items() if k in only.split(",")}
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
