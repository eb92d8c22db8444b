"""Per-workgroup latency of the TILE engine's roles (diagnostic, GPU only).

Builds tools/probe_tile.hip (the product TU + stamps), makes the headline
workload with opticalflowfromdepth_amd.synth, runs BIN-only and TILE-only
launches per chunk and prints per-role workgroup duration percentiles (us).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import synth  # noqa: E402

SO = os.path.join(REPO, "tools", "_build", "libprobe_tile.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-I", os.path.join(REPO, "include"), "-o", SO, os.path.join(REPO, "tools", "probe_tile.hip")],
                   check=True)


def main():
    build()
    lib = ctypes.CDLL(SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.probe_launch.argtypes = [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    B, H, W = 16, 768, 1024
    G = int(os.environ.get("G", "4"))
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev)
    C = obj.shape[1]
    out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
    slab = torch.full((lib.probe_slab_bytes(G, H, W),), 255, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(8 * 20000, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    args = lambda: (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(),
                    coll.data_ptr(), C, H, W, slab.data_ptr())
    for rep in range(2):
        for c0 in range(0, B, G):
            kind = "disp" if c0 < B // 2 else "ego"
            for role in ("bin", "tile"):
                stamps.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if role == "bin":
                    rc = lib.probe_launch(*args(), 0, 0, c0, G, G, stamps.data_ptr(), st)
                else:
                    rc = lib.probe_launch(*args(), c0, G, 0, 0, G, stamps.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                if rep == 0:
                    continue
                s = stamps.view(-1, 8).cpu().numpy()
                s = s[s[:, 1] > 0]
                dur = (s[:, 1] - s[:, 0]) / 100.0   # wall_clock64 = 100 MHz
                span = (s[:, 1].max() - s[:, 0].min()) / 100.0
                pct = np.percentile(dur, [10, 50, 90, 99, 100])
                print(f"chunk {c0:2d} {kind:4s} {role:4s} wgs={len(s):5d} launch={e0.elapsed_time(e1)*1e3:7.1f}us "
                      f"span={span:7.1f}us wg p10/50/90/99/max = " + " ".join(f"{v:6.1f}" for v in pct))
                if role == "tile":
                    ph = [(s[:, 4] - s[:, 0]) / 100.0, (s[:, 5] - s[:, 4]) / 100.0, (s[:, 6] - s[:, 5]) / 100.0,
                          (s[:, 1] - s[:, 6]) / 100.0]
                    names = ["init+segscan", "candscan+splat", "merge", "resolve"]
                    print("      phases median: " + "  ".join(f"{n}={np.median(v):5.1f}" for n, v in zip(names, ph)) +
                          f"  nseg median={np.median(s[:, 7]):.0f} max={s[:, 7].max()}")


if __name__ == "__main__":
    main()
