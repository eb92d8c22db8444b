"""Per-kernel times of the TILE engine and SPLAT workgroup phases (diagnostic, GPU only).

Builds tools/probe_tile.hip (the product TU + stamps), makes the headline
workload with opticalflowfromdepth_amd.synth, and for chunks of G images runs
BIN, SPLAT and RESOLVE as separate timed launches; prints launch times and the
SPLAT workgroups' phase medians (us).  Checks the result against the product
library on the same inputs.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import forward_warp_flow, synth  # noqa: E402

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
    lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), 768, 1024
    G = int(os.environ.get("G", "32"))
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev)
    C = obj.shape[1]
    out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
    slab = torch.full((lib.probe_slab_bytes(G, H, W),), 255, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(8 * 200000, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(), coll.data_ptr(),
            C, H, W, slab.data_ptr())
    names = ("bin", "splat", "resolve")
    for rep in range(2):
        tot = [0.0, 0.0, 0.0]
        for c0 in range(0, B, G):
            n = min(G, B - c0)
            for which in range(3):
                stamps.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.probe_launch(which, *base, c0, n, stamps.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                tot[which] += e0.elapsed_time(e1) * 1e3
                if rep == 1 and which == 1:
                    s = stamps.view(-1, 8).cpu().numpy()
                    s = s[s[:, 1] > 0]
                    ph = [(s[:, 4] - s[:, 0]) / 100.0, (s[:, 5] - s[:, 4]) / 100.0, (s[:, 6] - s[:, 5]) / 100.0,
                          (s[:, 1] - s[:, 6]) / 100.0, (s[:, 1] - s[:, 0]) / 100.0]
                    pn = ["segscan", "candscan+splat", "merge", "publish", "total"]
                    print(f"chunk {c0:3d}: splat wg phase medians " +
                          "  ".join(f"{k}={np.median(v):5.1f}" for k, v in zip(pn, ph)) +
                          f"  p99 total={np.percentile(ph[4], 99):.1f}  nseg median={np.median(s[:, 7]):.0f}")
                    span = (s[:, 1].max() - s[:, 0].min()) / 100.0
                    print(f"           splat span {span:.1f} us, mean resident workgroups "
                          f"{ph[4].sum() / span:.0f}, first-wave start spread "
                          f"{(np.sort(s[:, 0])[1023] - s[:, 0].min()) / 100.0:.1f} us")
                    t0s, t1s = s[:, 0] - s[:, 0].min(), s[:, 1] - s[:, 0].min()
                    pts = np.linspace(0, t1s.max(), 13)[:-1]
                    act = [int(((t0s <= t) & (t1s > t)).sum()) for t in pts]
                    print("           resident workgroups at 12 points of the span: " + " ".join(map(str, act)))
        if rep == 1:
            print("per-step launch totals (us): " + "  ".join(f"{k}={v:.1f}" for k, v in zip(names, tot)) +
                  f"  sum={sum(tot):.1f}  ({B} images, chunks of {G})")
    ref = forward_warp_flow(obj, flow, depth)
    if os.environ.get("SPLAT_SWEEP"):
        # SPLAT variants, interleaved round-robin over 15 rounds (each run
        # re-BINs first: SPLAT consumes the records); median per variant
        variants = ((1, "product"), (3, "plain stores"), (4, "nt all"), (5, "3 slots"),
                    (7, "images strided over XCDs"), (8, "images contiguous"))
        ts = {nm: [] for _, nm in variants}
        for rnd in range(16):
            for which, nm in variants:
                tot = 0.0
                for c0 in range(0, B, G):
                    lib.probe_launch(0, *base, c0, min(G, B - c0), stamps.data_ptr(), st)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rc = lib.probe_launch(which, *base, c0, min(G, B - c0), stamps.data_ptr(), st)
                    e1.record()
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    tot += e0.elapsed_time(e1) * 1e3
                if rnd > 0:
                    ts[nm].append(tot)
        print(f"SPLAT variants, chunks of {G}, median of 15 interleaved (us): " +
              "  ".join(f"{nm}={np.median(v):.1f}" for nm, v in ts.items()))
    if os.environ.get("RESOLVE_SWEEP"):
        # RESOLVE variants over the winner map of the last chunk (G images)
        names_v = ["product", "1x16nt+ntw", "4x4", "1x8", "2x4", "1x4", "1x16nt", "2x8nt", "4x4nt", "8x2nt", "2x4nt",
                   "2x8nt+ntw", "4x4nt+ntw", "16x1nt"]
        c0 = B - G
        for rep in range(2):
            res = []
            for v in range(len(names_v)):
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rc = lib.probe_launch(10 + v, *base, c0, G, stamps.data_ptr(), st)
                    e1.record()
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    ts.append(e0.elapsed_time(e1) * 1e3)
                ok_v = torch.equal(out[c0:], ref[0][c0:])
                res.append(f"{names_v[v]}={np.median(ts):.1f}{'' if ok_v else '(BAD)'}")
            if rep == 1:
                print(f"RESOLVE variants, {G} images, median of 5 (us): " + "  ".join(res))
    ok = all(torch.equal(x, y) for x, y in zip((out, valid, coll), ref))
    print("probe result == product result:", ok)

if __name__ == "__main__":
    main()
