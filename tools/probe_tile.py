"""Per-kernel times of the TILE engine variants and SPLAT workgroup phases (diagnostic, GPU only).

Builds tools/probe_tile.hip (the product TU + stamps), makes the headline
workload with opticalflowfromdepth_amd.synth and times, interleaved over
rounds, each launch of:
  split : BIN (1 segment / wave) -> SPLAT (winner map) -> RESOLVE
  fused : BIN -> SPLAT gathering the output itself (one workgroup per tile)
  persist: BIN -> the same SPLAT as a persistent kernel over per-XCD tile queues
Prints per-launch medians, the SPLAT workgroups' phase medians (stamped
builds) and checks every variant's result against the product library.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import _native, forward_warp_flow, synth  # noqa: E402

SO = os.environ.get("PROBE_LIB") or os.path.join(REPO, "tools", "_build", "libprobe_tile.so")
NAMES = {0: "bin1", 3: "bin2", 4: "bin4", 1: "splat(stamped)", 5: "splat", 6: "fused(stamped)", 7: "fused",
         8: "persist(stamped)", 9: "persist", 10: "fused512_t2w8", 11: "fused256_t8w4", 12: "persist256_t8w4",
         13: "fused512_t8w4u3", 14: "fused256_t8w4u3", 2: "resolve"}


def build():
    if os.environ.get("PROBE_LIB"):
        return  # a prebuilt variant (e.g. another tile shape)
    srcs = [os.path.join(REPO, "tools", "probe_tile.hip"), os.path.join(REPO, "opticalflowfromdepth_amd", "csrc",
                                                                       "ofd_fw.hip")]
    if os.path.exists(SO) and all(os.path.getmtime(SO) > os.path.getmtime(x) for x in srcs):
        return  # built in-tree beforehand (it travels with the snapshot)
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-I", os.path.join(REPO, "include"), "-o", SO, os.path.join(REPO, "tools", "probe_tile.hip")],
                   check=True)


def phases(stamps, label):
    s = stamps.view(-1, 8).cpu().numpy()
    s = s[s[:, 1] > 0]
    ph = [(s[:, 4] - s[:, 0]) / 100.0, (s[:, 5] - s[:, 4]) / 100.0, (s[:, 6] - s[:, 5]) / 100.0,
          (s[:, 1] - s[:, 6]) / 100.0, (s[:, 1] - s[:, 0]) / 100.0]
    pn = ["segscan", "candscan+splat", "merge", "publish", "total"]
    span = (s[:, 1].max() - s[:, 0].min()) / 100.0
    print(f"{label}: wg phase medians " + "  ".join(f"{k}={np.median(v):5.1f}" for k, v in zip(pn, ph)) +
          f"  p99 total={np.percentile(ph[4], 99):.1f}  nseg median={np.median(s[:, 7]):.0f}")
    t0s, t1s = s[:, 0] - s[:, 0].min(), s[:, 1] - s[:, 0].min()
    pts = np.linspace(0, t1s.max(), 13)[:-1]
    act = [int(((t0s <= t) & (t1s > t)).sum()) for t in pts]
    print(f"    span {span:.1f} us, mean resident workgroups {ph[4].sum() / span:.0f}; resident at 12 points: " +
          " ".join(map(str, act)))


def main():
    build()
    lib = ctypes.CDLL(SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), int(os.environ.get("H", "768")), int(os.environ.get("W", "1024"))
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev,
                                             ego_fraction=float(os.environ.get("EGO", "0.5")))
    C = obj.shape[1]
    out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
    slab = torch.full((lib.probe_slab_bytes(B, H, W),), 255, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(8 * (B * 768 + 64), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(), coll.data_ptr(),
            C, H, W, slab.data_ptr(), 0, B, stamps.data_ptr(), st)

    nlib = _native.lib()
    prev = nlib.ofd_fw_set_engine(2)
    ref = forward_warp_flow(obj, flow, depth)
    nlib.ofd_fw_set_engine(prev)

    def seq(whichs):
        ts = []
        for w in whichs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.probe_launch(w, *base)
            e1.record()
            assert rc == 0, (w, rc)
            ts.append((e0, e1))
        torch.cuda.synchronize()
        return [a.elapsed_time(b) * 1e3 for a, b in ts]

    def check(label):
        ok = all(torch.equal(x, y) for x, y in zip((out, valid, coll), ref))
        print(f"{label} result == split-engine product result: {ok}")
        for t in (out, valid, coll):
            t.fill_(-7.0)
        return ok

    configs = {"split": [0, 5, 2], "fused": [0, 7], "persist": [0, 9], "f512t2": [0, 10], "f256t8": [0, 11],
               "p256t8": [0, 12], "f512u3": [0, 13], "f256u3": [0, 14]}
    for name, whichs in configs.items():
        seq(whichs)
        check(name)
    times = {k: [] for k in configs}
    for rnd in range(int(os.environ.get("ROUNDS", "12"))):
        for name, whichs in configs.items():
            times[name].append(seq(whichs))
    for name, whichs in configs.items():
        med = np.median(np.array(times[name]), axis=0)
        print(f"{name:12s} " + "  ".join(f"{NAMES[w]}={m:6.1f}" for w, m in zip(whichs, med)) +
              f"  sum={med.sum():6.1f} us")
    for label, whichs in (("split SPLAT", [0, 1]), ("fused SPLAT", [0, 6]), ("persistent fused SPLAT", [0, 8])):
        stamps.zero_()
        seq(whichs)
        phases(stamps, label)
    check("fused (stamped)")

    # the product library, every engine, against the split reference
    for eng, nm in ((0, "tile(fused)"), (2, "tile-split"), (1, "atomic")):
        nlib.ofd_fw_set_engine(eng)
        got = forward_warp_flow(obj, flow, depth)
        print(f"product engine {nm}: equal = {all(torch.equal(x, y) for x, y in zip(got, ref))}")
    nlib.ofd_fw_set_engine(prev)


if __name__ == "__main__":
    main()
