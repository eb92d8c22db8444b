"""Persistent SPLAT tile order variants (OFD_TILE_ORDER) at the headline workload (diagnostic, GPU only).

Builds tools/probe_tile.hip once per order on the CPU side (python tools/probe_order.py build),
then on the GPU times BIN + persistent SPLAT of each variant, interleaved over rounds, and checks
every variant's output against the product library's.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ORDERS = [int(x) for x in os.environ.get("ORDERS", "0,1,3").split(",")]


def so(order):
    return os.path.join(REPO, "tools", "_build", f"libprobe_tile_o{order}.so")


def build():
    os.makedirs(os.path.join(REPO, "tools", "_build"), exist_ok=True)
    for o in ORDERS:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        f"-DOFD_TILE_ORDER={o}", "-I", os.path.join(REPO, "include"), "-o", so(o),
                        os.path.join(REPO, "tools", "probe_tile.hip")], check=True)


def main():
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), 768, 1024
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev)
    C = obj.shape[1]
    ref = forward_warp_flow(obj, flow, depth)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    libs = {}
    for o in ORDERS:
        lib = ctypes.CDLL(so(o))
        lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
        lib.probe_slab_bytes.argtypes = [I64] * 3
        lib.probe_slab_bytes.restype = ctypes.c_size_t
        out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
        slab = torch.full((lib.probe_slab_bytes(B, H, W),), 255, dtype=torch.uint8, device=dev)
        base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(),
                coll.data_ptr(), C, H, W, slab.data_ptr(), 0, B, None, torch.cuda.current_stream().cuda_stream)
        libs[o] = (lib, base, (out, valid, coll), slab)

    def run(o):
        lib, base, _, _ = libs[o]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        assert lib.probe_launch(0, *base) == 0
        ev[1].record()
        assert lib.probe_launch(9, *base) == 0
        ev[2].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e3, ev[1].elapsed_time(ev[2]) * 1e3

    for o in ORDERS:
        run(o)
        ok = all(torch.equal(x, y) for x, y in zip(libs[o][2], ref))
        print(f"order {o}: result == product: {ok}", flush=True)
    t = {o: [] for o in ORDERS}
    for _ in range(int(os.environ.get("ROUNDS", "15"))):
        for o in ORDERS:
            t[o].append(run(o))
    for o in ORDERS:
        a = np.array(t[o])
        print(f"order {o}: BIN {np.median(a[:, 0]):6.1f} us  SPLAT {np.median(a[:, 1]):6.1f} us "
              f"(min {a[:, 1].min():6.1f})  sum {np.median(a.sum(1)):6.1f} us", flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    else:
        main()
