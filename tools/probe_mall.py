"""Does the persistent SPLAT gain when BIN's flow reads are still in the Infinity Cache?

Times SPLAT (tools/probe_tile.hip case 9) right after BIN (case 0), and after
BIN followed by a cache flush (a 1 GiB read), for several batch sizes B.  If
SPLAT per image is clearly faster without the flush at small B (flow + the
SPLAT stream inside 256 MiB), fusing BIN into the SPLAT's job queue a couple
of images ahead would pay.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import probe_tile as pt  # noqa: E402
from opticalflowfromdepth_amd import synth  # noqa: E402


def main():
    import ctypes
    pt.build()
    lib = ctypes.CDLL(pt.SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.probe_launch.argtypes = [ctypes.c_int] + [P] * 6 + [I64] * 3 + [P, I64, ctypes.c_int, P, P]
    lib.probe_slab_bytes.argtypes = [I64] * 3
    lib.probe_slab_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    H, W = 768, 1024
    flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
    acc = torch.zeros((), device=dev)
    objA, flowA, depthA = synth.stage_one_batch([12345 + i for i in range(64)], H, W, dev)
    for B in (2, 4, 8, 16, 64):
        # half disparity, half ego like the headline batch
        idx = list(range(B // 2)) + list(range(32, 32 + B - B // 2))
        obj, flow, depth = objA[idx].contiguous(), flowA[idx].contiguous(), depthA[idx].contiguous()
        C = obj.shape[1]
        out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
        slab = torch.full((lib.probe_slab_bytes(B, H, W),), 255, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        base = (obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(), valid.data_ptr(),
                coll.data_ptr(), C, H, W, slab.data_ptr(), 0, B, None, st)
        res = {}
        for mode in ("hot", "flushed", "flushed", "hot"):
            ts = []
            for _ in range(12):
                torch.cuda.synchronize()
                acc += flush.sum()  # evict everything
                assert lib.probe_launch(0, *base) == 0
                if mode == "flushed":
                    acc += flush.sum()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert lib.probe_launch(9, *base) == 0
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            res.setdefault(mode, []).append(float(np.median(ts[2:])))
        h, f = min(res["hot"]), min(res["flushed"])
        print(f"B={B:3d}: SPLAT after BIN {h:8.1f} us ({h / B:6.2f}/img), after BIN + flush {f:8.1f} us "
              f"({f / B:6.2f}/img): {100 * (f - h) / f:5.1f}% faster hot", flush=True)


if __name__ == "__main__":
    main()
