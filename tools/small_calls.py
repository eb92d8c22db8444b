"""The short warp calls of the bench line, for a kernel trace (diagnostic, GPU only).

Runs, each REPS times back to back on one stream: config 2 (32 x 480x640,
C = 6, f32), config 5 f32 and bf16 (64 x 368x560), printing the wall-clock ms
per call of each.  Under ``rocprofv3 --kernel-trace --stats`` the trace shows
BIN / SPLAT durations and the gaps between them.
    rocprofv3 --kernel-trace --stats -d gpurun_out/sc -o sc -- python tools/small_calls.py
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import forward_warp_flow, synth  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    reps = int(os.environ.get("REPS", "50"))
    dev = torch.device("cuda:0")
    o2, f2, d2 = synth.stage_one_batch([12345 + i for i in range(32)], 480, 640, dev)
    out2 = (torch.empty_like(o2), torch.empty_like(d2), torch.empty_like(d2))
    o5, f5, d5 = synth.stage_one_batch([7000 + i for i in range(64)], 368, 560, dev)
    o5b = o5.to(torch.bfloat16)
    out5 = (torch.empty_like(o5), torch.empty_like(d5), torch.empty_like(d5))
    out5b = (torch.empty_like(o5b), torch.empty_like(d5), torch.empty_like(d5))
    for name, fn in (("config2 f32", lambda: forward_warp_flow(o2, f2, d2, out=out2)),
                     ("config5 f32", lambda: forward_warp_flow(o5, f5, d5, out=out5)),
                     ("config5 bf16", lambda: forward_warp_flow(o5b, f5, d5, out=out5b))):
        print(f"{name}: {timed(fn, reps):.4f} ms per call", flush=True)
        time.sleep(0.05)  # a visible gap between the groups in the trace


if __name__ == "__main__":
    main()
