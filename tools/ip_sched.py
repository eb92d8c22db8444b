"""Hole-fill schedule sweep (diagnostic, GPU only): ofd_inpaint_set_schedule(launch_layers, thin_cap).

Times ops.inpaint on the headline warped batch (64 x 768x1024, tools/ip_time.py's
input) for each (launch_layers, thin_cap) pair given on the command line as
L:T (-1 = the library default), interleaved over rounds, and checks every
schedule's output equals the default's bit for bit.
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, synth  # noqa: E402


def main():
    scheds = [tuple(int(v) for v in a.split(":")) for a in (sys.argv[1:] or ["-1:-1", "8:-1", "32:-1"])]
    dev = torch.device("cuda:0")
    seeds = [12345 + i for i in range(64)]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    lib = _native.lib()
    lib.ofd_inpaint_set_schedule(-1, -1)
    ref = ops.inpaint(rgb, valid, coll)
    ops.inpaint(rgb, valid, coll)
    torch.cuda.synchronize()
    times = {s: [] for s in scheds}
    for rnd in range(5):
        for s in scheds:
            lib.ofd_inpaint_set_schedule(*s)
            r = ops.inpaint(rgb, valid, coll)  # one call to settle the lagged statistics
            torch.cuda.synchronize()
            if rnd == 0:
                assert torch.equal(r, ref), f"schedule {s} differs"
            t = time.perf_counter()
            for _ in range(3):
                ops.inpaint(rgb, valid, coll)
            torch.cuda.synchronize()
            times[s].append((time.perf_counter() - t) / 3 * 1e3)
    lib.ofd_inpaint_set_schedule(-1, -1)
    for s in scheds:
        print(f"launch_layers {s[0]:4d} thin_cap {s[1]:7d}: median {np.median(times[s]):7.3f} ms "
              f"(min {min(times[s]):7.3f})", flush=True)


if __name__ == "__main__":
    main()
