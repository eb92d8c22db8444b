"""Hole-fill phase of bench.py, one order per process, with progress lines:
python tools/hf_diag.py ORDER [B] [H W].  Prints each call's wall time and the
fault word (ofd_inpaint_faults)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, shard, synth  # noqa: E402

order = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H, W = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (768, 1024)
dev = torch.device("cuda", 0)
seeds = [shard.image_seed(i) for i in range(B)]
obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev, ego_fraction=0.5)
out = forward_warp_flow(obj, flow, depth)
torch.cuda.synchronize()
rgb = (out[0][:, 0:3] * out[1]).contiguous()
lib = _native.lib()
lib.ofd_inpaint_faults(1)
if os.environ.get("OFD_DIAG_SCHED"):
    lib.ofd_inpaint_set_schedule(*[int(v) for v in os.environ["OFD_DIAG_SCHED"].split(",")])
print(f"{order} B={B} {H}x{W} sched={os.environ.get('OFD_DIAG_SCHED')}: inputs ready", flush=True)
for k in range(4):
    t = time.perf_counter()
    ops.inpaint(rgb, out[1], out[2], order=order)
    torch.cuda.synchronize()
    print(f"  call {k}: {(time.perf_counter() - t) * 1e3:.2f} ms, faults {lib.ofd_inpaint_faults(0)}", flush=True)
