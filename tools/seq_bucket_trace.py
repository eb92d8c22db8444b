"""Per-bucket durations of the sequential fill's inner fast march (probe build
with -DOFD_BUCKET_TRACE, loaded through OFD_FW_LIB; RECORD / COLOUR are
skipped so the record area keeps the trace).  Prints, for the image with the
most buckets, the time split by bucket size.  Usage (GPU box):
  OFD_FW_LIB=tools/_probe/libofd_fw_btrace.so python tools/seq_bucket_trace.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflowfromdepth_amd import forward_warp_flow, ops, synth  # noqa: E402


def a256(x):
    return (x + 255) & ~255


B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H, W = 768, 1024
dev = torch.device("cuda:0")
seeds = [12345 + i for i in range(B)]
obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev)
out, valid, coll = forward_warp_flow(obj, flow, depth)
rgb = (out[:, 0:3] * valid).contiguous()
ops.inpaint(rgb, valid, coll, order="sequential")
torch.cuda.synchronize()
ws = ops._ip_workspaces[(dev.index, torch.cuda.current_stream().cuda_stream)]
eh, ew = H + 2, W + 2
en = eh * ew
pi = a256(en * 4) * 6 + a256(en * 8) * 2 + a256(eh * 4) + 32 * 4 + en * 160 + H * W * 4 + en * 8 + 768
G = min(B, (ws.numel() - 2048) // pi)
rec0 = 6 * a256(G * en * 4) + 2 * a256(G * en * 8) + a256(G * eh * 4) + a256(G * 32 * 4)
for march, off in (("inner", 8), ("outer", 20)):
  best = None
  for bl in range(G):
    base = rec0 + bl * en * 160
    q = (off * en + 4 * en) * 4
    nb = int(ws[base + q: base + q + 4].view(torch.int32).item())
    tr = ws[base + off * en * 4: base + off * en * 4 + nb * 32].view(torch.int32).cpu().numpy().reshape(nb, 8)
    tot = int(tr[:, 0].astype(np.int64).sum())
    if best is None or tot > best[0]:
        best = (tot, bl, nb)
  _, bl, nb = best
  base = rec0 + bl * en * 160 + off * en * 4
  tr = ws[base: base + nb * 32].view(torch.int32).cpu().numpy().reshape(nb, 8).astype(np.int64)
  dur = tr[:, 0] * 16 / 2.4e3  # us at ~2.4 GHz
  n, npush = tr[:, 1], tr[:, 2]
  print(f"{march} march, slowest image {bl}: {nb} buckets, {dur.sum() / 1e3:.2f} ms (clock 2.4 GHz assumed)")
  for lo, hi in ((0, 64), (64, 512), (512, 2048), (2048, 4096), (4096, 1 << 30)):
    sel = (n >= lo) & (n < hi)
    if sel.any():
        print(f"  keys in [{lo}, {hi}): {sel.sum():4d} buckets, {dur[sel].sum() / 1e3:6.2f} ms, "
              f"median {np.median(dur[sel]):7.1f} us, pushes {npush[sel].sum()}")
  print("  first 8 buckets (us, keys, pushes):",
        [(round(float(d), 1), int(a), int(b)) for d, a, b in zip(dur[:8], n[:8], npush[:8])])
  ph = tr[:, 4:8] * 16 / 2.4e3
  big = n > 4096
  for name, sel in (("large", big), ("small", ~big)):
      if sel.any():
          g_, so, cl, pu = (ph[sel, c].sum() / 1e3 for c in range(4))
          print(f"  {name} buckets: gather {g_:.2f}, sort {so:.2f}, claim {cl:.2f}, push {pu:.2f}, "
                f"distances+log {dur[sel].sum() / 1e3 - g_ - so - cl - pu:.2f} ms")

# Per-bucket detail of chosen images (OFD_TRACE_IMAGES="37,54"): time, keys,
# pushes, sweeps and the phase split of every bucket above 2048 keys.
for bl in [int(x) for x in os.environ.get("OFD_TRACE_IMAGES", "").split(",") if x]:
  for march, off in (("inner", 8), ("outer", 20)):
    base = rec0 + bl * en * 160
    q = (off * en + 4 * en) * 4
    nb = int(ws[base + q: base + q + 4].view(torch.int32).item())
    tr = ws[base + off * en * 4: base + off * en * 4 + nb * 32].view(torch.int32).cpu().numpy().reshape(nb, 8)
    tr = tr.astype(np.int64) & 0xFFFFFFFF
    dur = tr[:, 0] * 16 / 2.4e3
    sw = tr[:, 3] >> 16
    print(f"image {bl} {march}: {nb} buckets, {dur.sum() / 1e3:.2f} ms, sweeps {int(sw.sum())}, "
          f"keys {int(tr[:, 1].sum())}, pushes {int(tr[:, 2].sum())}")
    for r in range(nb):
        if tr[r, 1] > 2048 or r < 3:
            ph = tr[r, 4:8] * 16 / 2.4e3
            print(f"   k {int(tr[r, 3] & 0xFFFF)}: {dur[r]:.0f} us keys {int(tr[r, 1])} pushes {int(tr[r, 2])} "
                  f"sweeps {int(sw[r])} gather/sort/claim/push {[round(float(x)) for x in ph]} "
                  f"dist+log {dur[r] - ph.sum():.0f}")
