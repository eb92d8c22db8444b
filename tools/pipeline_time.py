"""Time the batched PreprocessPlusAugment on the GPU: the first stage (7 FW
calls + 5 hole-fills per image) and the 5 x 12 augment loop (45 special-flow
augmentations x (6 FW + 2 hole-fills)), B images per call, with or without
writing the 121 npz files per image.

usage: python tools/pipeline_time.py [B H W] [--save MODE ...] [--dir D]
  MODE: none (compute only), sync (np.savez_compressed in the caller, the
  reference's way, preprocess.py:446/:471), poolN:L (NpzWriter with N threads
  at zlib level L; 6 = numpy's level), gpuN (GpuNpzWriter: arrays deflated on
  the GPU, N host threads assemble and write the zips).
"""
import argparse
import os
import shutil
import sys
import tempfile
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from opticalflowfromdepth_amd import preprocess as pp, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("shape", nargs="*", type=int, default=[64, 768, 1024])
ap.add_argument("--save", nargs="*", default=["none"])
ap.add_argument("--dir", default=None)
ap.add_argument("--no-augment", action="store_true")
ap.add_argument("--ip-schedule", default=None, help="L:T -> ofd_inpaint_set_schedule(L, T) (hole-fill launch knobs)")
args = ap.parse_args()
B, H, W = (args.shape + [64, 768, 1024][len(args.shape):])[:3]
dev = torch.device("cuda:0")
if args.ip_schedule:
    from opticalflowfromdepth_amd import _native
    _native.lib().ofd_inpaint_set_schedule(*(int(v) for v in args.ip_schedule.split(":")))
seeds = [12345 + i for i in range(B)]
img0 = synth.synthetic_rgb(seeds, H, W, dev)
depth = synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64)
# warm-up: one full batch, so the timed call finds every stream's warp and
# hole-fill workspaces allocated (the steady state of a run over many batches)
_warm = pp.PreprocessPlusAugment(dev)
_warm.run_batch(seeds, img0, depth, augment=not args.no_augment)
torch.cuda.synchronize()
root = args.dir or tempfile.gettempdir()
for mode in args.save:
    workers, level = 0, 6
    if mode.startswith("pool"):
        n, level = mode[4:].split(":")
        workers, level = int(n), int(level)
    ppa = pp.PreprocessPlusAugment(dev, writer_workers=workers, compresslevel=level)
    ppa._streams = _warm._streams  # the warmed streams (their workspaces are cached per stream)
    if mode.startswith("gpu"):
        from opticalflowfromdepth_amd.npz_gpu import GpuNpzWriter
        ppa.writer = GpuNpzWriter(workers=int(mode[3:] or 8))
    out = None
    if mode != "none":
        base = tempfile.mkdtemp(prefix="ppa_", dir=root)
        out = [os.path.join(base, f"img{i}") for i in range(B)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    ppa.run_batch(seeds, img0, depth, out_dirs=out, augment=not args.no_augment)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    size = 0
    if out is not None:
        size = sum(os.path.getsize(os.path.join(d, f)) for d in out for f in os.listdir(d))
        nfiles = sum(len(os.listdir(d)) for d in out)
        shutil.rmtree(base)
    what = "stage one only" if args.no_augment else "stage one + 60 augmentations"
    print(f"{what}, save={mode}: B={B} {H}x{W}: {el:.3f} s, {B / el:.3f} images/s"
          + (f", {nfiles} files, {size / 1e9:.2f} GB written ({size / el / 1e9:.2f} GB/s)" if out else ""),
          flush=True)
    if ppa.writer is not None:
        ppa.writer.close()
