"""Time the batched PreprocessPlusAugment on the GPU (no npz writing): the
first stage (7 FW calls + 5 hole-fills per image) and the 5 x 12 augment loop
(45 special-flow augmentations x (6 FW + 2 hole-fills)), B images per call."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from opticalflowfromdepth_amd import preprocess as pp, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (768, 1024)
dev = torch.device("cuda:0")
seeds = [12345 + i for i in range(B)]
img0 = synth.synthetic_rgb(seeds, H, W, dev)
depth = synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64)
ppa = pp.PreprocessPlusAugment(dev)
ppa.run_batch(seeds[:2], img0[:2], depth[:2], augment=False)  # warm-up
for aug in (False, True):
    torch.cuda.synchronize()
    t = time.perf_counter()
    ppa.run_batch(seeds, img0, depth, augment=aug)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(f"{'stage one + 60 augmentations' if aug else 'stage one only'}: B={B} {H}x{W}: {el:.3f} s, "
          f"{B / el:.2f} images/s", flush=True)
