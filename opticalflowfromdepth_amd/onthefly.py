"""On-the-fly training pairs inside a RAFT-style or GMFlow-style train loop
(BASELINE.json configs[4]).

The reference trains on pairs preprocess.py wrote to npz beforehand:
adjusted_RAFT/train.py:184-211 pulls (image1, image2, flow, ..., valid) from a
DataLoader over those files (dataloader.py:243-251 -> np.load), adds noise
(:188-191), runs the model, takes sequence_loss (:51-76), then backward, clip,
step (:205-211) under nn.DataParallel (:143).  Here the collated batch is
(image, raw depth, camera draw) and the pair is made in the training process,
on the GPU, after collation:

    depth  = normalize_depth(raw)                         utils.py:102-116
    flow   = disparity flow (preprocess.py:239-254) or ego-motion flow
             (:265-298 with geometry.py:17-67), per image
    image2 = FW(image1 bf16, flow, depth) * valid, holes filled   :358-366
    valid  = source pixels whose target lies inside the image

with the bf16 warp (ops.forward_warp_flow on a bfloat16 obj) and the GPU
hole-fill (ops.inpaint), then the step of train.py:185-211 under
DistributedDataParallel over RCCL (one process per GPU, torchrun env) instead
of DataParallel.  The flow network is a small stand-in with RAFT's interface
(model(image1, image2, iters) -> list of full-resolution flows); RAFT itself is
out of scope.  The GMFlow loop (adjusted_gmflow/main.py:450-494)
is ``gmflow_train_step`` with ``flow_loss_func`` (adjusted_gmflow/loss.py) and
a global-matching stand-in, ``GlobalMatchFlowNet`` (``--arch gmflow``).

``PairOps`` carries the three device ops; the CPU multi-rank test
(tests/test_onthefly.py) swaps in the CPU restatements kept under oracle/, the product
default is the HIP path and fails loudly without it.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import synth

MAX_FLOW = 400  # adjusted_RAFT/train.py:46


# ---------------------------------------------------------------- data
class SyntheticDepthImages(torch.utils.data.Dataset):
    """Stands in for the image/depth readers (dataloader.py:13-58): item i is
    (rgb [3,H,W] float32 integer-valued, raw depth [1,H,W] float32, s, T [4,4],
    kind) for seed ``base + i``; kind 0 = disparity flow, 1 = ego-motion."""

    def __init__(self, n: int, h: int, w: int, base: int = 0):
        self.n, self.h, self.w, self.base = n, h, w, base

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        seed = self.base + int(i)
        depth = torch.from_numpy(synth.synthetic_depth_np(self.h, self.w, seed)).view(1, self.h, self.w)
        rgb = torch.from_numpy(np.floor(np.random.default_rng(seed + 1000).uniform(0, 256, (3, self.h, self.w)))
                               .astype(np.float32))
        s, T = synth.batch_camera_params([seed])
        return rgb, depth, s[0], T[0], torch.tensor(seed % 2)


# ---------------------------------------------------------------- pairs
def _gpu_ego_flow(depth, T):
    from . import ops
    P, ik = synth.projection(depth.shape[-2], depth.shape[-1], T, depth.device)
    return ops.ego_flow(depth, P, ik)


def _gpu_warp(obj, flow, depth):
    from . import ops
    return ops.forward_warp_flow(obj, flow, depth)


def _gpu_fill(img, valid, coll):
    from . import ops
    return ops.inpaint(img, valid, coll)


@dataclass
class PairOps:
    """The device ops a pair needs: warp(obj, flow, depth) -> (out, valid,
    collision) (alt_cuda/fw.py:27-54), ego_flow(depth [B,1,H,W], T [B,4,4]) ->
    flow [B,2,H,W] float32, fill(img, valid, collision) -> float32 image
    (utils.py:136-151)."""
    warp: Callable = _gpu_warp
    ego_flow: Callable = _gpu_ego_flow
    fill: Callable = _gpu_fill


def make_pairs(rgb, raw_depth, s, T, kind, ops: PairOps = PairOps(), dtype=torch.bfloat16):
    """(image1, image2, flow, valid) for a collated batch already on the device.

    image1 / image2 in ``dtype`` (integer values 0..255 are exact in bf16),
    flow [B,2,H,W] float32 (image1 -> image2), valid [B,H,W] float32."""
    B, _, H, W = rgb.shape
    depth = synth.normalize_depth(raw_depth.to(torch.float32))
    # both flows for every image, selected per image: no host round trip to
    # split the batch (the ego flow is one elementwise pass)
    flow = torch.where(kind.to(torch.bool).view(B, 1, 1, 1), ops.ego_flow(depth.contiguous(), T),
                       synth.disparity_flow(depth, s).to(torch.float32)).contiguous()
    image1 = rgb.to(dtype).contiguous()
    out, warped_valid, coll = ops.warp(image1, flow, depth.contiguous())
    image2 = ops.fill((out.to(torch.float32) * warped_valid), warped_valid, coll).to(dtype)
    # the reference training data's supervision mask (adjusted_RAFT/core/datasets.py:282-288):
    # flow components under 1000 px, and no sky / invalid depth (normalize_depth's sentinel 100)
    valid = ((flow[:, 0].abs() < 1000) & (flow[:, 1].abs() < 1000) & (depth[:, 0] != 100)).to(torch.float32)
    return image1, image2, flow, valid


# ---------------------------------------------------------------- model
class IterativeFlowNet(nn.Module):
    """A small RAFT-shaped flow network: shared encoder at 1/4 resolution, an
    update block applied ``iters`` times to a running flow, every iterate
    upsampled to full resolution (RAFT's forward contract, adjusted_RAFT/core/raft.py)."""

    def __init__(self, dim: int = 64):
        super().__init__()
        self.enc = nn.Sequential(nn.Conv2d(3, 32, 7, 2, 3), nn.ReLU(inplace=True),
                                 nn.Conv2d(32, dim, 3, 2, 1), nn.ReLU(inplace=True))
        self.update = nn.Sequential(nn.Conv2d(2 * dim + 2, dim, 3, 1, 1), nn.ReLU(inplace=True),
                                    nn.Conv2d(dim, 2, 3, 1, 1))

    def forward(self, image1, image2, iters: int = 4) -> List[torch.Tensor]:
        x = torch.cat((image1, image2), 0)
        x = 2 * (x / 255.0) - 1.0
        f = self.enc(x)
        f1, f2 = f.chunk(2, 0)
        B, _, h, w = f1.shape
        flow = torch.zeros(B, 2, h, w, device=f1.device, dtype=f1.dtype)
        preds = []
        for _ in range(iters):
            flow = flow + self.update(torch.cat((f1, f2, flow), 1))
            preds.append(F.interpolate(flow * 4, scale_factor=4, mode="bilinear", align_corners=True))
        return preds


def sequence_loss(flow_preds, flow_gt, valid, gamma=0.8, max_flow=MAX_FLOW):
    """adjusted_RAFT/train.py:51-76: gamma-weighted L1 over the iterates on
    valid pixels with |flow| < max_flow; returns (loss, metrics tensors)."""
    n = len(flow_preds)
    mag = torch.sum(flow_gt ** 2, dim=1).sqrt()
    valid = (valid >= 0.5) & (mag < max_flow)
    loss = 0.0
    for i in range(n):
        w = gamma ** (n - i - 1)
        loss = loss + w * (valid[:, None] * (flow_preds[i].float() - flow_gt).abs()).mean()
    epe = torch.sum((flow_preds[-1].float() - flow_gt) ** 2, dim=1).sqrt().view(-1)[valid.view(-1)]
    return loss, {"epe": epe.mean(), "1px": (epe < 1).float().mean(), "3px": (epe < 3).float().mean(),
                  "5px": (epe < 5).float().mean()}


# ---------------------------------------------------------------- step
@dataclass
class StepArgs:
    iters: int = 4
    gamma: float = 0.8
    clip: float = 1.0
    add_noise: bool = False
    amp: bool = True  # bf16 autocast for the network (the warp is bf16 regardless)


def train_step(model, optimizer, scheduler, batch, device, args: StepArgs, ops: PairOps = PairOps(),
               dtype=torch.bfloat16, pair=None):
    """One iteration of adjusted_RAFT/train.py:185-211 on a collated batch of
    (rgb, raw depth, s, T, kind); the pair is warped on the fly (make_pairs),
    or passed in ready (``pair``, e.g. from a PairPrefetcher).
    Returns the loss and metrics as tensors (no host sync)."""
    optimizer.zero_grad(set_to_none=True)
    if pair is None:
        rgb, raw, s, T, kind = [x.to(device, non_blocking=True) for x in batch]
        pair = make_pairs(rgb, raw, s, T, kind, ops, dtype)
    image1, image2, flow, valid = pair
    if args.add_noise:  # :188-191
        stdv = np.random.uniform(0.0, 5.0)
        image1 = (image1.float() + stdv * torch.randn(image1.shape, device=device)).clamp(0.0, 255.0)
        image2 = (image2.float() + stdv * torch.randn(image2.shape, device=device)).clamp(0.0, 255.0)
    dev_type = torch.device(device).type
    with torch.autocast(dev_type, dtype=torch.bfloat16, enabled=args.amp):
        preds = model(image1.float(), image2.float(), iters=args.iters)
    loss, metrics = sequence_loss(preds, flow, valid, args.gamma)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip)
    optimizer.step()
    if scheduler is not None:
        scheduler.step()
    return loss.detach(), {k: v.detach() for k, v in metrics.items()}


def fetch_optimizer(model, lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100):
    """adjusted_RAFT/train.py:83-90: AdamW + OneCycleLR."""
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wdecay, eps=epsilon)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, lr, num_steps + 100, pct_start=0.05, cycle_momentum=False,
                                                anneal_strategy="linear")
    return opt, sched


def shard_loader(n_images, h, w, batch, rank, world, base=0, workers=0):
    """Rank r's share of the synthetic images (indices r::world), collated."""
    ds = SyntheticDepthImages(n_images, h, w, base)
    idx = list(range(rank, n_images, world))
    return torch.utils.data.DataLoader(torch.utils.data.Subset(ds, idx), batch_size=batch, shuffle=False,
                                       num_workers=workers, drop_last=True)


# ---------------------------------------------------------------- GMFlow-style step
# adjusted_gmflow/main.py:450-494 trains GMFlow on the same npz pairs with its
# own loss (adjusted_gmflow/loss.py:4-37), AdamW(lr 4e-4, weight decay 1e-4,
# :230-231), a cosine OneCycleLR over num_steps + 10 (:425-432), clip 1.0
# (:51, :489), and skips a step whose loss is NaN (:479-480).  GMFlow itself is
# out of scope like RAFT; the stand-in below has its forward contract
# (model(img1, img2, attn_splits_list, corr_radius_list, prop_radius_list) ->
# {'flow_preds': [...]}) and its core operation, global matching.
GMFLOW_MAX_FLOW = 400  # adjusted_gmflow/main.py:39


def flow_loss_func(flow_preds, flow_gt, valid, gamma=0.9, max_flow=GMFLOW_MAX_FLOW):
    """adjusted_gmflow/loss.py:4-37: gamma-weighted L1 over the predictions on
    valid pixels with |flow| < max_flow; metrics count epe ABOVE 1 / 3 / 5 px
    (RAFT's sequence_loss counts below).  Metrics stay tensors (no host sync)."""
    n = len(flow_preds)
    mag = torch.sum(flow_gt ** 2, dim=1).sqrt()
    valid = (valid >= 0.5) & (mag < max_flow)
    loss = 0.0
    for i in range(n):
        w = gamma ** (n - i - 1)
        loss = loss + w * (valid[:, None] * (flow_preds[i].float() - flow_gt).abs()).mean()
    epe = torch.sum((flow_preds[-1].float() - flow_gt) ** 2, dim=1).sqrt().view(-1)[valid.view(-1)]
    return loss, {"epe": epe.mean(), "1px": (epe > 1).float().mean(), "3px": (epe > 3).float().mean(),
                  "5px": (epe > 5).float().mean()}


class GlobalMatchFlowNet(nn.Module):
    """A small GMFlow-shaped network: features at 1/8 resolution, global
    matching (softmax over every position of image 2 of the scaled feature
    correlation; flow = expected match - position), one convolutional
    refinement; each flow upsampled x8 to full resolution, returned as
    {'flow_preds': [matching, refined]} (adjusted_gmflow/gmflow/gmflow.py)."""

    def __init__(self, dim: int = 64):
        super().__init__()
        self.enc = nn.Sequential(nn.Conv2d(3, 32, 7, 2, 3), nn.ReLU(inplace=True),
                                 nn.Conv2d(32, 48, 3, 2, 1), nn.ReLU(inplace=True),
                                 nn.Conv2d(48, dim, 3, 2, 1))
        self.refine = nn.Sequential(nn.Conv2d(dim + 2, dim, 3, 1, 1), nn.ReLU(inplace=True),
                                    nn.Conv2d(dim, 2, 3, 1, 1))

    @staticmethod
    def _up8(flow):
        return F.interpolate(flow * 8, scale_factor=8, mode="bilinear", align_corners=True)

    def forward(self, img1, img2, attn_splits_list=None, corr_radius_list=None, prop_radius_list=None):
        x = torch.cat((img1, img2), 0) / 255.0
        mean = x.new_tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)  # gmflow/utils.py normalize_img
        std = x.new_tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
        f = self.enc((x - mean) / std)
        f1, f2 = f.chunk(2, 0)
        B, C, h, w = f1.shape
        ys, xs = torch.meshgrid(torch.arange(h, device=f.device, dtype=f.dtype),
                                torch.arange(w, device=f.device, dtype=f.dtype), indexing="ij")
        grid = torch.stack((xs, ys), -1).view(1, h * w, 2)
        corr = torch.bmm(f1.flatten(2).transpose(1, 2), f2.flatten(2)) / C ** 0.5  # [B, hw, hw]
        match = torch.bmm(torch.softmax(corr, -1), grid.expand(B, -1, -1).to(corr.dtype))
        flow = (match - grid).transpose(1, 2).reshape(B, 2, h, w)
        preds = [self._up8(flow)]
        flow = flow + self.refine(torch.cat((f1, flow.to(f1.dtype)), 1))
        preds.append(self._up8(flow))
        return {"flow_preds": preds}


def nan_on_any_rank(loss: torch.Tensor) -> bool:
    """main.py:479-480 skips a step whose loss is NaN.  Under DDP with more
    than one rank the skip must be collective: a rank that skipped backward
    alone would leave the others blocked in the gradient all-reduce.  So the
    NaN flag is all-reduced (MAX) and every rank skips together (the one
    host sync of the step, as in the reference)."""
    import torch.distributed as dist
    nan = torch.isnan(loss.detach()).reshape(1).to(torch.float32)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo":
            nan = nan.cpu()
        dist.all_reduce(nan, op=dist.ReduceOp.MAX)
    return bool(nan.item() > 0)


def fetch_gmflow_optimizer(model, lr=4e-4, weight_decay=1e-4, num_steps=100):
    """adjusted_gmflow/main.py:230-231, :425-432: AdamW + cosine OneCycleLR."""
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, lr, num_steps + 10, pct_start=0.05, cycle_momentum=False,
                                                anneal_strategy="cos")
    return opt, sched


def gmflow_train_step(model, optimizer, lr_scheduler, batch, device, args: StepArgs = StepArgs(gamma=0.9),
                      ops: PairOps = PairOps(), dtype=torch.bfloat16, grad_clip=1.0,
                      max_flow=GMFLOW_MAX_FLOW, pair=None):
    """One iteration of adjusted_gmflow/main.py:450-494 on a collated batch
    of (rgb, raw depth, s, T, kind), the pair warped on the fly (make_pairs)
    or passed in ready (``pair``).
    Returns (loss, metrics) as tensors, or None for a step the reference skips
    (a NaN loss, :479-480: no update, no scheduler step -- the one host sync)."""
    if pair is None:
        rgb, raw, s, T, kind = [x.to(device, non_blocking=True) for x in batch]
        pair = make_pairs(rgb, raw, s, T, kind, ops, dtype)
    image1, image2, flow_gt, valid = pair
    dev_type = torch.device(device).type
    with torch.autocast(dev_type, dtype=torch.bfloat16, enabled=args.amp):
        results = model(image1.float(), image2.float(), attn_splits_list=[2], corr_radius_list=[-1],
                        prop_radius_list=[-1])
    loss, metrics = flow_loss_func(results["flow_preds"], flow_gt, valid, gamma=args.gamma, max_flow=max_flow)
    if nan_on_any_rank(loss):
        return None
    for p in model.parameters():  # :483-485
        p.grad = None
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), grad_clip)
    optimizer.step()
    if lr_scheduler is not None:
        lr_scheduler.step()
    return loss.detach(), {k: v.detach() for k, v in metrics.items()}


# ---------------------------------------------------------------- pair prefetch
class PairPrefetcher:
    """Builds the next steps' pairs on side streams while the current step
    trains: the cv2-order hole-fill holds one workgroup per image (its time
    is the deepest image's chain), so the network's kernels and other pairs'
    fills run beside it on the rest of the chip.  ``put(batch)`` starts a
    pair (round-robin over ``streams`` side streams); ``get(batch)`` returns
    the pair for ``batch`` (built earlier by ``put`` or now), with the
    caller's stream ordered after it and its tensors marked as used there."""

    def __init__(self, device, ops: PairOps = PairOps(), dtype=torch.bfloat16, streams: int = 2):
        self.device, self.ops, self.dtype = torch.device(device), ops, dtype
        self.sides = [torch.cuda.Stream(self.device) for _ in range(streams)] if self.device.type == "cuda" else []
        self.pending = {}  # id(batch) -> (batch, pair, event)
        self.k = 0

    def _build(self, batch):
        xs = [x.to(self.device, non_blocking=True) for x in batch]
        return make_pairs(*xs, ops=self.ops, dtype=self.dtype)

    def put(self, batch):
        if id(batch) in self.pending:
            return
        if not self.sides:
            self.pending[id(batch)] = (batch, self._build(batch), None)
            return
        side = self.sides[self.k % len(self.sides)]
        self.k += 1
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            pair = self._build(batch)
            ev = torch.cuda.Event()
            ev.record(side)
        self.pending[id(batch)] = (batch, pair, ev)

    def get(self, batch):
        if id(batch) not in self.pending:
            self.put(batch)
        _, pair, ev = self.pending.pop(id(batch))
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in pair:
                t.record_stream(cur)
        return pair


# ---------------------------------------------------------------- driver
def main(argv: Optional[Sequence[str]] = None):
    """torchrun entry: one process per GPU, DDP over RCCL (backend "nccl").

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m opticalflowfromdepth_amd.onthefly --steps 20"""
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per rank per step")
    ap.add_argument("--size", type=int, nargs=2, default=(368, 560))
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--arch", choices=("raft", "gmflow"), default="raft",
                    help="train step of adjusted_RAFT/train.py or adjusted_gmflow/main.py")
    ap.add_argument("--no-prefetch", action="store_true", help="build each pair in the step (no side stream)")
    a = ap.parse_args(argv)
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # DDP over RCCL whenever a launcher started this process (one rank included)
    pg = world > 1 or "WORLD_SIZE" in os.environ
    if pg:
        dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(0)
    gm = a.arch == "gmflow"
    model = (GlobalMatchFlowNet() if gm else IterativeFlowNet()).to(dev)
    if pg:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[local])
    opt, sched = (fetch_gmflow_optimizer if gm else fetch_optimizer)(model, num_steps=a.steps + a.warmup)
    h, w = a.size
    total = a.steps + a.warmup
    loader = shard_loader(a.batch * world * total, h, w, a.batch, rank, world, workers=a.workers)
    args = StepArgs(iters=a.iters, gamma=0.9) if gm else StepArgs(iters=a.iters)

    ahead = int(os.environ.get("OFD_PAIRS_AHEAD", "2"))  # pairs in flight beside the current step
    pf = None if a.no_prefetch else PairPrefetcher(dev, streams=max(ahead, 1))

    def step(b, nxt=()):
        pair = None
        if pf is not None:
            for n in nxt:
                pf.put(n)  # the next steps' pairs build on the side streams during this step
            pair = pf.get(b)
        if gm:
            r = gmflow_train_step(model, opt, sched, b, dev, args, pair=pair)
            return r if r is not None else (torch.tensor(float("nan")), {"epe": torch.tensor(float("nan"))})
        return train_step(model, opt, sched, b, dev, args, pair=pair)

    it = iter(loader)
    batches = [next(it) for _ in range(total)]  # host-side data ready: the step is what is timed
    warm = batches[:a.warmup]
    for i, b in enumerate(warm):
        step(b, warm[i + 1:i + 1 + ahead])
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    t0 = time.perf_counter()
    timed = batches[a.warmup:]
    for i, b in enumerate(timed):
        loss, m = step(b, timed[i + 1:i + 1 + ahead])
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev)
    # the pair builder alone over the same (device-resident) batches
    resident = [[x.to(dev) for x in b] for b in batches[a.warmup:]]
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for b in resident:
        make_pairs(*b)
    torch.cuda.synchronize()
    el_pairs = time.perf_counter() - t1
    if pg:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        pairs = a.steps * a.batch * world
        print(json.dumps({"metric": "training pairs/s (on-the-fly bf16 warp + step)", "arch": a.arch,
                          "pair_prefetch": not a.no_prefetch,
                          "value": pairs / el.item(),
                          "n_gpus": world, "steps": a.steps, "ms_per_step": el.item() / a.steps * 1e3,
                          "pairs_ms_per_step": el_pairs / a.steps * 1e3,
                          "loss": float(loss), "epe": float(m["epe"]), "config": {"size": [h, w],
                                                                                   "batch_per_rank": a.batch}}))
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
