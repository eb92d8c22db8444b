"""``FW`` -- drop-in for the reference's ``alt_cuda.fw.FW`` (alt_cuda/fw.py:11-59).

Same constructor, same ``forward(obj, flow, depth) -> (output, valid, collision)``
contract as preprocess.py uses it (3-D inputs obj [C,H,W], flow [2,H,W] with
channel 0 = x, depth [1,H,W]; 3-D float32 outputs).  Additionally accepts 4-D
batched inputs ([B,C,H,W], [B,2,H,W], [B,1,H,W]) and returns 4-D outputs.

What the reference wrapper does per call -- build the pixel meshgrid on the
CPU and copy it to the device (fw.py:27-29), add the flow (fw.py:31, in the
flow's dtype), clamp (fw.py:37-38), truncate through int64 (fw.py:41-42), four
casts and contiguous copies -- happens here inside the splat kernel, in the
same arithmetic, with no temporaries and no host->device copy.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops

__all__ = ["FW", "ForwardWarp", "forward_warp"]


class FW(nn.Module):
    """Forward warping (z-buffered splat) module; no parameters, no autograd."""

    def __init__(self, device=None):
        super().__init__()
        self.device = device

    def set_shape(self, obj_shape):  # fw.py:16-17
        print(f"{obj_shape = }")

    def forward(self, obj: torch.Tensor, flow: torch.Tensor, depth: torch.Tensor):
        batched = obj.dim() == 4
        if not batched:  # fw.py:20-22
            obj, flow, depth = obj.unsqueeze(0), flow.unsqueeze(0), depth.unsqueeze(0)
        if obj.dim() != 4 or flow.dim() != 4 or depth.dim() != 4:
            raise RuntimeError("FW expects obj [C,H,W], flow [2,H,W], depth [1,H,W] (or batched 4-D)")
        # fw.py:40,43 -- obj and depth go to float32; fw.py:31 -- the add is in
        # the promoted dtype of (float32 p0, flow): float64 stays float64, every
        # other floating dtype computes in float32.
        obj = obj.to(torch.float32).contiguous()
        depth = depth.to(torch.float32).contiguous()
        if flow.dtype != torch.float64:
            flow = flow.to(torch.float32)
        flow = flow.contiguous()
        output, valid, collision = ops.forward_warp_flow(obj, flow, depth)
        if self.device is not None:  # fw.py:56-58
            output, valid, collision = output.to(self.device), valid.to(self.device), collision.to(self.device)
        if not batched:
            output, valid, collision = output.squeeze(0), valid.squeeze(0), collision.squeeze(0)
        return output, valid, collision


class ForwardWarp(torch.autograd.Function):
    """``torch.autograd.Function`` form of FW.forward (BASELINE.json north_star:
    "fw.forward_warp / torch.autograd.Function signature").  The reference
    imports ``Function`` (alt_cuda/fw.py:3) but never defines one and FW has
    no backward: a z-buffered splat selects a source per target, so there is
    no gradient to give.  ``backward`` therefore raises; valid / collision are
    marked non-differentiable."""

    @staticmethod
    def forward(ctx, obj, flow, depth):
        output, valid, collision = FW()(obj, flow, depth)
        ctx.mark_non_differentiable(valid, collision)
        return output, valid, collision

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError("forward warping has no backward (alt_cuda/fw.py defines none)")


def forward_warp(obj: torch.Tensor, flow: torch.Tensor, depth: torch.Tensor):
    """Functional FW: ``ForwardWarp.apply(obj, flow, depth) -> (output, valid, collision)``."""
    return ForwardWarp.apply(obj, flow, depth)
