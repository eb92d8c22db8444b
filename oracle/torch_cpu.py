"""oracle/torch_cpu.py -- TEST INFRASTRUCTURE ONLY (CPU baseline leg).

The PyTorch-CPU formulation of the reference forward warp that BASELINE.md §3
names as part 3 of the CPU baseline: the reference has no CPU path
(alt_cuda/fw_cuda.cpp:11,20-23 reject non-CUDA tensors), so the "PyTorch-CPU
warp" is this restatement, timed by bench.py beside the C loop of
fw_oracle.c.  Only tests/ and bench.py's cpu_baseline leg import it.

    fw_flow_scatter(obj, flow, depth)
        FW.forward (alt_cuda/fw.py:27-43: meshgrid + flow in the flow's dtype,
        clamp, truncation through int64) followed by the z-buffer of
        alt_cuda/fw_cuda_kernel.cu:28-47 written as one
        ``scatter_reduce_(..., "amin")`` over 64-bit keys
        (orderable(depth) << 32 | raster index, the lexicographic minimum the
        serial loop computes -- SURVEY.md 0.1 item 1) and one gather.

Bit-identical to oracle.fw_flow (tests/test_oracle.py checks it).  The flow
synthesis half of the baseline (geometry.py depth -> flow on torch-CPU) is
opticalflowfromdepth_amd.synth.ego_motion_flow / disparity_flow run on CPU
tensors, which restate geometry.py:17-67 / preprocess.py:239-298.
"""
from __future__ import annotations

import torch

_I64_MAX = torch.iinfo(torch.int64).max
_UNTOUCHED = _I64_MAX          # no source landed
_NOWIN = _I64_MAX - 1          # landed, none with depth < 1000 (collision)


def _signed_orderable(d: torch.Tensor) -> torch.Tensor:
    """float32 -> int64 in [-2^31, 2^31) with the order of the floats, -0 == +0."""
    d = torch.where(d == 0, torch.zeros_like(d), d)  # -0 -> +0
    u = d.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    neg = (u & 0x80000000) != 0
    o = torch.where(neg, (~u) & 0xFFFFFFFF, u | 0x80000000)  # unsigned orderable
    return o - 0x80000000                                    # shift into signed range


def fw_flow_scatter(obj: torch.Tensor, flow: torch.Tensor, depth: torch.Tensor):
    """Batched FW.forward on CPU tensors: obj [B,C,H,W], flow [B,2,H,W]
    (float32 or float64), depth [B,1,H,W] -> (output, valid, collision) float32."""
    obj = obj.to(torch.float32)
    depth = depth.to(torch.float32)
    if flow.dtype != torch.float64:
        flow = flow.to(torch.float32)
    B, C, H, W = obj.shape
    HW = H * W
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                            indexing="ij")
    px = xs.to(flow.dtype) + flow[:, 0]                       # fw.py:31
    py = ys.to(flow.dtype) + flow[:, 1]
    ok = ~(torch.isnan(px) | torch.isnan(py))                # NaN: dropped (DESIGN.md "Defined behaviour")
    px = px.clamp(0, W - 1).nan_to_num(0).to(torch.int64)    # fw.py:37-42 (trunc through int64)
    py = py.clamp(0, H - 1).nan_to_num(0).to(torch.int64)
    t = (py * W + px).reshape(B, HW)
    d = depth.reshape(B, HW)
    src = torch.arange(HW, dtype=torch.int64).expand(B, HW)
    key = torch.where(d < 1000, (_signed_orderable(d) << 32) | src, torch.full_like(src, _NOWIN))
    okf = ok.reshape(B, HW)
    t = torch.where(okf, t, torch.full_like(t, HW))          # dropped sources land in a spill slot
    best = torch.full((B, HW + 1), _UNTOUCHED, dtype=torch.int64)
    best.scatter_reduce_(1, t, key, reduce="amin", include_self=True)
    best = best[:, :HW]
    valid = best != _UNTOUCHED
    win = valid & (best != _NOWIN)
    widx = torch.where(win, best & 0xFFFFFFFF, torch.zeros_like(best))
    out = torch.gather(obj.reshape(B, C, HW), 2, widx.unsqueeze(1).expand(B, C, HW))
    out = torch.where(win.unsqueeze(1), out, torch.zeros_like(out))
    return (out.reshape(B, C, H, W), valid.to(torch.float32).reshape(B, 1, H, W),
            (valid & ~win).to(torch.float32).reshape(B, 1, H, W))
