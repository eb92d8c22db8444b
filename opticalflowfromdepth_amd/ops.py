"""Torch-facing forward-warp ops over the C ABI (include/ofd_fw.h).

``forward_warping`` mirrors the reference extension op
``fw_cuda.forward_warping(obj, safe_y, safe_x, depth) -> [output, valid, collision]``
(alt_cuda/fw_cuda.cpp:15-30, alt_cuda/fw_cuda_kernel.cu:52-83): same argument
meaning, same checks and messages, same outputs, for any batch size B.

``forward_warp_flow`` is the batched FW.forward path (alt_cuda/fw.py:19-59)
with the coordinate arithmetic fused into the splat kernel.

``warp_disparity`` / ``warp_ego`` fuse the first stage's flow synthesis into
the warp (preprocess.py:356-359 / :371-373, :385-387); ``ego_flow`` is the
ego-motion flow plane alone (preprocess.py:265-298).

``inpaint`` is the batched hole-fill that replaces ``utils.inpaint``
(utils.py:136-151): by default cv2's sequential Telea order run on the GPU
(csrc/ofd_inpaint_seq.hip, ``order="sequential"``), or the faster layered
re-specification (csrc/ofd_inpaint.hip, ``order="layered"``).

Both launch asynchronously on the current HIP stream of the input's device.
There is no CPU path: the reference raises for non-GPU tensors
(fw_cuda.cpp:11) and so does this module.
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import List, Tuple

import torch

from . import _native

_F32, _F64, _BF16 = torch.float32, torch.float64, torch.bfloat16

# Reusable key workspaces, one per (device, stream) -- a workspace is
# stream-ordered scratch, so two streams never share one; each call leaves its
# workspace in the initial all-ones state (see include/ofd_fw.h).  The caches
# are LRU-bounded: a caller that creates a stream per call or per worker
# recycles workspaces instead of keeping one (~0.3-0.7 GB at 64 images of
# 768x1024) per stream ever seen.  A dropped workspace was allocated on its
# stream, so the caching allocator hands its memory out again only in that
# stream's order.
_ws_lock = threading.Lock()
# (8: the pipeline's caller stream and three augmentation streams, plus a
# few more, keep their workspaces; OFD_WS_CACHE_MAX overrides)
_WS_CACHE_MAX = int(os.environ.get("OFD_WS_CACHE_MAX", "8"))
_workspaces: "OrderedDict[Tuple[int, int], torch.Tensor]" = OrderedDict()
# hole-fill scratch, one per (device, stream); needs no initialisation
_ip_workspaces: "OrderedDict[Tuple[int, int], torch.Tensor]" = OrderedDict()


# bytes all cached workspaces of one kind may hold together (the hole-fill's
# reach ~21 GB per stream at 128 images of 768x1024): least recently used
# entries beyond it are dropped, the newest one always stays
_WS_CACHE_BYTES = int(float(os.environ.get("OFD_WS_CACHE_GB", "128")) * (1 << 30))


def _cache_put(cache: OrderedDict, key, ws: torch.Tensor) -> None:
    cache[key] = ws
    cache.move_to_end(key)
    while len(cache) > _WS_CACHE_MAX:
        cache.popitem(last=False)
    while len(cache) > 1 and sum(t.numel() for t in cache.values()) > _WS_CACHE_BYTES:
        cache.popitem(last=False)


def _check_input(x: torch.Tensor, name: str) -> None:
    # fw_cuda.cpp:11-13 (CHECK_CUDA / CHECK_CONTIGUOUS)
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not x.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def workspace(device: torch.device, nbytes: int, stream: torch.cuda.Stream) -> torch.Tensor:
    """A >= nbytes initialised key workspace for (device, stream)."""
    key = (device.index, stream.cuda_stream)
    with _ws_lock:
        ws = _workspaces.get(key)
        if ws is None or ws.numel() < nbytes:
            _workspaces.pop(key, None)  # release the smaller one before allocating
            ws = None
            with torch.cuda.device(device), torch.cuda.stream(stream):
                ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
            _native.check(_native.lib().ofd_fw_workspace_init(ws.data_ptr(), ws.numel(), stream.cuda_stream),
                          "ofd_fw_workspace_init")
        _cache_put(_workspaces, key, ws)
        return ws


def _ws_bytes(B: int, H: int, W: int, f64: bool) -> int:
    return int(_native.lib().ofd_fw_workspace_bytes(B, H, W, 1 if f64 else 0))


def _check_out(out, shapes, dtypes, dev):
    """Validate caller-supplied (output, valid, collision) like forward_warp_flow does."""
    if len(out) != 3:
        raise RuntimeError("out must be (output, valid, collision)")
    for x, n, shp, dt in zip(out, ("output", "valid", "collision"), shapes, dtypes):
        _check_input(x, n)
        if tuple(x.shape) != tuple(shp) or x.dtype != dt or x.device != dev:
            raise RuntimeError(f"out {n} must be {dt} {tuple(shp)} on {dev}")
    return out


def forward_warping(obj: torch.Tensor, safe_y: torch.Tensor, safe_x: torch.Tensor,
                    depth: torch.Tensor) -> List[torch.Tensor]:
    """Drop-in for ``fw_cuda.forward_warping`` (alt_cuda/fw_cuda.cpp:15-26).

    obj [B,C,H,W]; safe_y, safe_x, depth [B,1,H,W]; one float dtype (float32 or
    float64) for all four.  Coordinates are truncated toward zero as the
    reference's accessor indexing does.  Returns ``[output, valid, collision]``
    with output [B,C,H,W] and valid/collision [B,1,H,W] in that dtype.
    """
    for x, n in ((obj, "obj"), (safe_y, "safe_y"), (safe_x, "safe_x"), (depth, "depth")):
        _check_input(x, n)
    if obj.dim() != 4:
        raise RuntimeError(f"obj must be 4-D [B,C,H,W], got {obj.dim()}-D")
    B, C, H, W = obj.shape
    for x, n in ((safe_y, "safe_y"), (safe_x, "safe_x"), (depth, "depth")):
        if tuple(x.shape) != (B, 1, H, W):
            raise RuntimeError(f"{n} must have shape {(B, 1, H, W)}, got {tuple(x.shape)}")
        if x.dtype != obj.dtype:
            raise RuntimeError(f"expected scalar type {obj.dtype} for {n} but found {x.dtype}")
        if x.device != obj.device:
            raise RuntimeError(f"{n} is on {x.device}, obj on {obj.device}")
    if obj.dtype not in (_F32, _F64):
        raise RuntimeError(f"forward_warping supports float32/float64, got {obj.dtype}")
    f64 = obj.dtype == _F64
    dev = obj.device
    with torch.cuda.device(dev):  # fw_cuda.cpp:24 device guard
        stream = torch.cuda.current_stream(dev)
        output = torch.empty_like(obj)
        valid = torch.empty_like(depth)
        collision = torch.empty_like(depth)
        nbytes = _ws_bytes(B, H, W, f64)
        ws = workspace(dev, nbytes, stream) if nbytes else None
        fn = _native.lib().ofd_fw_forward_warping_f64 if f64 else _native.lib().ofd_fw_forward_warping_f32
        rc = fn(obj.data_ptr(), safe_y.data_ptr(), safe_x.data_ptr(), depth.data_ptr(),
                output.data_ptr(), valid.data_ptr(), collision.data_ptr(), B, C, H, W,
                ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                stream.cuda_stream)
        _native.check(rc, "forward_warping")
    return [output, valid, collision]


def forward_warp_flow(obj: torch.Tensor, flow: torch.Tensor, depth: torch.Tensor,
                      out: Tuple[torch.Tensor, torch.Tensor, torch.Tensor] = None
                      ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Batched FW.forward core (alt_cuda/fw.py:27-54) in one native call.

    obj [B,C,H,W] float32, flow [B,2,H,W] float32 or float64 (channel 0 = x /
    u, channel 1 = y / v), depth [B,1,H,W] float32, all contiguous on one
    device.  Target = trunc(clamp(p0 + flow)) with the add in the flow's dtype.
    ``out`` optionally supplies preallocated (output, valid, collision).

    A bfloat16 obj (with a float32 flow) selects the training-loop variant
    (no reference counterpart): output in bfloat16,
    valid / collision float32, the same winners as the float32 op, so the
    output equals the float32 op's on ``obj.float()`` rounded back to bf16.
    """
    for x, n in ((obj, "obj"), (flow, "flow"), (depth, "depth")):
        _check_input(x, n)
    if obj.dim() != 4:
        raise RuntimeError(f"obj must be 4-D [B,C,H,W], got {obj.dim()}-D")
    B, C, H, W = obj.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise RuntimeError(f"flow must have shape {(B, 2, H, W)}, got {tuple(flow.shape)}")
    if tuple(depth.shape) != (B, 1, H, W):
        raise RuntimeError(f"depth must have shape {(B, 1, H, W)}, got {tuple(depth.shape)}")
    if obj.dtype not in (_F32, _BF16) or depth.dtype != _F32:
        raise RuntimeError("forward_warp_flow expects a float32 or bfloat16 obj and a float32 depth")
    if flow.dtype not in (_F32, _F64):
        raise RuntimeError(f"flow must be float32 or float64, got {flow.dtype}")
    bf16 = obj.dtype == _BF16
    if bf16 and flow.dtype != _F32:
        raise RuntimeError("the bfloat16 warp takes a float32 flow")
    if flow.device != obj.device or depth.device != obj.device:
        raise RuntimeError("obj, flow and depth must be on one device")
    dev = obj.device
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        if out is None:
            output = torch.empty_like(obj)
            valid = torch.empty_like(depth)
            collision = torch.empty_like(depth)
        else:
            output, valid, collision = _check_out(out, ((B, C, H, W), (B, 1, H, W), (B, 1, H, W)),
                                                  (obj.dtype, _F32, _F32), dev)
        nbytes = _ws_bytes(B, H, W, False)
        ws = workspace(dev, nbytes, stream) if nbytes else None
        lib = _native.lib()
        fn = (lib.ofd_fw_forward_warp_flow_bf16 if bf16 else
              lib.ofd_fw_forward_warp_flow_f64flow if flow.dtype == _F64 else lib.ofd_fw_forward_warp_flow_f32)
        rc = fn(obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), output.data_ptr(), valid.data_ptr(),
                collision.data_ptr(), B, C, H, W,
                ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                stream.cuda_stream)
        _native.check(rc, "forward_warp_flow")
    return output, valid, collision


INPAINT_ORDERS = ("sequential", "layered")

# Hole-fill workspace budget per (device, stream) cache entry, in bytes
# (OFD_INPAINT_WS_GB, default 32 GiB: 3 x 64 headline images in one chunk; at most
# _WS_CACHE_MAX entries live).
_INPAINT_WS_BUDGET = int(float(os.environ.get("OFD_INPAINT_WS_GB", "32")) * (1 << 30))


def inpaint_chunk_images(ws_bytes_fn, H: int, W: int) -> int:
    """Images per hole-fill chunk under the workspace budget (at least one)."""
    one = int(ws_bytes_fn(1, H, W))
    two = int(ws_bytes_fn(2, H, W))
    per = max(two - one, 1)
    return max(1, (_INPAINT_WS_BUDGET - (one - per)) // per)


def default_inpaint_order() -> str:
    """The hole-fill order ops.inpaint uses when none is given: OFD_INPAINT_ORDER, else "sequential"."""
    o = os.environ.get("OFD_INPAINT_ORDER", "sequential")
    if o not in INPAINT_ORDERS:
        raise ValueError(f"OFD_INPAINT_ORDER must be one of {INPAINT_ORDERS}, got {o!r}")
    return o


def inpaint(img: torch.Tensor, valid: torch.Tensor, collision: torch.Tensor, radius: int = 3,
            order: str = None) -> torch.Tensor:
    """Drop-in for ``utils.inpaint(img, valid, collision)`` (utils.py:136-151), batched.

    img [C,H,W] with valid / collision [1,H,W] (the reference's call shape), or
    img [B,C,H,W] with [B,1,H,W] masks.  Pixels the keep mask of
    utils.py:137-142 drops are filled (Telea; see
    include/ofd_inpaint.h); every pixel of the result is float32 of the
    uint8 cast of utils.py:148, on img's device, like the reference's return.

    ``order="sequential"`` (the default, include/ofd_inpaint.h
    ofd_inpaint_telea_seq_f32) fills in cv2's exact order: heap pops by
    (distance, push order), each hole coloured from the pixels reached before
    it -- bit-exact against the CPU restatement of OpenCV's Telea
    (oracle/inpaint_oracle.c; OpenCV itself is absent from the build image).
    ``order="layered"`` (ofd_inpaint_telea_f32) is the faster re-specification:
    holes are finalised in layers of equal L1 distance, so its values are NOT
    cv2's -- the specified divergence (DESIGN.md section 5,
    tests/test_inpaint.py): on warped random-RGB images 85 % of hole values
    differ from the sequential order, mean 5.7 grey levels, p99 40; within 1-2
    levels on smooth images.  Both keep the reference's mask algebra, cast and
    kept pixels exactly.  The call never blocks the host.
    """
    order = default_inpaint_order() if order is None else order
    if order not in INPAINT_ORDERS:
        raise ValueError(f"order must be one of {INPAINT_ORDERS}, got {order!r}")
    seq = order == "sequential"
    for x, n in ((img, "img"), (valid, "valid"), (collision, "collision")):
        if not isinstance(x, torch.Tensor):
            raise TypeError(f"{n} must be a torch.Tensor")
        if not x.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")
    squeeze = img.dim() == 3
    if squeeze:
        img, valid, collision = img.unsqueeze(0), valid.unsqueeze(0), collision.unsqueeze(0)
    if img.dim() != 4:
        raise RuntimeError(f"img must be [C,H,W] or [B,C,H,W], got {img.dim()}-D")
    B, C, H, W = img.shape
    for x, n in ((valid, "valid"), (collision, "collision")):
        if tuple(x.shape) != (B, 1, H, W):
            raise RuntimeError(f"{n} must have shape {(B, 1, H, W)[1 if squeeze else 0:]}, "
                               f"got {tuple(x.shape)[1 if squeeze else 0:]}")
        if x.device != img.device:
            raise RuntimeError(f"{n} is on {x.device}, img on {img.device}")
    dev = img.device
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        img = img.to(_F32).contiguous()
        valid = valid.to(_F32).contiguous()
        collision = collision.to(_F32).contiguous()
        out = torch.empty_like(img)
        lib = _native.lib()
        wsb = lib.ofd_inpaint_seq_workspace_bytes if seq else lib.ofd_inpaint_workspace_bytes
        # the library fills the batch in chunks of as many images as the
        # workspace holds: cap it at a byte budget (~210 B per padded pixel for
        # the sequential fill, ~32 GB for 3 x 64 headline images otherwise)
        nbytes = int(wsb(min(B, inpaint_chunk_images(wsb, H, W)), H, W))
        ws = None
        if nbytes:
            key = (dev.index, stream.cuda_stream)
            with _ws_lock:
                ws = _ip_workspaces.get(key)
                if ws is None or ws.numel() < nbytes:
                    _ip_workspaces.pop(key, None)
                    ws = None
                    with torch.cuda.stream(stream):
                        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                _cache_put(_ip_workspaces, key, ws)
        fn = lib.ofd_inpaint_telea_seq_f32 if seq else lib.ofd_inpaint_telea_f32
        rc = fn(img.data_ptr(), valid.data_ptr(), collision.data_ptr(), out.data_ptr(),
                B, C, H, W, int(radius), ws.data_ptr() if ws is not None else None,
                ws.numel() if ws is not None else 0, stream.cuda_stream)
        _native.check(rc, "inpaint")
    return out[0] if squeeze else out


def inpaint_faults(reset: bool = True) -> int:
    """The hole-fill's invariant-violation bits since the last reset
    (include/ofd_inpaint.h ofd_inpaint_faults: 2 / 4 a march bound, 8 the
    layered tail's wait, 32 a wait of the levels-free colour pass).  Any set
    bit means some fill since the reset is incomplete.  Blocking: a
    device-to-host copy of the fault words, so callers check once per batch,
    not per fill."""
    rc = int(_native.lib().ofd_inpaint_faults(1 if reset else 0))
    if rc < 0:
        raise RuntimeError("ofd_inpaint_faults: HIP error reading the fault words")
    return rc


def warp_disparity(obj: torch.Tensor, depth: torch.Tensor, s: torch.Tensor,
                   out: Tuple[torch.Tensor, torch.Tensor, torch.Tensor] = None
                   ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """preprocess.py:356-359 fused (include/ofd_fw.h ofd_fw_warp_disparity_*):

        flow = Convert.disparity_to_flow(Convert.depth_to_disparity(depth), random_sign=False)
        FW(torch.cat((obj[:, :3], depth, flow * -1.0, obj[:, 3:]), 1), flow, depth)

    in one native call that never stores the flow or the concatenation.
    obj [B,Cobj,H,W] float32, depth [B,1,H,W] float32 or float64, s [B] (the
    per-image draw of preprocess.py:240).  Returns (output [B,Cobj+3,H,W],
    valid, collision), bit-identical to the unfused FW call.
    """
    for x, n in ((obj, "obj"), (depth, "depth")):
        _check_input(x, n)
    if obj.dim() != 4 or depth.dim() != 4:
        raise RuntimeError("warp_disparity expects obj [B,C,H,W] and depth [B,1,H,W]")
    B, Cobj, H, W = obj.shape
    if tuple(depth.shape) != (B, 1, H, W):
        raise RuntimeError(f"depth must have shape {(B, 1, H, W)}, got {tuple(depth.shape)}")
    if obj.dtype != _F32:
        raise RuntimeError("warp_disparity expects a float32 obj")
    if depth.dtype not in (_F32, _F64):
        raise RuntimeError(f"depth must be float32 or float64, got {depth.dtype}")
    dev = obj.device
    if depth.device != dev:
        raise RuntimeError("obj and depth must be on one device")
    s = torch.as_tensor(s, dtype=_F32).reshape(-1).to(dev).contiguous()
    if s.numel() != B:
        raise RuntimeError(f"s must hold one scale per image ({B}), got {s.numel()}")
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        if out is None:
            output = torch.empty(B, Cobj + 3, H, W, dtype=_F32, device=dev)
            valid = torch.empty(B, 1, H, W, dtype=_F32, device=dev)
            collision = torch.empty_like(valid)
        else:
            output, valid, collision = _check_out(out, ((B, Cobj + 3, H, W), (B, 1, H, W), (B, 1, H, W)),
                                                  (_F32, _F32, _F32), dev)
        nbytes = _ws_bytes(B, H, W, False)
        ws = workspace(dev, nbytes, stream) if nbytes else None
        lib = _native.lib()
        fn = lib.ofd_fw_warp_disparity_f64depth if depth.dtype == _F64 else lib.ofd_fw_warp_disparity_f32
        rc = fn(obj.data_ptr(), Cobj, depth.data_ptr(), s.data_ptr(), output.data_ptr(), valid.data_ptr(),
                collision.data_ptr(), B, H, W, ws.data_ptr() if ws is not None else None,
                ws.numel() if ws is not None else 0, stream.cuda_stream)
        _native.check(rc, "warp_disparity")
    return output, valid, collision


def _ego_camera(B, P, inv_K, dev):
    P = torch.as_tensor(P, dtype=_F32).to(dev).contiguous()
    if tuple(P.shape) != (B, 3, 4):
        raise RuntimeError(f"P must have shape {(B, 3, 4)}, got {tuple(P.shape)}")
    ik = torch.as_tensor(inv_K, dtype=_F32).cpu().contiguous()
    if tuple(ik.shape) != (3, 3):
        raise RuntimeError(f"inv_K must be [3,3] (inv_K[:3,:3]), got {tuple(ik.shape)}")
    return P, ik


def ego_flow(depth: torch.Tensor, P: torch.Tensor, inv_K: torch.Tensor) -> torch.Tensor:
    """Convert.depth_to_random_flow's flow (preprocess.py:265-298, geometry.py:17-67)
    for a batch: depth [B,1,H,W] float32 / float64, P [B,3,4] = (K @ T)[:, :3]
    (synth.projection), inv_K [3,3] -> flow [B,2,H,W] float32, equal to the
    reference's to float32 rounding (include/ofd_fw.h ofd_fw_ego_flow_*)."""
    _check_input(depth, "depth")
    if depth.dim() != 4 or depth.shape[1] != 1:
        raise RuntimeError(f"depth must be [B,1,H,W], got {tuple(depth.shape)}")
    if depth.dtype not in (_F32, _F64):
        raise RuntimeError(f"depth must be float32 or float64, got {depth.dtype}")
    B, _, H, W = depth.shape
    dev = depth.device
    P, ik = _ego_camera(B, P, inv_K, dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        flow = torch.empty(B, 2, H, W, dtype=_F32, device=dev)
        lib = _native.lib()
        fn = lib.ofd_fw_ego_flow_f64depth if depth.dtype == _F64 else lib.ofd_fw_ego_flow_f32
        rc = fn(depth.data_ptr(), P.data_ptr(), ik.data_ptr(), flow.data_ptr(), B, H, W, stream.cuda_stream)
        _native.check(rc, "ego_flow")
    return flow


def rotation_flow(params: torch.Tensor, h: int, w: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """SpecialFlow._rotate's (special_flow, back_special_flow) [B,2,h,w] float32
    (preprocess.py:31-41, :63-77) on ``device``, from params [B,10] float32:
    c0x, c0y, rotate and reverse_rotate row-major.  Bit-identical to the
    reference's matmul (include/ofd_fw.h ofd_fw_rotation_flow_f32)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("rotation_flow needs a HIP device")
    params = params.to(device=dev, dtype=_F32).contiguous()
    if params.dim() != 2 or params.shape[1] != 10:
        raise RuntimeError(f"params must be [B,10], got {tuple(params.shape)}")
    B = params.shape[0]
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        flow = torch.empty(B, 2, h, w, dtype=_F32, device=dev)
        back = torch.empty_like(flow)
        rc = _native.lib().ofd_fw_rotation_flow_f32(params.data_ptr(), flow.data_ptr(), back.data_ptr(), B, h, w,
                                                    stream.cuda_stream)
        _native.check(rc, "rotation_flow")
    return flow, back


def warp_ego(obj: torch.Tensor, depth: torch.Tensor, P: torch.Tensor, inv_K: torch.Tensor,
             out: Tuple[torch.Tensor, torch.Tensor, torch.Tensor] = None
             ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """preprocess.py:371-373 / :385-387 fused (include/ofd_fw.h ofd_fw_warp_ego_*):

        flow = ego_flow(depth, P, inv_K)
        FW(torch.cat((obj[:, :3], depth, flow * -1.0, obj[:, 3:]), 1), flow, depth)

    in one native call that never stores the flow or the concatenation;
    bit-identical to forward_warp_flow on ``ego_flow``'s plane.  obj
    [B,Cobj,H,W] float32, depth [B,1,H,W] float32 / float64.  Returns
    (output [B,Cobj+3,H,W], valid, collision)."""
    for x, n in ((obj, "obj"), (depth, "depth")):
        _check_input(x, n)
    if obj.dim() != 4 or depth.dim() != 4:
        raise RuntimeError("warp_ego expects obj [B,C,H,W] and depth [B,1,H,W]")
    B, Cobj, H, W = obj.shape
    if tuple(depth.shape) != (B, 1, H, W):
        raise RuntimeError(f"depth must have shape {(B, 1, H, W)}, got {tuple(depth.shape)}")
    if obj.dtype != _F32:
        raise RuntimeError("warp_ego expects a float32 obj")
    if depth.dtype not in (_F32, _F64):
        raise RuntimeError(f"depth must be float32 or float64, got {depth.dtype}")
    dev = obj.device
    if depth.device != dev:
        raise RuntimeError("obj and depth must be on one device")
    P, ik = _ego_camera(B, P, inv_K, dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        if out is None:
            output = torch.empty(B, Cobj + 3, H, W, dtype=_F32, device=dev)
            valid = torch.empty(B, 1, H, W, dtype=_F32, device=dev)
            collision = torch.empty_like(valid)
        else:
            output, valid, collision = _check_out(out, ((B, Cobj + 3, H, W), (B, 1, H, W), (B, 1, H, W)),
                                                  (_F32, _F32, _F32), dev)
        nbytes = _ws_bytes(B, H, W, False)
        ws = workspace(dev, nbytes, stream) if nbytes else None
        lib = _native.lib()
        fn = lib.ofd_fw_warp_ego_f64depth if depth.dtype == _F64 else lib.ofd_fw_warp_ego_f32
        rc = fn(obj.data_ptr(), Cobj, depth.data_ptr(), P.data_ptr(), ik.data_ptr(), output.data_ptr(),
                valid.data_ptr(), collision.data_ptr(), B, H, W, ws.data_ptr() if ws is not None else None,
                ws.numel() if ws is not None else 0, stream.cuda_stream)
        _native.check(rc, "warp_ego")
    return output, valid, collision


def warp_flow_cat(obj: torch.Tensor, flow: torch.Tensor, depth: torch.Tensor,
                  out: Tuple[torch.Tensor, torch.Tensor, torch.Tensor] = None
                  ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """FW(torch.cat((obj[:, :3], depth, flow * -1.0, obj[:, 3:]), 1), flow, depth)
    on a flow plane the caller holds, in one native call that never stores the
    concatenation (include/ofd_fw.h ofd_fw_warp_flow_cat): preprocess.py:371-373,
    :385-387 (ego-motion flows), :400-402, :414-417 (composed flows).
    obj [B,Cobj,H,W] float32, flow [B,2,H,W] float32 / float64, depth [B,1,H,W]
    float32 / float64.  Returns (output [B,Cobj+3,H,W], valid, collision),
    bit-identical to forward_warp_flow on the concatenation."""
    for x, n in ((obj, "obj"), (flow, "flow"), (depth, "depth")):
        _check_input(x, n)
    if obj.dim() != 4:
        raise RuntimeError("warp_flow_cat expects obj [B,C,H,W]")
    B, Cobj, H, W = obj.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise RuntimeError(f"flow must have shape {(B, 2, H, W)}, got {tuple(flow.shape)}")
    if tuple(depth.shape) != (B, 1, H, W):
        raise RuntimeError(f"depth must have shape {(B, 1, H, W)}, got {tuple(depth.shape)}")
    if obj.dtype != _F32:
        raise RuntimeError("warp_flow_cat expects a float32 obj")
    for x, n in ((flow, "flow"), (depth, "depth")):
        if x.dtype not in (_F32, _F64):
            raise RuntimeError(f"{n} must be float32 or float64, got {x.dtype}")
    dev = obj.device
    if flow.device != dev or depth.device != dev:
        raise RuntimeError("obj, flow and depth must be on one device")
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        if out is None:
            output = torch.empty(B, Cobj + 3, H, W, dtype=_F32, device=dev)
            valid = torch.empty(B, 1, H, W, dtype=_F32, device=dev)
            collision = torch.empty_like(valid)
        else:
            output, valid, collision = _check_out(out, ((B, Cobj + 3, H, W), (B, 1, H, W), (B, 1, H, W)),
                                                  (_F32, _F32, _F32), dev)
        nbytes = _ws_bytes(B, H, W, False)
        ws = workspace(dev, nbytes, stream) if nbytes else None
        rc = _native.lib().ofd_fw_warp_flow_cat(
            obj.data_ptr(), Cobj, flow.data_ptr(), int(flow.dtype == _F64), depth.data_ptr(),
            int(depth.dtype == _F64), output.data_ptr(), valid.data_ptr(), collision.data_ptr(), B, H, W,
            ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, stream.cuda_stream)
        _native.check(rc, "warp_flow_cat")
    return output, valid, collision
