"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

Python face of the CPU restatement of the reference forward-warp.  Only tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this
module, and only as the checker / CPU baseline.  The product package
``opticalflowfromdepth_amd`` never imports it (a test asserts that).

Two independent restatements live here so that each pins the other:

* ``forward_warping`` / ``fw_flow`` call ``fw_oracle.c`` -- the literal serial
  raster loop of ``alt_cuda/fw_cuda_kernel.cu:28-47`` (+ host ``:52-83``) and
  the wrapper arithmetic of ``alt_cuda/fw.py:27-43``.
* ``forward_warping_lexmin`` is the set formulation: per target pixel, the
  winner is the lexicographic minimum of (depth, raster index) over landing
  sources with depth < 1000.  Pure numpy.

Parity status: the wrapper arithmetic is pinned by running the reference's own
``alt_cuda/fw.py`` (imported from /root/reference in the build container, with
this oracle injected as ``fw_cuda``) -- see tests/golden/make_golden.py.  The
kernel loop itself cannot be run from the reference (CUDA-only, sm_86,
CPython 3.9 / torch 1.12 binary), so it is pinned by the literal restatement
cross-checked against the independent lexmin formulation.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libfw_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile fw_oracle.c with gcc (oracle/Makefile)."""
    srcs = [os.path.join(_HERE, f) for f in ("fw_oracle.c", "inpaint_oracle.c", "Makefile")]
    if force or not os.path.exists(_LIB_PATH) or any(
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(f) for f in srcs
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.c_void_p
        L = ctypes.c_long
        for name, nptr in (("oracle_forward_warping_f32", 7), ("oracle_forward_warping_f64", 7),
                           ("oracle_fw_flow_f32", 6), ("oracle_fw_flow_f64flow", 6)):
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [fp] * nptr + [L, L, L, L, ctypes.c_int]
        lib.oracle_inpaint_f32.restype = ctypes.c_int
        lib.oracle_inpaint_f32.argtypes = [fp] * 4 + [L] * 4 + [ctypes.c_int] * 3
        lib.oracle_inpaint_mask.restype = ctypes.c_int
        lib.oracle_inpaint_mask.argtypes = [fp] * 3 + [L] * 3
        _lib = lib
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def forward_warping(obj, safe_y, safe_x, depth, nthreads: int = 0):
    """Restates ``fw_cuda.forward_warping`` (alt_cuda/fw_cuda.cpp:15-26).

    obj [B,C,H,W]; safe_y, safe_x, depth [B,1,H,W]; all float32 or all float64.
    Returns (output, valid, collision) numpy arrays of the same dtype.
    """
    obj = np.ascontiguousarray(obj)
    dt = obj.dtype
    if dt not in (np.float32, np.float64):
        raise TypeError("oracle: float32/float64 only")
    safe_y = np.ascontiguousarray(safe_y, dtype=dt)
    safe_x = np.ascontiguousarray(safe_x, dtype=dt)
    depth = np.ascontiguousarray(depth, dtype=dt)
    B, C, H, W = obj.shape
    for a in (safe_y, safe_x, depth):
        if a.shape != (B, 1, H, W):
            raise ValueError(f"oracle: expected [B,1,H,W] = {(B, 1, H, W)}, got {a.shape}")
    out = np.empty_like(obj)
    valid = np.empty((B, 1, H, W), dt)
    coll = np.empty((B, 1, H, W), dt)
    fn = _load().oracle_forward_warping_f32 if dt == np.float32 else _load().oracle_forward_warping_f64
    rc = fn(_p(obj), _p(safe_y), _p(safe_x), _p(depth), _p(out), _p(valid), _p(coll), B, C, H, W, nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return out, valid, coll


def fw_flow(obj, flow, depth, nthreads: int = 0):
    """Restates a batched ``FW.forward`` (alt_cuda/fw.py:19-59).

    obj [B,C,H,W] (cast to float32, fw.py:40), flow [B,2,H,W] float32 or float64
    (other float dtypes promote to float32 as torch would, fw.py:31), depth
    [B,1,H,W] (cast to float32, fw.py:43).  Returns float32 arrays.
    """
    obj = np.ascontiguousarray(obj, dtype=np.float32)
    depth = np.ascontiguousarray(depth, dtype=np.float32)
    flow = np.asarray(flow)
    if flow.dtype != np.float64:
        flow = flow.astype(np.float32)
    flow = np.ascontiguousarray(flow)
    B, C, H, W = obj.shape
    if flow.shape != (B, 2, H, W) or depth.shape != (B, 1, H, W):
        raise ValueError("oracle.fw_flow: shape mismatch")
    out = np.empty_like(obj)
    valid = np.empty((B, 1, H, W), np.float32)
    coll = np.empty((B, 1, H, W), np.float32)
    lib = _load()
    fn = lib.oracle_fw_flow_f64flow if flow.dtype == np.float64 else lib.oracle_fw_flow_f32
    rc = fn(_p(obj), _p(flow), _p(depth), _p(out), _p(valid), _p(coll), B, C, H, W, nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return out, valid, coll


def safe_coords(flow):
    """fw.py:27-42 in numpy: (safe_y, safe_x) [B,1,H,W] float32 from flow [B,2,H,W].

    NaN coordinates stay NaN (torch.clamp propagates NaN); the loop drops them.
    """
    flow = np.asarray(flow)
    B, _, H, W = flow.shape
    ct = np.float64 if flow.dtype == np.float64 else np.float32
    flow = flow.astype(ct, copy=False)
    xs = np.arange(W, dtype=np.float32).astype(ct)[None, None, None, :]
    ys = np.arange(H, dtype=np.float32).astype(ct)[None, None, :, None]
    with np.errstate(invalid="ignore"):
        px = xs + flow[:, 0:1]
        py = ys + flow[:, 1:2]
        px = np.where(np.isnan(px), px, np.clip(px, 0, W - 1))
        py = np.where(np.isnan(py), py, np.clip(py, 0, H - 1))
        sx = np.where(np.isnan(px), np.nan, np.trunc(px)).astype(np.float32)
        sy = np.where(np.isnan(py), np.nan, np.trunc(py)).astype(np.float32)
    return sy, sx


def _orderable32(d: np.ndarray) -> np.ndarray:
    d = np.where(d == 0, np.float32(0), d).astype(np.float32)  # -0 -> +0
    u = d.view(np.uint32).astype(np.uint64)
    neg = (u & 0x80000000) != 0
    return np.where(neg, (~u) & 0xFFFFFFFF, u | 0x80000000)


def forward_warping_lexmin(obj, safe_y, safe_x, depth):
    """Independent set formulation of the same op (float32 only).

    winner(t) = argmin over sources s landing on t with depth[s] < 1000 of the
    key (orderable(depth[s]) << 32 | s); valid(t) = any source landed;
    collision(t) = valid and no winner.  Sources with NaN / out-of-range
    coordinates are dropped (same defined behaviour as fw_oracle.c).
    """
    obj = np.asarray(obj, np.float32)
    B, C, H, W = obj.shape
    HW = H * W
    out = np.zeros_like(obj)
    valid = np.zeros((B, 1, H, W), np.float32)
    coll = np.zeros((B, 1, H, W), np.float32)
    src = np.arange(HW, dtype=np.uint64)
    for b in range(B):
        sx = np.asarray(safe_x[b, 0], np.float64).reshape(-1)
        sy = np.asarray(safe_y[b, 0], np.float64).reshape(-1)
        d = np.asarray(depth[b, 0], np.float32).reshape(-1)
        with np.errstate(invalid="ignore"):
            ok = (sx > -1) & (sx < W) & (sy > -1) & (sy < H)
        x = np.where(ok, np.trunc(np.where(ok, sx, 0)), 0).astype(np.int64)
        y = np.where(ok, np.trunc(np.where(ok, sy, 0)), 0).astype(np.int64)
        t = (y * W + x)[ok]
        v = np.zeros(HW, bool)
        v[t] = True
        with np.errstate(invalid="ignore"):
            part = ok & (d < np.float32(1000))
        tp = (y * W + x)[part]
        keys = (_orderable32(d[part]) << np.uint64(32)) | src[part]
        best = np.full(HW, np.iinfo(np.uint64).max, np.uint64)
        np.minimum.at(best, tp, keys)
        has = best != np.iinfo(np.uint64).max
        win = (best[has] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        ob = obj[b].reshape(C, HW)
        o = np.zeros((C, HW), np.float32)
        o[:, has] = ob[:, win]
        out[b] = o.reshape(C, H, W)
        valid[b, 0] = v.reshape(H, W)
        coll[b, 0] = (v & ~has).reshape(H, W)
    return out, valid, coll


def inpaint(img, valid, collision, radius: int = 3, layered: bool = False, nthreads: int = 0):
    """Restates a batched ``utils.inpaint`` (utils.py:136-151).

    img [B,C,H,W], valid / collision [B,1,H,W] (cast to float32).  layered =
    False: the sequential restatement of cv2.inpaint(..., INPAINT_TELEA)
    (parity unpinned: OpenCV is absent); True: the layered Telea the GPU runs.
    Returns float32 [B,C,H,W] holding uint8 values.
    """
    img = np.ascontiguousarray(img, dtype=np.float32)
    valid = np.ascontiguousarray(valid, dtype=np.float32)
    collision = np.ascontiguousarray(collision, dtype=np.float32)
    B, C, H, W = img.shape
    if valid.shape != (B, 1, H, W) or collision.shape != (B, 1, H, W):
        raise ValueError("oracle.inpaint: shape mismatch")
    out = np.empty_like(img)
    rc = _load().oracle_inpaint_f32(_p(img), _p(valid), _p(collision), _p(out), B, C, H, W,
                                    int(radius), int(bool(layered)), nthreads)
    if rc != 0:
        raise ValueError(f"oracle.inpaint rc={rc} (images must be at least 2x2)")
    return out


def inpaint_mask(valid, collision):
    """utils.py:137-142: uint8 [B,H,W], 1 where cv2.inpaint fills."""
    valid = np.ascontiguousarray(valid, dtype=np.float32)
    collision = np.ascontiguousarray(collision, dtype=np.float32)
    B, _, H, W = valid.shape
    hole = np.empty((B, H, W), np.uint8)
    rc = _load().oracle_inpaint_mask(_p(valid), _p(collision), _p(hole), B, H, W)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return hole
