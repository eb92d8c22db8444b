"""Loader for the native library (libofd_fw.so; C ABI in include/ofd_fw.h, ofd_inpaint.h, ofd_deflate.h).

The library is built in-tree by :func:`opticalflowfromdepth_amd.build.build_native`
(hipcc --offload-arch=gfx950).  There is deliberately NO fallback: if the
library is missing or does not load, every op raises -- a silent CPU or eager
torch path would hide that the HIP kernels are not the thing running.

torch is imported first so that its HIP runtime (libamdhip64.so.7, shipped in
torch/lib) is the one the library binds to: stream handles from
``torch.cuda.current_stream()`` are then valid inside the library.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must precede the CDLL load (shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OFD_FW_LIB") or os.path.join(_HERE, "_build", "libofd_fw.so")  # override: probe builds only
ABI_VERSION = 1

_lock = threading.Lock()
_lib = None

# (name, argtypes, restype) for every symbol declared in include/*.h
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t
SIGNATURES = {
    "ofd_fw_abi_version": ([], ctypes.c_int),
    "ofd_fw_build_id": ([], ctypes.c_char_p),
    "ofd_fw_strerror": ([ctypes.c_int], ctypes.c_char_p),
    "ofd_fw_set_engine": ([ctypes.c_int], ctypes.c_int),
    "ofd_fw_set_disparity_rows": ([ctypes.c_int], ctypes.c_int),
    "ofd_fw_set_persist_min": ([ctypes.c_int], ctypes.c_int),
    "ofd_fw_set_pack": ([ctypes.c_int], ctypes.c_int),
    "ofd_fw_set_profile_events": ([_P, _P], ctypes.c_int),
    "ofd_fw_set_profile_bin_event": ([_P], ctypes.c_int),
    "ofd_fw_set_short_tiles": ([ctypes.c_int], ctypes.c_int),
    "ofd_fw_workspace_bytes": ([_I64, _I64, _I64, ctypes.c_int], _SZ),
    "ofd_fw_workspace_init": ([_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_forward_warping_f32": ([_P] * 7 + [_I64] * 4 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_forward_warping_f64": ([_P] * 7 + [_I64] * 4 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_forward_warp_flow_f32": ([_P] * 6 + [_I64] * 4 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_forward_warp_flow_f64flow": ([_P] * 6 + [_I64] * 4 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_forward_warp_flow_bf16": ([_P] * 6 + [_I64] * 4 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_warp_disparity_f32": ([_P, _I64, _P, _P, _P, _P, _P] + [_I64] * 3 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_warp_disparity_f64depth": ([_P, _I64, _P, _P, _P, _P, _P] + [_I64] * 3 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_ego_flow_f32": ([_P] * 4 + [_I64] * 3 + [_P], ctypes.c_int),
    "ofd_fw_ego_flow_f64depth": ([_P] * 4 + [_I64] * 3 + [_P], ctypes.c_int),
    "ofd_fw_rotation_flow_f32": ([_P] * 3 + [_I64] * 3 + [_P], ctypes.c_int),
    "ofd_fw_warp_ego_f32": ([_P, _I64] + [_P] * 6 + [_I64] * 3 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_warp_ego_f64depth": ([_P, _I64] + [_P] * 6 + [_I64] * 3 + [_P, _SZ, _P], ctypes.c_int),
    "ofd_fw_warp_flow_cat": ([_P, _I64, _P, ctypes.c_int, _P, ctypes.c_int] + [_P] * 3 + [_I64] * 3 + [_P, _SZ, _P],
                             ctypes.c_int),
    "ofd_inpaint_workspace_bytes": ([_I64, _I64, _I64], _SZ),
    "ofd_inpaint_telea_f32": ([_P] * 4 + [_I64] * 4 + [ctypes.c_int, _P, _SZ, _P], ctypes.c_int),
    "ofd_inpaint_seq_workspace_bytes": ([_I64, _I64, _I64], _SZ),
    "ofd_inpaint_telea_seq_f32": ([_P] * 4 + [_I64] * 4 + [ctypes.c_int, _P, _SZ, _P], ctypes.c_int),
    "ofd_inpaint_set_schedule": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "ofd_inpaint_faults": ([ctypes.c_int], ctypes.c_int),
    "ofd_inpaint_tail_layers": ([ctypes.c_int], ctypes.c_int),
    "ofd_inpaint_seq_helper_device": ([ctypes.c_void_p], ctypes.c_int),
    "ofd_inpaint_seq_set_pipeline": ([ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "ofd_inpaint_seq_set_colour": ([ctypes.c_int], ctypes.c_int),
    "ofd_inpaint_seq_set_multi": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "ofd_deflate_bound": ([_I64], _SZ),
    "ofd_deflate_workspace_bytes": ([_I64, _I64], _SZ),
    "ofd_deflate_batch": ([_P, _I64, _I64, _P, _P, _P, _P, _SZ, _P], ctypes.c_int),
}


class NativeLibraryError(RuntimeError):
    """The HIP forward-warp library is missing or unusable."""


def _try_build():
    # Build in place when the source tree is present and hipcc is available
    # (e.g. a fresh checkout); otherwise report what is missing.
    from . import build as _build
    _build.build_native()


def lib():
    """Return the loaded ctypes library.  The in-tree library is (re)built
    first unless it was built from the current sources (build.needs_build: a
    content hash, recorded beside the .so), and after loading, the id the
    binary itself carries (ofd_fw_build_id) must equal that hash -- a stale
    .so that travelled with a tree can never stand in for the sources under
    test.  OFD_FW_LIB (probe builds) skips both checks."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        override = bool(os.environ.get("OFD_FW_LIB"))
        from . import build as _build
        if not override and (not os.path.exists(LIB_PATH) or _build.needs_build()):
            try:
                _try_build()
            except Exception as e:  # pragma: no cover - depends on toolchain
                raise NativeLibraryError(
                    f"libofd_fw.so at {LIB_PATH} is missing or stale and building it failed: {e}") from e
        try:
            l = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (argt, rest) in SIGNATURES.items():
            if override and not hasattr(l, name):
                continue  # a probe build from older sources may lack newer entry points
            fn = getattr(l, name)
            fn.argtypes = argt
            fn.restype = rest
        v = l.ofd_fw_abi_version()
        if v != ABI_VERSION:
            raise NativeLibraryError(f"libofd_fw ABI {v}, python expects {ABI_VERSION}; rebuild")
        if not override:
            got, want = l.ofd_fw_build_id().decode(), _build.source_hash()
            if got != want:
                raise NativeLibraryError(f"{LIB_PATH} carries build id {got}, the sources hash to {want}; "
                                         "rebuild (python -m opticalflowfromdepth_amd.build)")
        _lib = l
        return _lib


def build_id() -> str:
    """The loaded library's build id (include/ofd_fw.h: ofd_fw_build_id)."""
    return lib().ofd_fw_build_id().decode()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ofd_fw_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: {msg} (code {rc})")
