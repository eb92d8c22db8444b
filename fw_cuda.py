"""Drop-in for the reference's top-level extension module ``fw_cuda``.

The reference builds ``fw_cuda`` with ``forward_warping(obj, safe_y, safe_x,
depth) -> [output, valid, collision]`` (alt_cuda/fw_cuda.cpp:28-30); code that
does ``import fw_cuda`` (alt_cuda/fw.py:7) gets the HIP implementation here.
"""
from opticalflowfromdepth_amd import _native
from opticalflowfromdepth_amd.ops import forward_warping

_native.lib()

__all__ = ["forward_warping"]
