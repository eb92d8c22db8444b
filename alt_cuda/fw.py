"""Drop-in for the reference module ``alt_cuda/fw.py``: ``from alt_cuda.fw import FW``.

The reference imports the CUDA extension ``fw_cuda`` at module load
(fw.py:7); this module loads the HIP library the same way, eagerly, so a
missing native build fails at import exactly like the reference would.
"""
from opticalflowfromdepth_amd import _native
from opticalflowfromdepth_amd.fw import FW, ForwardWarp, forward_warp

_native.lib()

__all__ = ["FW", "ForwardWarp", "forward_warp"]
