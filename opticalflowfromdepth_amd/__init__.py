"""opticalflowfromdepth_amd -- MI355X-native forward-warp (z-buffered splat) engine.

The hot path of AegeanKI/OpticalFlowFromDepth (alt_cuda/fw_cuda_kernel.cu,
alt_cuda/fw_cuda.cpp, alt_cuda/fw.py) rebuilt as hand-written HIP kernels for
gfx950 behind a C ABI (include/ofd_fw.h), with the reference's Python surface:

* ``FW``               -- drop-in for ``alt_cuda.fw.FW``
* ``forward_warping``  -- drop-in for the extension op ``fw_cuda.forward_warping``
* ``forward_warp_flow``-- batched FW core (flow -> splat in one native call)
* ``warp_disparity``   -- preprocess.py:356-359 fused (depth -> disparity -> flow -> splat)
* ``warp_ego``         -- preprocess.py:371-373 / :385-387 fused (depth -> ego-motion flow -> splat)
* ``ego_flow``         -- the ego-motion flow plane (preprocess.py:265-298) in one kernel
* ``warp_flow_cat``    -- FW(cat(img, depth, flow * -1.0, ...), flow, depth) on a held flow plane,
                          the concatenation never stored (preprocess.py:371-417)
* ``inpaint``          -- batched GPU hole-fill replacing ``utils.inpaint``
"""
from .fw import FW
from .ops import ego_flow, forward_warp_flow, forward_warping, inpaint, warp_disparity, warp_ego, warp_flow_cat

__all__ = ["FW", "forward_warping", "forward_warp_flow", "warp_disparity", "warp_ego", "ego_flow", "warp_flow_cat", "inpaint"]
__version__ = "0.1.0"
