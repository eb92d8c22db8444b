"""The reference ``utils`` functions on the warp path (utils.py:96-151), on device.

* ``inpaint``          -- utils.py:136-151, GPU hole-fill (ops.inpaint), batched
* ``normalize_depth``  -- utils.py:102-116 (per image of a batch)
* ``fix_warped_depth`` -- utils.py:123-126 (in place)
* ``get_random``       -- utils.py:96-100 (torch CPU RNG draws, same order)
* ``set_seed``         -- utils.py:178-188 (torch / numpy / random seeds)

File I/O (get_img / get_depth / get_disparity) and flow colouring are out of
scope.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from .ops import inpaint
from .synth import fix_warped_depth, get_random, normalize_depth

__all__ = ["inpaint", "normalize_depth", "fix_warped_depth", "get_random", "set_seed"]


def set_seed(seed: int = 42, loader=None) -> None:
    """utils.py:178-188: seed torch (CPU and every GPU, lazily), numpy and python,
    and a DataLoader sampler's generator when one is given."""
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)
    try:
        loader.sampler.generator.manual_seed(seed)
    except AttributeError:
        pass
