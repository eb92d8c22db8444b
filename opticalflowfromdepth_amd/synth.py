"""Synthetic workload generators for the forward-warp path (callers of FW).

Restates, in batched device-agnostic torch, the reference's flow synthesis
that feeds ``FW`` in preprocess.py's first stage:

* ``get_random``               -- utils.py:96-100 (torch CPU RNG draws)
* ``normalize_depth``          -- utils.py:102-116, per image
* ``fix_warped_depth``         -- utils.py:123-126
* ``camera_params``            -- the RNG draw order of preprocess.py's first stage
                                  for one image seed: Convert.depth_to_disparity's
                                  scale s (:240), then Plausible.random_motion's
                                  T1 (:277 -> :212-235, geometry.py:70-153)
* ``intrinsics``               -- Plausible.K (preprocess.py:194-209)
* ``disparity_flow``           -- Convert.depth_to_disparity + disparity_to_flow
                                  (preprocess.py:239-254, random_sign=False as :357)
* ``ego_motion_flow``          -- Convert.depth_to_random_flow (preprocess.py:265-298)
                                  with geometry.BackprojectDepth / Project3D
                                  (geometry.py:17-67), batched over images

The synthetic depth itself (``synthetic_depth``) has no reference counterpart:
the reference reads DIML / ReDWeb images from disk (dataloader.py:13-58),
which are not available offline.  It is a smooth field (sum of sinusoids) with
10 % multiplicative noise and 5 % holes (0 -> the normalize_depth sentinel).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch

# ------------------------------------------------------------------ RNG restatement
def get_random(random_range, random_begin, random_sign=True):
    """utils.py:96-100: sign in {-1,1} (randint) times rand()*range + begin."""
    sign = torch.randint(0, 2, (1,))[0] * 2 - 1 if random_sign else torch.tensor(1)
    value = torch.rand(1)[0] * random_range + torch.tensor(random_begin)
    return sign * value


def _rot_from_axisangle(vec: torch.Tensor) -> torch.Tensor:
    """geometry.py:108-153 (B x 1 x 3 axis-angle -> B x 4 x 4)."""
    angle = torch.norm(vec, 2, 2, True)
    axis = vec / (angle + 1e-7)
    ca, sa = torch.cos(angle), torch.sin(angle)
    C = 1 - ca
    x, y, z = axis[..., 0].unsqueeze(1), axis[..., 1].unsqueeze(1), axis[..., 2].unsqueeze(1)
    xs, ys, zs = x * sa, y * sa, z * sa
    xC, yC, zC = x * C, y * C, z * C
    xyC, yzC, zxC = x * yC, y * zC, z * xC
    rot = torch.zeros((vec.shape[0], 4, 4), dtype=torch.float32, device=vec.device)
    rot[:, 0, 0] = torch.squeeze(x * xC + ca)
    rot[:, 0, 1] = torch.squeeze(xyC - zs)
    rot[:, 0, 2] = torch.squeeze(zxC + ys)
    rot[:, 1, 0] = torch.squeeze(xyC + zs)
    rot[:, 1, 1] = torch.squeeze(y * yC + ca)
    rot[:, 1, 2] = torch.squeeze(yzC - xs)
    rot[:, 2, 0] = torch.squeeze(zxC - ys)
    rot[:, 2, 1] = torch.squeeze(yzC + xs)
    rot[:, 2, 2] = torch.squeeze(z * zC + ca)
    rot[:, 3, 3] = 1
    return rot


def _transformation_from_parameters(axisangle: torch.Tensor, translation: torch.Tensor) -> torch.Tensor:
    """geometry.py:70-88 with invert=False: M = T @ R."""
    R = _rot_from_axisangle(axisangle)
    t = translation.clone()
    T = torch.zeros(t.shape[0], 4, 4, dtype=torch.float32, device=t.device)  # geometry.py:91-105
    T[:, 0, 0] = 1
    T[:, 1, 1] = 1
    T[:, 2, 2] = 1
    T[:, 3, 3] = 1
    T[:, :3, 3, None] = t.contiguous().view(-1, 3, 1)
    return torch.matmul(T, R)


def random_motion(axisangle_range=1. / 36., axisangle_base=1. / 36.,
                  translation_range=0.1, translation_base=0.1) -> torch.Tensor:
    """Plausible.random_motion (preprocess.py:212-235): [1,4,4] float32."""
    ang = [get_random(math.pi * axisangle_range, math.pi * axisangle_base) for _ in range(3)]
    mot = [get_random(translation_range, translation_base) for _ in range(3)]
    axisangle = torch.tensor([[ang]], dtype=torch.float32)
    translation = torch.tensor([[mot]], dtype=torch.float32)
    return _transformation_from_parameters(axisangle, translation)


def camera_params(seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(s, T1) drawn exactly as preprocess.py's first stage draws them after
    ``utils.set_seed(seed)`` (preprocess.py:555): s from depth_to_disparity
    (:356 -> :240), then T1 from depth_to_random_flow (:372 -> :277)."""
    torch.manual_seed(seed)  # utils.set_seed (utils.py:178-188), torch CPU RNG part
    s = get_random(0.3, 0.8, random_sign=False)
    T = random_motion()
    return s.to(torch.float32), T[0]


def batch_camera_params(seeds: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stacked (s [B], T [B,4,4]) for a list of image seeds.  Restores the
    caller's global torch RNG state afterwards."""
    state = torch.random.get_rng_state()
    try:
        ss, Ts = zip(*(camera_params(int(s)) for s in seeds))
    finally:
        torch.random.set_rng_state(state)
    return torch.stack(ss), torch.stack(Ts)


def intrinsics(h: int, w: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Plausible.K (preprocess.py:194-209): K, inv(K) as [4,4] float32 (CPU)."""
    K = torch.tensor([[0.58, 0, 0.5, 0],
                      [0, 0.58, 0.5, 0],
                      [0, 0, 1, 0],
                      [0, 0, 0, 1]], dtype=torch.float32)
    K[0, :] *= w
    K[1, :] *= h
    return K, torch.linalg.inv(K.unsqueeze(0))[0]


# ------------------------------------------------------------------ depth
def synthetic_depth_np(h: int, w: int, seed: int) -> np.ndarray:
    """Smooth synthetic raw depth [h,w] float64 in (0, ~95], 5 % zero holes."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    d = np.zeros((h, w))
    for _ in range(4):
        fx, fy = rng.uniform(0.5, 3.0, 2)
        ph = rng.uniform(0, 2 * np.pi, 2)
        d += np.sin(2 * np.pi * fx * xx / w + ph[0]) * np.cos(2 * np.pi * fy * yy / h + ph[1])
    d = (d - d.min()) / (d.max() - d.min() + 1e-12)
    d = 2 + 85 * d
    d *= 1 + 0.1 * rng.uniform(-1, 1, (h, w))
    d[rng.random((h, w)) < 0.05] = 0
    return d


def synthetic_depth(seeds: Sequence[int], h: int, w: int, device, dtype=torch.float32) -> torch.Tensor:
    """Batched device version of the same field family: [B,1,h,w].

    Wave parameters come from numpy with the image seed (as synthetic_depth_np);
    the noise and holes come from a device generator seeded with the image
    seed, so the values are NOT bit-identical to synthetic_depth_np (tests that
    need identity use the numpy version)."""
    out = torch.empty(len(seeds), 1, h, w, device=device, dtype=dtype)
    yy = torch.arange(h, device=device, dtype=torch.float32).view(h, 1)
    xx = torch.arange(w, device=device, dtype=torch.float32).view(1, w)
    g = torch.Generator(device=device)
    for n, seed in enumerate(seeds):
        rng = np.random.default_rng(int(seed))
        d = torch.zeros(h, w, device=device, dtype=torch.float32)
        for _ in range(4):
            fx, fy = rng.uniform(0.5, 3.0, 2)
            ph = rng.uniform(0, 2 * np.pi, 2)
            d += torch.sin(2 * math.pi * float(fx) * xx / w + float(ph[0])) * \
                torch.cos(2 * math.pi * float(fy) * yy / h + float(ph[1]))
        d = (d - d.min()) / (d.max() - d.min() + 1e-12)
        d = 2 + 85 * d
        g.manual_seed(int(seed))
        d = d * (1 + 0.1 * (torch.rand(h, w, device=device, generator=g) * 2 - 1))
        d[torch.rand(h, w, device=device, generator=g) < 0.05] = 0
        out[n, 0] = d.to(dtype)
    return out


def synthetic_rgb(seeds: Sequence[int], h: int, w: int, device) -> torch.Tensor:
    """Integer-valued float32 RGB in [0,255], [B,3,h,w] (cv2.imread-like values)."""
    g = torch.Generator(device=device)
    out = torch.empty(len(seeds), 3, h, w, device=device, dtype=torch.float32)
    for n, seed in enumerate(seeds):
        g.manual_seed(int(seed) + 1000)
        out[n] = torch.floor(torch.rand(3, h, w, device=device, generator=g) * 256)
    return out


def normalize_depth(depth: torch.Tensor) -> torch.Tensor:
    """utils.py:102-116 applied per image of a [B,1,H,W] batch (returns a new tensor)."""
    d = depth.clone()
    d[d == 0] = 100
    d[d > 100] = 100
    flat = d.flatten(1)
    dmin = flat.amin(dim=1).view(-1, 1, 1, 1)
    d[d == 100] = 0
    dmax = d.flatten(1).amax(dim=1).view(-1, 1, 1, 1)
    d = (d - dmin) * 98 / (dmax - dmin) + 1
    sentinel = (0 - dmin) * 98 / (dmax - dmin) + 1
    d = torch.where(d == sentinel, torch.full_like(d, 100), d)
    return d


def fix_warped_depth(depth: torch.Tensor) -> torch.Tensor:
    """utils.py:123-126 (in place, returns its argument)."""
    depth[depth == 0] = 100
    depth[depth > 99.5] = 100
    return depth


# ------------------------------------------------------------------ flows
def disparity_flow(depth: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """Convert.depth_to_disparity + disparity_to_flow (preprocess.py:239-254).

    depth [B,1,H,W], s [B] -> flow [B,2,H,W] = cat(s*50*1/depth, 0) * -1,
    in depth's dtype (float64 depth gives a float64 flow, as in the reference)."""
    sB = s.to(depth.device).view(-1, 1, 1, 1)
    disparity = sB * 50 * 1 / depth
    return torch.cat((disparity, torch.zeros_like(disparity)), dim=1) * -1.0


def projection(h: int, w: int, T: torch.Tensor, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Project3D's P = (K @ T)[:, :3] (geometry.py:57) on ``device`` [B,3,4], and
    inv_K[:3,:3] (geometry.py:38) as a CPU [3,3] float32 tensor -- the camera
    inputs of ops.ego_flow / ops.warp_ego.

    P is multiplied on the host, one image at a time in the reference's own
    shapes ([1,4,4] @ [1,4,4]), and then copied to ``device``: with that P the
    device flow is bit for bit the reference's CPU run (the 4x4 product on
    the GPU rounds some entries differently, which moved the flow by up to
    8 ulp; tests/test_ego.py, tests/golden/ppa_fill_large.npz)."""
    K, inv_K = intrinsics(h, w)
    Tc = T.detach().to(device="cpu", dtype=torch.float32)
    Kc = K.to("cpu").unsqueeze(0)
    P = torch.cat([torch.matmul(Kc, Tc[b:b + 1]) for b in range(Tc.shape[0])])[:, :3, :]
    return P.contiguous().to(device), inv_K[:3, :3].contiguous()


def ego_motion_flow(depth: torch.Tensor, T: torch.Tensor) -> torch.Tensor:
    """Convert.depth_to_random_flow (preprocess.py:265-298), batched.

    depth [B,1,H,W] (float32, or float64 as the first stage passes it: the
    product with the camera rays is taken in float64 and then rounded, as
    geometry.py:39-40 does), T [B,4,4] -> flow [B,2,H,W] float32."""
    B, _, h, w = depth.shape
    dev = depth.device
    K, inv_K = intrinsics(h, w)
    K, inv_K = K.to(dev), inv_K.to(dev)
    ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
    pix = torch.stack([xs.reshape(-1).float(), ys.reshape(-1).float(),
                       torch.ones(h * w, device=dev)], 0)                       # geometry.py:27-35
    # the reference's shapes exactly ([1,3,3] @ [1,3,HW]): a 2-D matmul takes
    # another BLAS path on some hosts and rounds differently
    cam = torch.matmul(inv_K[None, :3, :3], pix.unsqueeze(0))                    # :38
    cam = depth.reshape(B, 1, -1) * cam                                          # :39 (depth's dtype)
    cam = torch.cat([cam, torch.ones(B, 1, h * w, device=dev, dtype=cam.dtype)], 1).to(torch.float32)  # :40
    P = torch.matmul(K.unsqueeze(0), T.to(dev))[:, :3, :]                        # :57
    cp = torch.matmul(P, cam)                                                    # :59
    pc = cp[:, :2, :] / (cp[:, 2, :].unsqueeze(1) + 1e-7)                        # :61
    pc = pc.view(B, 2, h, w)
    px = pc[:, 0] / (w - 1)                                                      # :64
    py = pc[:, 1] / (h - 1)                                                      # :65
    px = (px - 0.5) * 2                                                          # :66
    py = (py - 0.5) * 2
    px = (px + 1) / 2 * (w - 1)                                                  # preprocess.py:284-286
    py = (py + 1) / 2 * (h - 1)
    flow = torch.stack([px - xs.float(), py - ys.float()], 1)                    # :288-291
    return flow


def stage_one_batch(seeds: Sequence[int], h: int, w: int, device, ego_fraction: float = 0.5,
                    camera: Tuple[torch.Tensor, torch.Tensor] = None):
    """The headline FW workload (preprocess.py:358/387 calls), batched.

    For each image seed: synthetic depth -> normalize_depth -> a flow (the
    first ``(1-ego_fraction)*B`` images a disparity flow, the rest an
    ego-motion flow, both from the image's seed) -> obj C=6 =
    [RGB, depth, -flow] (preprocess.py:358 / :386).
    ``camera`` optionally supplies (s [B], T [B,4,4]) already drawn for these
    seeds (e.g. received by broadcast); otherwise they are drawn here.
    Returns (obj [B,6,h,w], flow [B,2,h,w], depth [B,1,h,w]) float32 on device.
    """
    B = len(seeds)
    s, T = camera if camera is not None else batch_camera_params(seeds)
    depth = normalize_depth(synthetic_depth(seeds, h, w, device))
    rgb = synthetic_rgb(seeds, h, w, device)
    n_disp = B - int(round(B * ego_fraction))
    flow = torch.empty(B, 2, h, w, device=device, dtype=torch.float32)
    if n_disp > 0:
        flow[:n_disp] = disparity_flow(depth[:n_disp], s[:n_disp]).to(torch.float32)
    if n_disp < B:
        flow[n_disp:] = ego_motion_flow(depth[n_disp:], T[n_disp:])
    obj = torch.cat((rgb, depth, flow * -1.0), dim=1).contiguous()
    return obj, flow.contiguous(), depth.contiguous()
