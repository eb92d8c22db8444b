"""The reference's preprocess.py around the warp, on device and batched.

Every FW call and every hole-fill here goes through the HIP engine
(``FW`` -> csrc/ofd_fw.hip, ``utils.inpaint`` -> csrc/ofd_inpaint.hip); the
flow algebra around them is torch on the same device.  Names, argument
meaning and the torch CPU RNG draw order follow the reference, so a caller
switching imports gets the same random parameters for the same seeds:

* ``Plausible``, ``Convert``          -- preprocess.py:184-298
* ``ConcatFlow``, ``BackFlow``         -- preprocess.py:301-326
* ``SpecialFlow``, ``augment_flow``    -- preprocess.py:24-182
* ``PreprocessPlusAugment``            -- preprocess.py:329-506 (per image, writes
  the same npz files), plus ``PreprocessPlusAugment.run_batch``: B images at a
  time, every FW / inpaint call batched over the images, the per-image random
  parameters replayed from each image's seed (``draw_image_params``).
* ``save_group`` / ``save_augment``    -- the npz layout of preprocess.py:437-476.

Behaviour the reference leaves broken is defined here:
the stereo branch uses the module's device (the reference reads an undefined
global ``device``, preprocess.py:353), and the augmented-pair save closes the
parenthesis that preprocess.py:463 leaves open.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import synth
from .fw import FW
from .npz_gpu import atomic_path, zip_complete
from .ops import ego_flow, inpaint, rotation_flow, warp_disparity, warp_flow_cat
from .synth import fix_warped_depth, get_random, normalize_depth

AUGMENT_SCHEDULE = (0, 5, 6, 7, 1, 5, 6, 7, 2, 5, 6, 7)  # preprocess.py:454
N_GROUPS = 5  # preprocess.py:427-432
_GRAY = ((0.2989, 0.2989, 0.2989), (0.5870, 0.5870, 0.5870), (0.1140, 0.1140, 0.1140))  # :152-154


# ---------------------------------------------------------------- Plausible / Convert
class Plausible:
    """preprocess.py:184-235."""

    @staticmethod
    def f():
        return 1

    @staticmethod
    def B():
        return 50

    @staticmethod
    def K(size, another=False):
        h, w = size
        K = torch.tensor([[[0.58, 0, 0.5, 0], [0, 0.58, 0.5, 0], [0, 0, 1, 0], [0, 0, 0, 1]]], dtype=torch.float32)
        if another:
            K[:, :2, :2] *= 2
        K[:, 0, :] *= w
        K[:, 1, :] *= h
        return K, torch.linalg.inv(K)

    @staticmethod
    def random_motion(axisangle_range, axisangle_base, translation_range, translation_base,
                      another_axisangle=None, another_translation=None):
        ang = [get_random(math.pi * axisangle_range, math.pi * axisangle_base) for _ in range(3)]
        mot = [get_random(translation_range, translation_base) for _ in range(3)]
        axisangle = torch.tensor([[ang]], dtype=torch.float32)
        translation = torch.tensor([[mot]], dtype=torch.float32)
        if another_axisangle is not None and another_translation is not None:
            T = synth._transformation_from_parameters(axisangle + another_axisangle, translation + another_translation)
        else:
            T = synth._transformation_from_parameters(axisangle, translation)
        return T, axisangle, translation


class Convert:
    """preprocess.py:237-298; depth / disparity [1,H,W] or batched [B,1,H,W]."""

    @staticmethod
    def depth_to_disparity(depth, s=None):
        """s * B * f / depth with s = get_random(0.3, 0.8, False) (drawn unless given: [B] per image)."""
        if s is None:
            s = get_random(0.3, 0.8, random_sign=False)
        elif torch.is_tensor(s) and s.dim() == 1:
            s = s.to(depth.device).view(-1, *([1] * (depth.dim() - 1)))
        return s * Plausible.B() * Plausible.f() / depth

    @staticmethod
    def disparity_to_flow(disparity, device=None, random_sign=True):
        cdim = disparity.dim() - 3
        flow = torch.cat((disparity, torch.zeros_like(disparity)), dim=cdim) * -1.0
        if random_sign:
            flow = flow * get_random(0, 1)
        return flow.to(device) if device is not None else flow

    @staticmethod
    def disparity_to_depth(disparity):
        return Plausible.B() * Plausible.f() / (disparity + 0.005)

    @staticmethod
    def depth_to_random_flow(depth, device=None, segment=None, T1=None):
        """Ego-motion flow (preprocess.py:265-298, geometry.py:17-67); T1 drawn unless given."""
        if T1 is None:
            T1, _, _ = Plausible.random_motion(1. / 36., 1. / 36., 0.1, 0.1)
        batched = depth.dim() == 4
        d = depth if batched else depth.unsqueeze(0)
        T = T1 if T1.dim() == 3 else T1.unsqueeze(0)
        if T.shape[0] != d.shape[0]:
            T = T.expand(d.shape[0], 4, 4)
        if d.is_cuda:
            # the one-kernel flow plane (ops.ego_flow, bit-exact vs the
            # reference's CPU run: tests/test_ego.py; vs its CUDA run unpinned)
            P, ik = synth.projection(d.shape[-2], d.shape[-1], T, d.device)
            flow = ego_flow(d.contiguous(), P, ik)
        else:
            # host tensors (the reference's code accepts them): its own
            # arithmetic, as restated in synth (pinned by tests/golden)
            flow = synth.ego_motion_flow(d, T.to(d.device))
        if device is not None:
            flow = flow.to(device)
        return (flow if batched else flow[0]), T1


# ---------------------------------------------------------------- ConcatFlow / BackFlow
class ConcatFlow(nn.Module):
    """preprocess.py:301-313: flowAC = (FW(flowBC, back_flowAB, depthB) + flowAB) * valid."""

    def __init__(self, device=None):
        super().__init__()
        self.device = device
        self.fw = FW(device)

    def forward(self, flowAB, back_flowAB, flowBC, imgB_depth):
        with torch.no_grad():
            concat_flow, valid, collision = self.fw(flowBC, back_flowAB, imgB_depth)
        concat_flow = (concat_flow + flowAB) * valid
        return concat_flow.to(self.device) if self.device is not None else concat_flow, valid


class BackFlow(nn.Module):
    """preprocess.py:315-326: back flow = -FW(flowAB, flowAB, depthA) * valid."""

    def __init__(self, device=None):
        super().__init__()
        self.device = device
        self.fw = FW(device)

    def forward(self, flowAB, imgA_depth):
        with torch.no_grad():
            back_flow, valid, collision = self.fw(flowAB, flowAB, imgA_depth)
        back_flow = (back_flow * -1.0) * valid
        return back_flow.to(self.device) if self.device is not None else back_flow, valid


# ---------------------------------------------------------------- SpecialFlow
def _p0(h, w, device):
    ys, xs = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    return xs.to(torch.float32), ys.to(torch.float32)


def special_flow_from_params(h, w, kind, params, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """(special_flow, back_special_flow) [B,2,h,w] for per-image parameters.

    kind 5 = flip (vertical: a fresh SpecialFlow toggles horizontal_flip to
    False, preprocess.py:49-54), 6 = rotate (params [B,3]: cx, cy, theta),
    7 = shear (vertical for a fresh instance, :83-91; params [B]: shear).
    The rotation's 2x2 product (:74-75) rounds as the reference's matmul
    does (ops.rotation_flow on the device); the shear's (:94-95) has a zero
    term and is a multiply and an add."""
    x, y = _p0(h, w, device)
    if kind >= 7:
        s = params.to(device=device, dtype=torch.float32).view(-1, 1, 1)
        fy = (x * s + y) - y
        by = (x * (-s) + y) - y
        zero = torch.zeros_like(fy)
        return torch.stack((zero, fy), 1), torch.stack((zero, by), 1)
    if kind >= 6:
        # rotate / reverse_rotate built on the host from the drawn theta
        # exactly as :66-71 build them (torch.cos / sin of the float32 angle
        # and of its negation), then (p0 - c0) @ R + c0 - p0 per pixel
        p = params.detach().to(device="cpu", dtype=torch.float32)
        th = p[:, 2]
        mats = []
        for t in (th, -th):
            c, sn = torch.cos(t), torch.sin(t)
            mats.append(torch.stack((c, -sn, sn, c), 1))
        rp = torch.cat((p[:, 0:2], mats[0], mats[1]), 1)                  # [B,10]
        if torch.device(device).type == "cuda":
            return rotation_flow(rp, h, w, device)
        # host tensors: the reference's own matmul, image by image in its shapes
        p0 = torch.stack((x, y), -1)                                      # [h,w,2]
        out = []
        for k in (2, 6):
            fl = [((p0 - rp[b, 0:2]) @ rp[b, k:k + 4].view(2, 2) + rp[b, 0:2]) - p0 for b in range(rp.shape[0])]
            out.append(torch.stack(fl).permute(0, 3, 1, 2).contiguous())
        return out[0], out[1]
    B = params.shape[0] if params is not None else 1
    fy = (float(h - 1) - y) - y
    f = torch.stack((torch.zeros_like(fy), fy), 0).unsqueeze(0).expand(B, 2, h, w).contiguous()
    return f, f.clone()


class SpecialFlow(nn.Module):
    """preprocess.py:24-105 (flip / rotate / shear dense flows, with the
    instance's alternating flip and shear orientation)."""

    def __init__(self, device=None):
        super().__init__()
        self.device = device
        self.horizontal_flip = True
        self.horizontal_shear = True

    def forward(self, size, augment_flow_type):
        h, w = size
        dev = self.device if self.device is not None else "cpu"
        if augment_flow_type >= 7.:
            return self._shear(size)
        if augment_flow_type >= 6.:
            c0x = get_random(w / 4, w / 2) + w / 2
            c0y = get_random(h / 4, h / 2) + h / 2
            theta = torch.deg2rad(get_random(2, 8))
            f, b = special_flow_from_params(h, w, 6, torch.stack((c0x, c0y, theta)).view(1, 3), dev)
            return f[0], b[0]
        if augment_flow_type >= 5.:
            self.horizontal_flip = not self.horizontal_flip
            x, y = _p0(h, w, dev)
            if self.horizontal_flip:
                f = torch.stack(((float(w - 1) - x) - x, torch.zeros_like(x)), 0)
            else:
                f = torch.stack((torch.zeros_like(y), (float(h - 1) - y) - y), 0)
            return f, f.clone()
        raise ValueError(f"SpecialFlow: augment_flow_type {augment_flow_type} < 5")

    def _shear(self, size):
        h, w = size
        dev = self.device if self.device is not None else "cpu"
        self.horizontal_shear = not self.horizontal_shear
        s = get_random(0.15, 0.2)
        x, y = _p0(h, w, dev)
        if self.horizontal_shear:  # p0 @ [[1, 0], [s, 1]]: x' = x + y * s
            fx, bx = (x + y * s.to(dev)) - x, (x + y * (-s).to(dev)) - x
            z = torch.zeros_like(fx)
            return torch.stack((fx, z), 0), torch.stack((bx, z), 0)
        f, b = special_flow_from_params(h, w, 7, s.view(1), dev)
        return f[0], b[0]


# ---------------------------------------------------------------- augment_flow
def draw_augment_params(kind: int, h: int, w: int):
    """The torch CPU RNG draws augment_flow makes for one call of this type
    (preprocess.py:111, :64-66, :84, :157-162), in order."""
    if kind >= 7:
        return get_random(0.15, 0.2)
    if kind >= 6:
        c0x = get_random(w / 4, w / 2) + w / 2
        c0y = get_random(h / 4, h / 2) + h / 2
        theta = torch.deg2rad(get_random(2, 8))
        return torch.stack((c0x, c0y, theta)).to(torch.float32)
    if kind >= 2:  # flip, the unused 3-4 and gray draw nothing
        return None
    if kind >= 1:
        channel = int(get_random(3, 0, False))
        shift = get_random(10, 15)
        return (channel, shift)
    return get_random(1, 0, False)


def _stack_params(kind, params: List):
    if kind >= 7:
        return torch.stack([p.to(torch.float32) for p in params])
    if kind >= 6:
        return torch.stack(params)
    return None


def augment_flow_batch(img0, img0_depth, img1, img1_depth, flow01, back_flow01, kind, params: List,
                       fw: Optional[FW] = None, specials: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                       inpaint_fn=None):
    """augment_flow (preprocess.py:107-182) over a batch: every tensor [B,...],
    ``params`` the per-image draws of draw_augment_params.  Returns (set1, set2,
    kind, specials) like the reference (specials None for kinds < 5).
    ``specials`` optionally supplies the (special, back_special) flows;
    ``inpaint_fn`` replaces the hole-fill (default ops.inpaint)."""
    fw = fw or FW()
    inpaint_ = inpaint_fn or inpaint
    cf, bf = ConcatFlow(), BackFlow()
    B, _, h, w = img0.shape
    dev = img0.device
    if kind >= 5:
        if specials is not None:
            sf, bsf = specials
        else:
            sf, bsf = special_flow_from_params(h, w, kind, _stack_params(kind, params) if kind >= 6 else
                                               torch.zeros(B), dev)
        a0_flow, _ = cf(bsf, sf, flow01, img0_depth)
        a1_flow, _ = cf(flow01, back_flow01, sf, img1_depth)
        a0_all, valid0, coll0 = fw(torch.cat((img0, img0_depth), 1), sf, img0_depth)
        a1_all, valid1, coll1 = fw(torch.cat((img1, img1_depth), 1), sf, img1_depth)
        # the two hole-fills (:164, :170) in one call over 2B images: the fill
        # is per image, and one launch keeps twice the workgroups busy
        a01 = inpaint_(torch.cat((a0_all[:, 0:3], a1_all[:, 0:3])), torch.cat((valid0, valid1)),
                       torch.cat((coll0, coll1)))
        a0, a1 = a01[:B], a01[B:]
        a0_depth = fix_warped_depth(a0_all[:, 3:4])
        a1_depth = fix_warped_depth(a1_all[:, 3:4])
        back_a0_flow, _ = bf(a0_flow, a0_depth)
        back_a1_flow, _ = bf(a1_flow, img0_depth)
        return ((a0, a0_depth, a0_flow, back_a0_flow, img1, img1_depth),
                (img0, img0_depth, a1_flow, back_a1_flow, a1, a1_depth), int(kind), (sf, bsf))
    if kind >= 3:
        return None  # preprocess.py:148-149 (`pass`): the reference returns None
    if kind >= 2:
        g = torch.tensor(_GRAY, dtype=torch.float32, device=dev)
        fn = lambda im: (im.permute(0, 2, 3, 1) @ g).permute(0, 3, 1, 2)
    elif kind >= 1:
        shift = torch.zeros_like(img0)
        for b, (ch, v) in enumerate(params):
            shift[b, ch] = v.to(dev)
        fn = lambda im: im + shift
    else:
        sc = torch.stack([p.to(torch.float32) for p in params]).to(dev).view(-1, 1, 1, 1)
        fn = lambda im: im * sc
    return ((fn(img0), img0_depth, flow01, back_flow01, img1, img1_depth),
            (img0, img0_depth, flow01, back_flow01, fn(img1), img1_depth), int(kind), None)


def augment_flow(img0, img0_depth, img1, img1_depth, flow01, back_flow01, device=None, augment_flow_type=None):
    """Drop-in for preprocess.py:107-182 (3-D inputs), same RNG draws."""
    _, h, w = img0.shape
    if augment_flow_type is None:
        augment_flow_type = get_random(8, 0, False)
    kind = float(augment_flow_type)
    p = draw_augment_params(int(kind) if kind < 8 else 7, h, w)
    if 3. <= kind < 5.:
        return None
    res = augment_flow_batch(img0[None], img0_depth[None], img1[None], img1_depth[None], flow01[None],
                             back_flow01[None], kind, [p])
    set1, set2, k, spec = res
    set1 = tuple(t[0] for t in set1)
    set2 = tuple(t[0] for t in set2)
    if spec is not None:
        spec = (spec[0][0], spec[1][0])
    return set1, set2, k, spec


# ---------------------------------------------------------------- per-image RNG replay
def draw_image_params(seed: int, h: int, w: int, schedule: Sequence[int] = AUGMENT_SCHEDULE,
                      n_groups: int = N_GROUPS) -> Dict:
    """Everything PreprocessPlusAugment.forward draws from the torch CPU RNG for
    one image after utils.set_seed(seed) (preprocess.py:555), in draw order:
    s (:356 -> :240), T1 (:372 -> :277), then per (group, augment) the draws of
    augment_flow (:458).  The caller's RNG state is restored afterwards."""
    state = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)
        s = get_random(0.3, 0.8, random_sign=False)
        T1, _, _ = Plausible.random_motion(1. / 36., 1. / 36., 0.1, 0.1)
        aug = [[draw_augment_params(t, h, w) for t in schedule] for _ in range(n_groups)]
    finally:
        torch.random.set_rng_state(state)
    return {"s": s.to(torch.float32), "T1": T1[0], "augment": aug}


# ---------------------------------------------------------------- PreprocessPlusAugment
class PreprocessPlusAugment(nn.Module):
    """preprocess.py:329-506: first-stage warps of one image (7 FW calls, 5
    hole-fills) into the 44-channel group, then 5 x 12 augmentations."""

    def __init__(self, device, inpaint_fn=None, writer_workers: int = 0, compresslevel: int = 6):
        """``inpaint_fn`` replaces utils.inpaint (default: the GPU hole-fill,
        ops.inpaint); ``writer_workers`` > 0 writes the npz files from a
        thread pool (NpzWriter) that overlaps the copies and the zlib work
        with the GPU; ``compresslevel`` is the zip deflate level (6 =
        np.savez_compressed's)."""
        super().__init__()
        self.device = device
        self.fw = FW(device)
        self.cf = ConcatFlow(device)
        self.bf = BackFlow(device)
        self.inpaint_fn = inpaint_fn or inpaint
        self.writer = NpzWriter(writer_workers, compresslevel) if writer_workers > 0 else None
        # side streams for the augmentations: with the caller's stream, 4 =
        # the HIP runtime's hardware queues per process (GPU_MAX_HW_QUEUES);
        # more share queues and serialise (profiles/r03_pipeline_streams.txt)
        self.aug_streams = int(os.environ.get("OFD_PPA_STREAMS", "3"))
        self._streams = None

    # -- the first stage, batched: img0 [B,3,H,W], img0_depth [B,1,H,W] (raw), params per image
    def stage_one(self, img0, img0_depth, params: List[Dict]):
        fw, cf = self.fw, self.cf
        s = torch.stack([p["s"] for p in params])
        T1 = torch.stack([p["T1"] for p in params])
        img0_depth = normalize_depth(img0_depth)                                      # :355
        disp0 = Convert.depth_to_disparity(img0_depth, s)                              # :356
        flow01 = Convert.disparity_to_flow(disp0, random_sign=False)                   # :357
        # :358-359 as one fused warp (depth -> disparity -> flow inside the
        # kernel; bit-identical to fw(cat(img0, depth, -flow01), flow01, depth))
        o, img1_valid, coll = warp_disparity(img0.to(torch.float32).contiguous(), img0_depth.contiguous(), s)
        img1, img1_depth, back_flow01 = o[:, 0:3], o[:, 3:4], o[:, 4:6]
        img1 = img1 * img1_valid
        img1_depth = img1_depth * img1_valid
        back_flow01 = back_flow01 * img1_valid
        img1_depth = fix_warped_depth(img1_depth)
        coll1 = coll

        # :385-387 -- independent of img1's fill, so its hole-fill shares one
        # call with img1's (the fill is per image; one launch over 2B images
        # keeps twice the workgroups busy).  The ego-motion flow plane is a
        # group output, so the warp reads it (warp_flow_cat: obj's depth and
        # flow channels generated from the winner, the concatenation never
        # stored) instead of deriving the flow again.
        flow03, _ = Convert.depth_to_random_flow(img0_depth, T1=T1)                    # :385
        o, img3_valid, coll3 = warp_flow_cat(img0.to(torch.float32).contiguous(), flow03.contiguous(),
                                             img0_depth.contiguous())
        img3, img3_depth, back_flow03 = o[:, 0:3], o[:, 3:4], o[:, 4:6]
        img3 = img3 * img3_valid
        img3_depth = img3_depth * img3_valid
        back_flow03 = back_flow03 * img3_valid
        B = img1.shape[0]
        f13 = self.inpaint_fn(torch.cat((img1, img3)), torch.cat((img1_valid, img3_valid)),
                              torch.cat((coll1, coll3)))                                          # :366, :391
        img1, img3 = f13[:B], f13[B:]
        img3_depth = fix_warped_depth(img3_depth)

        # :372-373: bit-identical to
        # fw(cat(img1, img1_depth, flow12 * -1.0, img1_valid), flow12, img1_depth)
        flow12, _ = Convert.depth_to_random_flow(img1_depth, T1=T1)                    # :372
        o, valid, coll2 = warp_flow_cat(torch.cat((img1, img1_valid), 1).to(torch.float32), flow12.contiguous(),
                                        img1_depth.contiguous())
        img2, img2_depth, back_flow12, fw_img1_valid = o[:, 0:3], o[:, 3:4], o[:, 4:6], o[:, 6:7]
        img2_valid = valid * fw_img1_valid
        img2 = img2 * img2_valid
        img2_depth = img2_depth * img2_valid
        back_flow12 = back_flow12 * img2_valid
        img2_depth = fix_warped_depth(img2_depth)

        flow02, flow02_valid = cf(flow01, back_flow01, flow12, img1_depth)             # :400
        # :401-402 (fw(cat(img0, img0_depth, flow02 * -1.0, flow02_valid), flow02, img0_depth))
        o, valid, coll2p = warp_flow_cat(torch.cat((img0, flow02_valid), 1).to(torch.float32), flow02.contiguous(),
                                         img0_depth.contiguous())
        img2p, img2p_depth, back_flow02p, fw_flow02_valid = o[:, 0:3], o[:, 3:4], o[:, 4:6], o[:, 6:7]
        img2p_valid = valid * fw_flow02_valid
        img2p = img2p * img2p_valid
        img2p_depth = img2p_depth * img2p_valid
        back_flow02p = back_flow02p * img2p_valid
        img2p_depth = fix_warped_depth(img2p_depth)

        flow13, flow13_valid = cf(back_flow01, flow01, flow03, img1_depth)             # :414
        flow13_valid = flow13_valid * img1_valid
        # :416-417 (fw(cat(img1, img1_depth, flow13 * -1.0, flow13_valid), flow13, img1_depth))
        o, valid, coll3p = warp_flow_cat(torch.cat((img1, flow13_valid), 1).to(torch.float32), flow13.contiguous(),
                                         img1_depth.contiguous())
        img3p, img3p_depth, back_flow13p, fw_flow13_valid = o[:, 0:3], o[:, 3:4], o[:, 4:6], o[:, 6:7]
        img3p_valid = valid * fw_flow13_valid
        img3p = img3p * img3p_valid
        img3p_depth = img3p_depth * img3p_valid
        back_flow13p = back_flow13p * img3p_valid
        img3p_depth = fix_warped_depth(img3p_depth)

        # the three remaining hole-fills (:379, :407, :421) in one call over 3B images
        f = self.inpaint_fn(torch.cat((img2, img2p, img3p)), torch.cat((img2_valid, img2p_valid, img3p_valid)),
                            torch.cat((coll2, coll2p, coll3p)))
        img2, img2p, img3p = f[:B], f[B:2 * B], f[2 * B:]

        groups = [(img0, img0_depth, img1, img1_depth, flow01, back_flow01),           # :427-432
                  (img1, img1_depth, img2, img2_depth, flow12, back_flow12),
                  (img0, img0_depth, img2p, img2p_depth, flow02, back_flow02p),
                  (img0, img0_depth, img3, img3_depth, flow03, back_flow03),
                  (img1, img1_depth, img3p, img3p_depth, flow13, back_flow13p)]
        group44 = torch.cat((img0, img0_depth, img1, img1_depth, img2, img2_depth, img3, img3_depth,
                             img2p, img2p_depth, img3p, img3p_depth,
                             flow01, back_flow01, flow12, back_flow12, flow02, back_flow02p,
                             flow03, back_flow03, flow13, back_flow13p), 1)                # :437-440
        return group44, groups

    def augment(self, groups, params: List[Dict], schedule: Sequence[int] = AUGMENT_SCHEDULE):
        """Yields (group_idx, augment_idx, kind, data1 [B,8,H,W], data2 [B,8,H,W]) (preprocess.py:453-476).

        The augmentations are independent of each other, and each one's
        hole-fill (cv2's order: one workgroup per image, bound by the deepest
        image's chain) leaves most of the chip idle, so on the GPU they run
        round-robin on ``self.aug_streams`` side streams (OFD_PPA_STREAMS,
        default 3; 0 = the caller's stream): consecutive augmentations' warps
        and fills overlap.  Every yielded tensor is ready on the caller's
        stream (it waits for the augmentation's event), and the caller's
        stream waits for every side stream before the generator finishes."""
        dev = groups[0][0].device
        n_st = self.aug_streams if dev.type == "cuda" else 0
        main = torch.cuda.current_stream(dev) if n_st else None
        # created once per instance: each stream keeps its warp and hole-fill
        # workspaces (ops' per-stream caches) across batches
        if n_st and (self._streams is None or self._streams[0].device != dev):
            self._streams = [torch.cuda.Stream(dev) for _ in range(n_st)]
        streams = self._streams if n_st else []
        for st in streams:
            st.wait_stream(main)  # the groups were made on the caller's stream
        k = 0
        try:
            for g, (imgA, dA, imgB, dB, fAB, bAB) in enumerate(groups):
                for a, kind in enumerate(schedule):
                    ps = [p["augment"][g][a] for p in params]
                    if not streams:
                        set1, set2, _, _ = augment_flow_batch(imgA, dA, imgB, dB, fAB, bAB, kind, ps, self.fw,
                                                              inpaint_fn=self.inpaint_fn)
                        yield g, a, kind, torch.cat(set1[0:4], 1), torch.cat(set2[2:6], 1)
                        continue
                    st = streams[k % len(streams)]
                    k += 1
                    with torch.cuda.stream(st):
                        set1, set2, _, _ = augment_flow_batch(imgA, dA, imgB, dB, fAB, bAB, kind, ps, self.fw,
                                                              inpaint_fn=self.inpaint_fn)
                        d1, d2 = torch.cat(set1[0:4], 1), torch.cat(set2[2:6], 1)
                        ev = torch.cuda.Event()
                        ev.record(st)
                    main.wait_event(ev)
                    d1.record_stream(main)
                    d2.record_stream(main)
                    yield g, a, kind, d1, d2
        finally:
            for st in streams:
                main.wait_stream(st)

    def run_batch(self, seeds: Sequence[int], img0, img0_depth, is_stereo=False, out_dirs=None,
                  schedule: Sequence[int] = AUGMENT_SCHEDULE, augment=True, camera=None):
        """B images at once.  ``img0_depth`` is the raw depth (or the disparity
        when is_stereo, :352-353).  With ``out_dirs`` every image's npz files
        are written like the reference; returns the group tensor [B,44,H,W].
        ``camera`` = (s [B], T [B,4,4]) replaces the per-seed draws of the
        camera scale and ego-motion (shard.broadcast_camera_params: rank 0's
        draws, bit-identical to every rank's own)."""
        h, w = img0.shape[-2:]
        params = [draw_image_params(int(s), h, w, schedule) for s in seeds]
        if camera is not None:
            for p, s_i, T_i in zip(params, camera[0], camera[1]):
                p["s"] = s_i.to(torch.float32)
                p["T1"] = T_i.to(torch.float32)
        img0 = img0.to(self.device)
        d0 = img0_depth.to(self.device)
        if is_stereo:
            d0 = Convert.disparity_to_depth(d0)
        group44, groups = self.stage_one(img0, d0, params)
        if out_dirs is not None:
            save_group(out_dirs, group44, self.writer)
        if augment:
            for g, a, kind, d1, d2 in self.augment(groups, params, schedule):
                if out_dirs is not None:
                    save_augment(out_dirs, g, a, kind, d1, d2, self.writer)
        if self.writer is not None:
            self.writer.flush()
        check_fill_faults(out_dirs, self.device)
        return group44

    def forward(self, datas, output_dir, is_stereo=False, n_continuous=4):
        """preprocess.py:341-506 for one image under the caller's current RNG
        state (the reference seeds with utils.set_seed before each call)."""
        if not is_stereo:
            img0, d0 = datas
        else:
            img0, _, d0 = datas
        h, w = img0.shape[-2:]
        # the draws use the global RNG in the reference's order (see draw_image_params)
        s = get_random(0.3, 0.8, random_sign=False)
        T1, _, _ = Plausible.random_motion(1. / 36., 1. / 36., 0.1, 0.1)
        aug = [[draw_augment_params(t, h, w) for t in AUGMENT_SCHEDULE] for _ in range(N_GROUPS)]
        params = [{"s": s.to(torch.float32), "T1": T1[0], "augment": aug}]
        img0 = img0.to(self.device)[None]
        d0 = d0.to(self.device)[None]
        if is_stereo:
            d0 = Convert.disparity_to_depth(d0)
        os.makedirs(output_dir, exist_ok=True)
        group44, groups = self.stage_one(img0, d0, params)
        save_group([output_dir], group44, self.writer)
        for g, a, kind, d1, d2 in self.augment(groups, params):
            save_augment([output_dir], g, a, kind, d1, d2, self.writer)
        if self.writer is not None:
            self.writer.flush()
        check_fill_faults([output_dir], self.device)


def check_fill_faults(out_dirs: Optional[Sequence[str]], device) -> None:
    """After a batch: raise if any hole-fill of it hit a bounded wait or bound
    (ops.inpaint_faults; unreachable while the fill's invariants hold).  The
    batch's files are removed first, so no wrong fill is left on disk and a
    --skip-existing run redoes those images."""
    if torch.device(device).type != "cuda":
        return
    from . import ops
    bits = ops.inpaint_faults(reset=True)
    if not bits:
        return
    for d in out_dirs or ():
        for f in os.listdir(d) if os.path.isdir(d) else ():
            if f.endswith(".npz"):
                os.remove(os.path.join(d, f))
    raise RuntimeError(f"hole-fill fault bits {bits:#x} (include/ofd_inpaint.h ofd_inpaint_faults): "
                       f"the batch's fills are incomplete; its files were removed")


# ---------------------------------------------------------------- npz writer
def write_npz(path: str, compresslevel: int = 6, **arrays) -> None:
    """np.savez_compressed's file (a deflated zip of .npy members, read back
    by np.load) with a chosen zlib level; level 6 is numpy's own."""
    import zipfile
    from numpy.lib import format as npformat
    with atomic_path(path) as tmp, zipfile.ZipFile(tmp, mode="w", compression=zipfile.ZIP_DEFLATED,
                                                   compresslevel=compresslevel, allowZip64=True) as zf:
        for k, v in arrays.items():
            with zf.open(k + ".npy", mode="w", force_zip64=True) as f:
                npformat.write_array(f, np.asanyarray(v), allow_pickle=False)


def savez_compressed(path: str, **arrays) -> None:
    """np.savez_compressed (preprocess.py:446, :471-476) into a temporary file
    renamed onto ``path`` once complete."""
    with atomic_path(path) as tmp, open(tmp, "wb") as f:
        np.savez_compressed(f, **arrays)


class NpzWriter:
    """The npz files of preprocess.py:446, :471-476 written off the GPU's
    critical path: each save copies the tensor to pinned host memory on the
    current stream (non-blocking) behind an event, and a thread pool waits
    for the event, then deflates and writes (zlib releases the GIL, so the
    workers compress in parallel).  Pending bytes are capped: a save blocks
    while more than ``max_pending_bytes`` wait to be written."""

    def __init__(self, workers: int = 16, compresslevel: int = 6, max_pending_bytes: int = 8 << 30):
        import threading
        from concurrent.futures import ThreadPoolExecutor
        self.pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="npz")
        self.level = compresslevel
        self.cap = max_pending_bytes
        self.pending = 0
        self.cv = threading.Condition()
        self.futures = []
        self.bytes_written = 0

    def _host(self, t):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            return h
        return t

    def save(self, path: str, **arrays) -> None:
        nbytes = sum(int(t.numel() * t.element_size()) for t in arrays.values() if isinstance(t, torch.Tensor))
        with self.cv:
            while self.pending > 0 and self.pending + nbytes > self.cap:
                self.cv.wait()
            self.pending += nbytes
        host = {k: self._host(v) for k, v in arrays.items()}
        ev = torch.cuda.Event() if any(isinstance(v, torch.Tensor) and v.is_pinned() for v in host.values()) else None
        if ev is not None:
            ev.record()

        def job():
            try:
                if ev is not None:
                    ev.synchronize()
                write_npz(path, self.level, **{k: (v.numpy() if isinstance(v, torch.Tensor) else v)
                                               for k, v in host.items()})
            finally:
                with self.cv:
                    self.pending -= nbytes
                    self.bytes_written += nbytes
                    self.cv.notify_all()
        self.futures.append(self.pool.submit(job))

    def flush(self) -> None:
        """Wait for every pending file, then re-raise the first write error."""
        futs, self.futures = self.futures, []
        first = None
        for f in futs:
            try:
                f.result()
            except BaseException as e:  # noqa: BLE001 - re-raised below
                if first is None:
                    first = e
        if first is not None:
            raise first

    def close(self) -> None:
        self.flush()
        self.pool.shutdown()


def save_group(out_dirs: Sequence[str], group44: torch.Tensor, writer: Optional[NpzWriter] = None) -> None:
    """group.npz, key img_depth_flow = [44,H,W] (preprocess.py:434-447)."""
    assert group44.shape[1] == 44, "wrong data shape"
    if writer is not None and hasattr(writer, "save_batch"):  # GpuNpzWriter: one deflate launch for the batch
        for d in out_dirs:
            os.makedirs(d, exist_ok=True)
        writer.save_batch([os.path.join(d, "group.npz") for d in out_dirs], group44.detach(), "img_depth_flow")
        return
    for d, x in zip(out_dirs, group44.detach()):
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "group.npz")
        if writer is not None:
            writer.save(path, img_depth_flow=x)
        else:
            savez_compressed(path, img_depth_flow=x.cpu().numpy())


def save_augment(out_dirs: Sequence[str], g: int, a: int, kind: int, d1: torch.Tensor, d2: torch.Tensor,
                 writer: Optional[NpzWriter] = None) -> None:
    """{g}_{a}_1.npz / {g}_{a}_2.npz, keys img_depth_flow [8,H,W] and
    augment_flow_type (preprocess.py:462-476)."""
    assert d1.shape[1] == 8 and d2.shape[1] == 8
    if writer is not None and hasattr(writer, "save_batch"):
        for k, x in ((1, d1), (2, d2)):
            writer.save_batch([os.path.join(d, f"{g}_{a}_{k}.npz") for d in out_dirs], x.detach(), "img_depth_flow",
                              {"augment_flow_type": np.array(kind)})
        return
    for d, x1, x2 in zip(out_dirs, d1.detach(), d2.detach()):
        for k, x in ((1, x1), (2, x2)):
            path = os.path.join(d, f"{g}_{a}_{k}.npz")
            if writer is not None:
                writer.save(path, img_depth_flow=x, augment_flow_type=np.array(kind))
            else:
                savez_compressed(path, img_depth_flow=x.cpu().numpy(), augment_flow_type=kind)


# ---------------------------------------------------------------- driver (preprocess.py:508-561)
N_FILES_PER_IMAGE = 1 + 2 * N_GROUPS * len(AUGMENT_SCHEDULE)  # group.npz + 120 augmented pairs


def image_complete(d: str, schedule: Sequence[int] = AUGMENT_SCHEDULE, augment: bool = True) -> bool:
    """Every product file of one image exists and was finished (resume:
    --skip-existing).  The writers rename a file into place only once it is
    complete; a file that still ends without a zip end record (e.g. left by
    an older, interrupted writer) makes the image incomplete."""
    names = ["group.npz"]
    if augment:
        names += [f"{g}_{a}_{k}.npz" for g in range(N_GROUPS) for a in range(len(schedule)) for k in (1, 2)]
    return all(zip_complete(os.path.join(d, n)) for n in names)


def make_writer(kind: str):
    """--writer: ``gpu`` (default) deflates on the GPU (npz_gpu.GpuNpzWriter),
    ``zlib`` a 16-thread host zlib pool (NpzWriter, numpy's level 6),
    ``sync`` the reference's synchronous np.savez_compressed (preprocess.py:446)."""
    if kind == "gpu":
        from .npz_gpu import GpuNpzWriter
        return GpuNpzWriter(workers=int(os.environ.get("OFD_WRITER_WORKERS", "8")))
    if kind == "zlib":
        return NpzWriter(int(os.environ.get("OFD_WRITER_WORKERS", "16")), 6)
    if kind == "sync":
        return None
    raise ValueError(f"unknown writer {kind!r}")


def main(argv=None) -> dict:
    """``python -m opticalflowfromdepth_amd.preprocess`` -- the reference's
    ``__main__`` (preprocess.py:521-561) on synthetic depth maps (the DIML /
    ReDWeb readers are file I/O, out of scope): the same --gpu / --split /
    --split_id sharding (shard.shard_range), the same per-image seeds
    12345 + img_idx + epoch * N over two epochs, the same output tree
    (<out>/<img_idx + epoch * N>/group.npz and {g}_{a}_{1,2}.npz), B images
    per batched call.  Under torchrun (WORLD_SIZE set) it joins a process
    group (RCCL; OFD_PPA_BACKEND=gloo for CPU collectives), --split /
    --split_id default to the world size / rank (one process per GPU), and the
    camera parameters (s, T) of every image of an epoch come from rank 0 in
    one broadcast (shard.broadcast_camera_params); the data path has no
    collective.  The files are written by the GPU deflate writer by default
    (--writer).  Returns (and prints as one JSON line) this rank's images,
    files, bytes and images/s with every file written."""
    import argparse
    import json
    import time
    import torch.distributed as dist
    from . import shard
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="synthetic", choices=["synthetic"])
    ap.add_argument("--n-images", type=int, default=8, help="synthetic dataset size")
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--gpu", default=None, type=int)
    ap.add_argument("--split", default=None, type=int)
    ap.add_argument("--split_id", default=None, type=int)
    ap.add_argument("--epochs", default=2, type=int)
    ap.add_argument("--batch", default=8, type=int,
                    help="images per batched call (larger batches amortise the hole-fill latency; the writer "
                         "bounds the product at any batch)")
    ap.add_argument("--out", default="datasets/AugmentedDatasets/synthetic")
    ap.add_argument("--writer", default="gpu", choices=["gpu", "zlib", "sync"])
    ap.add_argument("--skip-existing", action="store_true", help="resume: skip images whose 121 files exist")
    ap.add_argument("--no-augment", action="store_true")
    ap.add_argument("--no-save", action="store_true")
    a = ap.parse_args(argv)
    launched = "WORLD_SIZE" in os.environ
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    split = a.split if a.split is not None else world
    split_id = a.split_id if a.split_id is not None else rank
    gpu = a.gpu if a.gpu is not None else int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    backend = os.environ.get("OFD_PPA_BACKEND", "nccl")
    if launched and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    N, h, w = a.n_images, a.height, a.width
    start, end = shard.shard_range(N, split, split_id)
    writer = None if a.no_save else make_writer(a.writer)
    ppa = PreprocessPlusAugment(dev)
    ppa.writer = writer
    done = skipped = 0
    t0 = time.perf_counter()
    try:
        for epoch in range(a.epochs):
            # every rank takes part in the broadcast of the whole epoch's camera
            # parameters (17 floats per image), then keeps its own shard's
            seeds_all = [shard.image_seed(i, epoch, N) for i in range(N)]
            s_all, T_all = shard.broadcast_camera_params(seeds_all, device=coll_dev)
            todo = list(range(start, end))
            if a.skip_existing and not a.no_save:
                keep = [i for i in todo if not image_complete(os.path.join(a.out, str(i + epoch * N)),
                                                              augment=not a.no_augment)]
                skipped += len(todo) - len(keep)
                todo = keep
            for b0 in range(0, len(todo), a.batch):
                idx = todo[b0:b0 + a.batch]
                seeds = [seeds_all[i] for i in idx]
                img0 = synth.synthetic_rgb(seeds, h, w, dev)
                depth = synth.synthetic_depth(seeds, h, w, dev, dtype=torch.float64)  # utils.get_depth is float64
                dirs = None if a.no_save else [os.path.join(a.out, str(i + epoch * N)) for i in idx]
                ppa.run_batch(seeds, img0, depth, out_dirs=dirs, augment=not a.no_augment,
                              camera=(s_all[idx], T_all[idx]))
                done += len(idx)
                print(f"rank {rank}: epoch {epoch} images {idx[0]}..{idx[-1]} done", flush=True)
        if writer is not None:
            writer.flush()
        torch.cuda.synchronize(dev)
    finally:
        if writer is not None and hasattr(writer, "close"):
            writer.close()
    el = time.perf_counter() - t0
    rep = {"rank": rank, "split": split, "split_id": split_id, "shard": [start, end], "epochs": a.epochs,
           "images": done, "skipped": skipped, "height": h, "width": w, "batch": a.batch,
           "writer": None if a.no_save else a.writer,
           "files": 0 if a.no_save else done * (N_FILES_PER_IMAGE if not a.no_augment else 1),
           "bytes_written": getattr(writer, "bytes_written", None), "seconds": round(el, 3),
           "images_per_s": round(done / el, 3) if el > 0 else None}
    print(json.dumps(rep), flush=True)
    if launched and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return rep


if __name__ == "__main__":
    main()
