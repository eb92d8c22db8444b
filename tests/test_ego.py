"""Ego-motion flow and the fused ego-motion warp.

Reference: Convert.depth_to_random_flow (preprocess.py:265-298) with
geometry.BackprojectDepth / Project3D (geometry.py:17-67), and the first
stage's ego-motion warps (preprocess.py:371-373, :385-387).

Parity bar:
* the parity bar: the flow plane (ops.ego_flow) equals the reference's own
  CPU runs bit for bit (tests/golden/pipeline.npz, ppa_fill_large.npz: since
  round 5 P = K @ T is multiplied on the host in the reference's shapes).
  The reference pipeline itself runs on cuda:{gpu}; its device GEMM rounding
  cannot be reproduced here (no CUDA device), so parity with that run is
  unpinned;
* a cross-check, not the parity bar: against this repo's torch restatement
  evaluated on the GPU (torch's device GEMMs round differently) the flows
  agree within a tolerance -- |d flow| <= 8 ulp of
  max(|p1|, size - 1) per axis (TOL_ULP below; p1 is computed in the
  normalised [-1, 1] domain and scaled by (size - 1) / 2, so its rounding
  error is set by the image size, not by |p1|: 9.5e-6 at 60x80, ~6e-5 at
  768x1024, where 1 ulp of 1023 is 6.1e-5);
* the fused warp (ops.warp_ego) is bit-identical to FW on ops.ego_flow's plane
  (one device function computes the flow for both);
* against FW on the reference-arithmetic flow, the targets whose truncated
  p1 flips because the flow moved by rounding are counted and reported; the
  bar is a flip rate below 1e-4 of the sources.
"""
import os

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import oracle

TOL_ULP = 8


def _tol(flow_ref, h, w):
    """8 ulp of max(|p1|, size - 1) per element and axis (float32)."""
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
    p1 = np.abs(np.stack([xx, yy]) + flow_ref)
    size = np.array([w - 1, h - 1], np.float32).reshape(2, 1, 1)
    return TOL_ULP * np.spacing(np.maximum(np.maximum(p1, size), 1.0).astype(np.float32))


def _golden():
    return np.load(os.path.join(REPO, "tests", "golden", "pipeline.npz"))


@pytest.mark.gpu
@pytest.mark.parametrize("img", ["img0", "img1"])
def test_ego_flow_vs_reference_fixture(img):
    """flow03 of the golden pipeline, the reference's own code on float32
    depth: bit for bit (round 5: P = K @ T multiplied on the host in the
    reference's shapes, synth.projection; the per-pixel sequence -- k-order
    fused multiply-adds, IEEE divisions -- is the reference's CPU rounding)."""
    from opticalflowfromdepth_amd import ego_flow, synth
    g = _golden()
    d = torch.from_numpy(g[f"{img}/norm_depth"]).float()[None]  # preprocess.py:385 passes float32 here
    h, w = d.shape[-2:]
    dev = torch.device("cuda:0")
    P, ik = synth.projection(h, w, torch.from_numpy(g[f"{img}/T1"]), dev)
    got = ego_flow(d.to(dev), P, ik)[0].cpu().numpy()
    ref = g[f"{img}/flow03"]
    assert np.array_equal(got, ref), int((got != ref).sum())


@pytest.mark.gpu
def test_ego_flow_float64_depth_vs_reference_run():
    """flow03 of the 192x256 pipeline fixture (preprocess.py:385 on the
    float64 normalised depth, the reference's run, ppa_fill_large.npz): bit
    for bit."""
    from opticalflowfromdepth_amd import ego_flow, synth
    z = np.load(os.path.join(REPO, "tests", "golden", "ppa_fill_large.npz"))
    h, w = int(z["h"]), int(z["w"])
    _, T = synth.camera_params(int(z["seeds"][0]))
    d0 = synth.normalize_depth(torch.from_numpy(z["i0/raw_depth"].copy())[None, None])
    assert d0.dtype == torch.float64
    dev = torch.device("cuda:0")
    P, ik = synth.projection(h, w, T[None], dev)
    got = ego_flow(d0.to(dev), P, ik)[0].cpu().numpy()
    assert np.array_equal(got, z["i0/ref_flow03"]), int((got != z["i0/ref_flow03"]).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(4, 48, 64), (2, 37, 53), (2, 368, 560), (1, 768, 1024)])
def test_ego_flow_vs_torch_restatement(dtype, shape):
    from opticalflowfromdepth_amd import ego_flow, synth
    B, H, W = shape
    dev = torch.device("cuda:0")
    seeds = [900 + H + i for i in range(B)]
    d = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64)).to(dtype)
    T = synth.batch_camera_params(seeds)[1]
    ref = synth.ego_motion_flow(d, T)
    P, ik = synth.projection(H, W, T, dev)
    got = ego_flow(d, P, ik)
    for b in range(B):
        r = ref[b].cpu().numpy()
        err = np.abs(got[b].cpu().numpy() - r)
        assert (err <= _tol(r, H, W)).all(), (b, float(err.max()))


def _inputs(B, H, W, dtype, seed, extra):
    from opticalflowfromdepth_amd import synth
    dev = torch.device("cuda:0")
    seeds = [seed + i for i in range(B)]
    d = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64)).to(dtype)
    rgb = synth.synthetic_rgb(seeds, H, W, dev)
    T = synth.batch_camera_params(seeds)[1]
    P, ik = synth.projection(H, W, T, dev)
    ex = (torch.rand(B, extra, H, W, generator=torch.Generator().manual_seed(seed)) > 0.5).float().to(dev)
    return rgb, d, T, P, ik, ex


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape,extra", [((3, 48, 64), 0), ((2, 37, 53), 1), ((1, 2, 9), 0), ((2, 96, 128), 2)])
def test_warp_ego_bit_exact_vs_fw_on_its_flow(dtype, shape, extra):
    from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, warp_ego
    B, H, W = shape
    rgb, d, T, P, ik, ex = _inputs(B, H, W, dtype, 300 + H, extra)
    flow = ego_flow(d, P, ik)
    obj = torch.cat((rgb, d.float(), flow * -1.0, ex), 1)
    exp = forward_warp_flow(obj, flow, d.float())
    got = warp_ego(torch.cat((rgb, ex), 1), d, P, ik)
    for g_, e_, n in zip(got, exp, ("output", "valid", "collision")):
        assert torch.equal(g_, e_), n
    # and the oracle agrees with FW on that flow
    cpu = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), d.float().cpu().numpy())
    for g_, c_, n in zip(got, cpu, ("output", "valid", "collision")):
        assert np.array_equal(g_.cpu().numpy(), c_), n


@pytest.mark.gpu
def test_warp_ego_headline_batch_and_flip_rate():
    """64 x 768x1024 float64 depth (preprocess.py:385's img0_depth): the fused
    warp equals FW on ego_flow's plane bit for bit; against FW on the torch
    restatement's flow, the sources whose target moved by a rounding flip are
    counted (reported in the assertion message) and must stay below 1e-4."""
    from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, synth, warp_ego
    B, H, W = 64, 768, 1024
    rgb, d, T, P, ik, _ = _inputs(B, H, W, torch.float64, 12345, 0)
    flow = ego_flow(d, P, ik)
    got = warp_ego(rgb, d, P, ik)
    exp = forward_warp_flow(torch.cat((rgb, d.float(), flow * -1.0), 1), flow, d.float())
    for g_, e_ in zip(got, exp):
        assert torch.equal(g_, e_)
    ref = synth.ego_motion_flow(d, T)
    ys, xs = torch.meshgrid(torch.arange(H, device=d.device), torch.arange(W, device=d.device), indexing="ij")

    def targets(f):
        tx = torch.clamp(xs.float() + f[:, 0], 0, W - 1).long()
        ty = torch.clamp(ys.float() + f[:, 1], 0, H - 1).long()
        return tx, ty
    (ax, ay), (bx, by) = targets(flow), targets(ref)
    flips = int(((ax != bx) | (ay != by)).sum())
    rate = flips / (B * H * W)
    assert rate < 1e-4, f"{flips} flipped sources ({rate:.2e})"


@pytest.mark.gpu
def test_warp_ego_argument_errors():
    from opticalflowfromdepth_amd import ego_flow, warp_ego
    dev = torch.device("cuda:0")
    d = torch.ones(2, 1, 8, 8, device=dev)
    P = torch.zeros(2, 3, 4, device=dev)
    ik = torch.eye(3)
    with pytest.raises(RuntimeError, match="P must have shape"):
        ego_flow(d, P[:1], ik)
    with pytest.raises(RuntimeError, match="inv_K"):
        ego_flow(d, P, torch.eye(4))
    with pytest.raises(RuntimeError, match="depth must have shape"):
        warp_ego(torch.zeros(2, 3, 8, 8, device=dev), d[:1], P, ik)


def test_projection_matches_reference_K():
    """synth.projection's inv_K is the reference's (pipeline.npz invK_768x1024, Plausible.K)."""
    from opticalflowfromdepth_amd import synth
    g = _golden()
    P, ik = synth.projection(768, 1024, torch.eye(4)[None], "cpu")
    assert np.array_equal(ik.numpy(), g["invK_768x1024"][0, :3, :3])
    assert np.array_equal(P[0].numpy(), g["K_768x1024"][0, :3, :])
