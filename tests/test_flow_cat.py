"""GPU parity of ops.warp_flow_cat (include/ofd_fw.h ofd_fw_warp_flow_cat).

preprocess.py:371-373, :385-387, :400-402 and :414-417 all call
FW(torch.cat((img, depth, flow * -1.0[, mask])), flow, depth).  warp_flow_cat
takes the flow plane and generates obj's depth and flow channels from the
winner instead of concatenating; the bar is bit-identity with
forward_warp_flow on the materialised concatenation (cast to float32 as
fw.py:40 does) and with the oracle, for every flow / depth dtype pair.
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _cat_reference(obj, flow, depth):
    """The reference's concatenation (torch promotes to the widest dtype), then float32."""
    ob = torch.cat((obj[:, :3], depth, flow * -1.0, obj[:, 3:]), 1)
    return ob.float()


@pytest.mark.parametrize("flow_dt,depth_dt", [(np.float32, np.float32), (np.float32, np.float64),
                                              (np.float64, np.float32), (np.float64, np.float64)])
@pytest.mark.parametrize("cobj", [3, 4, 1, 0])
def test_warp_flow_cat_vs_concatenation(cuda_device, flow_dt, depth_dt, cobj):
    from opticalflowfromdepth_amd import forward_warp_flow, warp_flow_cat
    rng = np.random.default_rng(cobj * 10 + (flow_dt == np.float64) * 2 + (depth_dt == np.float64))
    B, H, W = 3, 45, 68
    obj = rng.integers(0, 256, (B, cobj, H, W)).astype(np.float32)
    flow = (rng.standard_normal((B, 2, H, W)) * 12).astype(flow_dt)
    flow[0, :, :5, :5] = 1e5                                     # border hot spot
    flow[1, 0, 3, 3] = np.nan
    depth = (rng.integers(0, 5, (B, 1, H, W)) * 0.5).astype(depth_dt)   # ties, zeros (key decodes 0)
    depth[rng.random(depth.shape) < 0.03] = -0.0
    depth[rng.random(depth.shape) < 0.03] = 1500.0                      # collision path
    depth[rng.random(depth.shape) < 0.02] = np.nan
    o, f, d = _t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device)
    got = warp_flow_cat(o, f, d)
    catobj = _cat_reference(o, f, d).contiguous()
    ref = forward_warp_flow(catobj, f, d.float().contiguous())
    for x, y in zip(got, ref):
        assert torch.equal(x, y)
    exp = oracle.fw_flow(catobj.cpu().numpy(), flow, depth.astype(np.float32))
    for g, e in zip(got, exp):
        assert np.array_equal(g.cpu().numpy(), e)


def test_warp_flow_cat_equals_warp_ego_on_the_ego_plane(cuda_device):
    """On ego_flow's plane, warp_flow_cat is the pipeline's replacement for
    warp_ego (preprocess.py:385-387): identical outputs."""
    from opticalflowfromdepth_amd import ego_flow, synth, warp_ego, warp_flow_cat
    B, H, W = 4, 96, 128
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, cuda_device, dtype=torch.float64))
    rgb = synth.synthetic_rgb(seeds, H, W, cuda_device)
    T = synth.batch_camera_params(seeds)[1].to(cuda_device)
    P, ik = synth.projection(H, W, T, cuda_device)
    flow = ego_flow(depth, P, ik)
    a = warp_ego(rgb, depth, P, ik)
    b = warp_flow_cat(rgb, flow, depth)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_warp_flow_cat_headline_shape(cuda_device):
    """64 x 768x1024 ego-motion images with their float64 depth: equal to FW
    on the concatenation for every image (size-independent property)."""
    from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, synth, warp_flow_cat
    B, H, W = 16, 768, 1024
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, cuda_device, dtype=torch.float64))
    rgb = synth.synthetic_rgb(seeds, H, W, cuda_device)
    T = synth.batch_camera_params(seeds)[1].to(cuda_device)
    P, ik = synth.projection(H, W, T, cuda_device)
    flow = ego_flow(depth, P, ik)
    got = warp_flow_cat(rgb, flow, depth)
    ref = forward_warp_flow(_cat_reference(rgb, flow, depth).contiguous(), flow, depth.float().contiguous())
    for x, y in zip(got, ref):
        assert torch.equal(x, y)
