"""Fused depth -> disparity -> flow -> splat (preprocess.py:356-359).

ops.warp_disparity must equal, bit for bit, the unfused sequence the
reference runs: flow = disparity_to_flow(depth_to_disparity(depth)),
obj = cat(rgb, depth, -flow[, extra]), FW(obj, flow, depth) -- both through
this repo's FW and through the CPU oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle


def _inputs(B, H, W, dtype, seed, extra=0):
    from opticalflowfromdepth_amd import synth
    seeds = [seed + i for i in range(B)]
    d = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, "cpu", dtype=torch.float64)).to(dtype)
    rgb = synth.synthetic_rgb(seeds, H, W, "cpu")
    s = synth.batch_camera_params(seeds)[0]
    ex = (torch.rand(B, extra, H, W, generator=torch.Generator().manual_seed(seed)) > 0.5).to(torch.float32)
    return rgb, d, s, ex


def _unfused(rgb, d, s, ex):
    from opticalflowfromdepth_amd import preprocess as pp
    flow = pp.Convert.disparity_to_flow(pp.Convert.depth_to_disparity(d, s), random_sign=False)
    obj = torch.cat((rgb, d, flow * -1.0, ex), 1).to(torch.float32)
    return obj, flow


def test_unfused_reference_sequence_on_cpu_matches_fixture_flow():
    """The unfused sequence used as the expectation is the reference's (pipeline.npz flow01)."""
    import os
    from conftest import REPO
    from opticalflowfromdepth_amd import preprocess as pp, synth
    g = np.load(os.path.join(REPO, "tests", "golden", "pipeline.npz"))
    d0 = torch.from_numpy(g["img0/norm_depth"])[None]
    torch.manual_seed(int(g["img0/seed"]))
    s = synth.get_random(0.3, 0.8, random_sign=False).view(1)
    flow = pp.Convert.disparity_to_flow(pp.Convert.depth_to_disparity(d0, s), random_sign=False)
    assert np.array_equal(flow[0].numpy(), g["img0/flow01"])


@pytest.fixture(params=[1, 0], ids=["rows", "tile"])
def disparity_engine(request):
    """The disparity warps' row kernel (default) and the TILE engine."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_fw_set_disparity_rows(request.param)
    yield request.param
    lib.ofd_fw_set_disparity_rows(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape,extra", [((3, 48, 64), 0), ((2, 37, 53), 1), ((1, 2, 9), 0), ((2, 96, 128), 2)])
def test_warp_disparity_bit_exact(dtype, shape, extra, disparity_engine):
    from opticalflowfromdepth_amd import forward_warp_flow, warp_disparity
    B, H, W = shape
    rgb, d, s, ex = _inputs(B, H, W, dtype, 100 + H, extra)
    obj, flow = _unfused(rgb, d, s, ex)
    dev = torch.device("cuda:0")
    objd = torch.cat((rgb, ex), 1).to(dev)
    got = warp_disparity(objd, d.to(dev), s)
    exp_gpu = forward_warp_flow(obj.to(dev), flow.to(dev), d.to(dev).to(torch.float32))
    exp_cpu = oracle.fw_flow(obj.numpy(), flow.numpy(), d.to(torch.float32).numpy())
    for g_, e_, c_, n in zip(got, exp_gpu, exp_cpu, ("output", "valid", "collision")):
        g_ = g_.cpu().numpy()
        assert np.array_equal(g_, e_.cpu().numpy()), n
        assert np.array_equal(g_, c_), n


@pytest.mark.gpu
def test_warp_disparity_obj_without_rgb_and_errors():
    from opticalflowfromdepth_amd import warp_disparity
    dev = torch.device("cuda:0")
    rgb, d, s, ex = _inputs(2, 16, 20, torch.float32, 5)
    obj, flow = _unfused(rgb[:, :0], d, s, ex)  # Cobj = 0: output = depth, disparity, +0
    got = warp_disparity(torch.empty(2, 0, 16, 20, device=dev), d.to(dev), s)
    exp = oracle.fw_flow(obj.numpy(), flow.numpy(), d.numpy())
    assert all(np.array_equal(g.cpu().numpy(), e) for g, e in zip(got, exp))
    with pytest.raises(RuntimeError):
        warp_disparity(rgb.to(dev), d.to(dev), s[:1])


@pytest.mark.gpu
def test_warp_disparity_headline_batch():
    """64 x 768x1024 float64 depth (utils.get_depth's dtype), every image vs the unfused FW."""
    from opticalflowfromdepth_amd import forward_warp_flow, warp_disparity
    dev = torch.device("cuda:0")
    rgb, d, s, ex = _inputs(64, 768, 1024, torch.float64, 12345)
    obj, flow = _unfused(rgb, d, s, ex)
    got = warp_disparity(rgb.to(dev), d.to(dev), s)
    exp = forward_warp_flow(obj.to(dev), flow.to(dev), d.to(dev).to(torch.float32))
    for g_, e_ in zip(got, exp):
        assert torch.equal(g_, e_)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("W", [64, 53])
def test_warp_disparity_special_depths(dtype, W, disparity_engine):
    """The row kernel (one workgroup per image row, 16-byte and scalar lanes)
    on depths the reference's z-test treats specially: 0 (infinite disparity,
    clamped onto column 0), NaN (dropped), >= 1000 (lands, never wins: a
    collision), negative and -0.0 (win), and runs of equal depths (ties go to
    the first source in raster order)."""
    from opticalflowfromdepth_amd import forward_warp_flow, warp_disparity
    B, H = 2, 12
    rgb, d, s, ex = _inputs(B, H, W, dtype, 77, 1)
    g = torch.Generator().manual_seed(3)
    pick = torch.rand(B, 1, H, W, generator=g)
    specials = torch.tensor([0.0, float("nan"), 1000.0, 2500.0, -1.5, -0.0, 0.25], dtype=dtype)
    idx = torch.randint(0, len(specials), (B, 1, H, W), generator=g)
    d = torch.where(pick < 0.25, specials[idx], d)
    d[:, :, 3, 10:30] = d[:, :, 3, 10:11]  # a run of equal depths: many sources tie on few targets
    obj, flow = _unfused(rgb, d, s, ex)
    dev = torch.device("cuda:0")
    got = warp_disparity(torch.cat((rgb, ex), 1).to(dev), d.to(dev), s)
    exp_gpu = forward_warp_flow(obj.to(dev), flow.to(dev), d.to(dev).to(torch.float32))
    exp_cpu = oracle.fw_flow(obj.numpy(), flow.numpy(), d.to(torch.float32).numpy())
    for g_, e_, c_, n in zip(got, exp_gpu, exp_cpu, ("output", "valid", "collision")):
        g_ = g_.cpu().numpy()
        assert np.array_equal(g_, e_.cpu().numpy(), equal_nan=True), n
        assert np.array_equal(g_, c_, equal_nan=True), n


@pytest.mark.gpu
@pytest.mark.parametrize("W", [8192, 8190, 8193, 8196])
def test_disparity_row_kernel_width_limit(W):
    """The row kernel serves rows up to kRowMaxW = 8192 (64 KB of LDS keys per
    workgroup); wider rows fall back to the TILE engine.  Both sides of the
    limit, with and without 16-byte vector rows (W % 4), bit-exact against the
    TILE engine on the same call."""
    from opticalflowfromdepth_amd import _native, warp_disparity
    lib = _native.lib()
    rgb, d, s, ex = _inputs(2, 3, W, torch.float32, 900 + W, extra=1)
    dev = torch.device("cuda:0")
    args = (torch.cat((rgb, ex), 1).to(dev), d.to(dev), s)
    prev = lib.ofd_fw_set_disparity_rows(1)
    try:
        rows = warp_disparity(*args)
        lib.ofd_fw_set_disparity_rows(0)
        tile = warp_disparity(*args)
    finally:
        lib.ofd_fw_set_disparity_rows(prev)
    for x, y in zip(rows, tile):
        assert torch.equal(x, y)
    obj, flow = _unfused(rgb, d, s, ex)
    exp = oracle.fw_flow(obj.numpy(), flow.numpy(), d.to(torch.float32).numpy())
    for g, e in zip(rows, exp):
        assert np.array_equal(g.cpu().numpy(), e)
