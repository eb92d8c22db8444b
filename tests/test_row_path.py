"""GPU parity tests of the TILE engine's row path (csrc/ofd_fw.hip row_item).

BIN checks per image and per call whether every source lands in its own row
(true of every disparity flow, preprocess.py:249-254); such images are
splatted row by row instead of through the tile lists.  The bar is the one of
tests/test_fw_gpu.py: bit-exact output / valid / collision against the oracle
(the serial loop of fw_cuda_kernel.cu:28-47), and equal to the same call with
the row path off.  Cases: ties and border hot spots inside rows, NaN / >= 1000 /
-0 depths, one off-row source or one NaN y flow in an otherwise row-local image
(the image must leave the row path), mixed batches, every width class (sub-band
splits, W = 4096 with one row per sub-band, W > 4096 where the path is off),
the safe-coordinate op, float64 and bf16 flows, chunked workspaces and calls
that alternate row-local and general images on one workspace.
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _assert_same(got, exp, what=""):
    for g, e, n in zip(got, exp, ("output", "valid", "collision")):
        g = g.detach().cpu().numpy()
        assert g.shape == e.shape, (what, n, g.shape, e.shape)
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)
            raise AssertionError(f"{what} {n}: {len(bad)} mismatches, first at {bad[:3].tolist()}")


@pytest.fixture
def lib():
    from opticalflowfromdepth_amd import _native
    return _native.lib()


def _both(lib, fn):
    """fn() with the row path on, then off; returns both results."""
    prev = lib.ofd_fw_set_row_path(1)
    try:
        on = fn()
        lib.ofd_fw_set_row_path(0)
        off = fn()
    finally:
        lib.ofd_fw_set_row_path(prev)
    return on, off


def _row_flow(rng, B, H, W, scale=30.0, dtype=np.float32):
    """Row-local flows: x anywhere (border clamps included), y = +-0."""
    flow = np.zeros((B, 2, H, W), dtype)
    flow[:, 0] = (rng.standard_normal((B, H, W)) * scale).astype(dtype)
    flow[:, 1] = np.where(rng.random((B, H, W)) < 0.5, 0.0, -0.0).astype(dtype)
    return flow


def _depth(rng, B, H, W):
    d = rng.integers(0, 5, (B, 1, H, W)).astype(np.float32)   # heavy ties
    d[rng.random(d.shape) < 0.02] = np.nan
    d[rng.random(d.shape) < 0.02] = 2000.0                     # collision path
    d[rng.random(d.shape) < 0.02] = -0.0
    return d


@pytest.mark.parametrize("H,W", [(96, 128), (480, 640), (37, 64), (8, 4096), (5, 4100), (64, 8), (1, 4)])
def test_row_local_vs_oracle(cuda_device, lib, H, W):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(H * 7919 + W)
    B, C = 3, 6
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = _row_flow(rng, B, H, W)
    flow[0, 0, :, : W // 3] = 1e6                              # a border hot spot in every row
    depth = _depth(rng, B, H, W)
    args = [_t(a, cuda_device) for a in (obj, flow, depth)]
    on, off = _both(lib, lambda: forward_warp_flow(*args))
    exp = oracle.fw_flow(obj, flow, depth)
    _assert_same(on, exp, f"row path {H}x{W}")
    _assert_same(off, exp, f"tile path {H}x{W}")


def test_one_off_row_source_leaves_the_row_path(cuda_device, lib):
    """A single source that leaves its row (or a NaN y flow) must send its
    image to the tile path; its row-local neighbours in the batch keep the
    row path.  Every image bit-exact."""
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(77)
    B, C, H, W = 4, 4, 64, 96
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = _row_flow(rng, B, H, W, scale=10.0)
    flow[1, 1, 40, 17] = 1.0            # lands one row down
    flow[2, 1, 0, 0] = np.nan           # dropped source
    flow[3, 1, 63, 95] = -70.0          # lands 70 rows up (clamped to 0)
    depth = rng.integers(1, 4, (B, 1, H, W)).astype(np.float32)
    depth[1, 0, 40, 17] = 0.5           # ... and wins where it lands
    args = [_t(a, cuda_device) for a in (obj, flow, depth)]
    on, off = _both(lib, lambda: forward_warp_flow(*args))
    exp = oracle.fw_flow(obj, flow, depth)
    _assert_same(on, exp, "row path")
    _assert_same(off, exp, "tile path")


def test_safe_coordinate_op_row_local(cuda_device, lib):
    import fw_cuda
    rng = np.random.default_rng(5)
    B, C, H, W = 2, 7, 48, 64
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    sy, sx = oracle.safe_coords(_row_flow(rng, B, H, W))
    sx = sx + rng.random(sx.shape).astype(np.float32) * 0.9   # non-integer x, same truncation row
    sx = np.minimum(sx, W - 1).astype(np.float32)
    depth = _depth(rng, B, H, W)
    args = [_t(a, cuda_device) for a in (obj, sy, sx, depth)]
    on, off = _both(lib, lambda: fw_cuda.forward_warping(*args))
    exp = oracle.forward_warping(obj, sy, sx, depth)
    _assert_same(on, exp, "row path")
    _assert_same(off, exp, "tile path")


def test_float64_flow_row_local(cuda_device, lib):
    """fw.py:31 adds a float64 flow in float64; the row path's x target must
    truncate the same float64 sum (near-integer flows flip otherwise)."""
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(6)
    B, C, H, W = 2, 3, 32, 64
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = _row_flow(rng, B, H, W, dtype=np.float64)
    flow[:, 0] = np.round(flow[:, 0]) - 1e-9                  # float32 rounding would move these
    depth = _depth(rng, B, H, W)
    args = [_t(a, cuda_device) for a in (obj, flow, depth)]
    on, off = _both(lib, lambda: forward_warp_flow(*args))
    exp = oracle.fw_flow(obj, flow, depth)
    _assert_same(on, exp, "row path")
    _assert_same(off, exp, "tile path")


def test_bf16_row_local_equals_f32(cuda_device, lib):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(8)
    B, C, H, W = 3, 6, 92, 140
    objf = torch.from_numpy(rng.standard_normal((B, C, H, W)).astype(np.float32)).to(cuda_device)
    objb = objf.to(torch.bfloat16)
    flow = _t(_row_flow(rng, B, H, W), cuda_device)
    depth = _t(_depth(rng, B, H, W), cuda_device)
    on, off = _both(lib, lambda: forward_warp_flow(objb, flow, depth))
    ref = forward_warp_flow(objb.float(), flow, depth)
    for x, y in zip(on, off):
        assert torch.equal(x.view(torch.int16) if x.dtype == torch.bfloat16 else x,
                           y.view(torch.int16) if y.dtype == torch.bfloat16 else y)
    assert torch.equal(on[0].view(torch.int16), ref[0].to(torch.bfloat16).view(torch.int16))
    assert torch.equal(on[1], ref[1]) and torch.equal(on[2], ref[2])


def test_alternating_calls_and_chunks_on_one_workspace(cuda_device, lib):
    """Row-local and general batches alternate on the cached workspace, and a
    small workspace splits a mixed batch into chunks: the per-chunk epochs
    must never let a stale 'row-local' verdict through."""
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    B, H, W = 6, 64, 96
    obj, flow_real, depth = synth.stage_one_batch([300 + i for i in range(B)], H, W, cuda_device,
                                                  ego_fraction=0.5)
    rng = np.random.default_rng(12)
    flow_row = _t(_row_flow(rng, B, H, W), cuda_device)
    cases = [flow_row, flow_real, flow_row, flow_row.flip(0).contiguous(), flow_real]
    exps = [oracle.fw_flow(obj.cpu().numpy(), f.cpu().numpy(), depth.cpu().numpy()) for f in cases]
    for k, (f, e) in enumerate(zip(cases, exps)):
        _assert_same(forward_warp_flow(obj, f, depth), e, f"call {k}")
    stream = torch.cuda.current_stream(cuda_device).cuda_stream
    one = lib.ofd_fw_workspace_bytes(1, H, W, 0)
    for per_chunk in (1, 2, 4):
        nbytes = per_chunk * one
        ws = torch.empty(nbytes, dtype=torch.uint8, device=cuda_device)
        assert lib.ofd_fw_workspace_init(ws.data_ptr(), nbytes, stream) == 0
        for k, (f, e) in enumerate(zip(cases, exps)):
            out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
            rc = lib.ofd_fw_forward_warp_flow_f32(obj.data_ptr(), f.data_ptr(), depth.data_ptr(), out.data_ptr(),
                                                  valid.data_ptr(), coll.data_ptr(), B, obj.shape[1], H, W,
                                                  ws.data_ptr(), nbytes, stream)
            assert rc == 0
            _assert_same((out, valid, coll), e, f"chunk {per_chunk} call {k}")


def test_headline_disparity_images_take_the_row_path(cuda_device, lib):
    """The headline batch's disparity half is row-local: with the row path on,
    the 768x1024 disparity images are bit-exact vs the oracle and equal to
    the tile path."""
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    B, H, W = 8, 768, 1024
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, cuda_device, ego_fraction=0.25)
    assert float(flow[:6, 1].abs().max()) == 0.0               # disparity images: y flow is -0
    on, off = _both(lib, lambda: forward_warp_flow(obj, flow, depth))
    for x, y in zip(on, off):
        assert torch.equal(x, y)
    _assert_same(on, oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy(), nthreads=16),
                 "768x1024")
