"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact output / valid / collision (the z-buffer winner is an index,
and output values are copies of obj values).  Every case here runs the native
library -- there is no fallback that could make these pass without it.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import golden_cases, load_golden
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


# ------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", ["ties_c1", "ties_c2", "ties_c4", "ties_c6", "ties_c7", "coll_c6",
                                  "negzero_c3", "hotspot_c6", "nonint_c2", "ties_f64_c4",
                                  "ragged_1x1", "ragged_1xw", "ragged_hx1"])
def test_forward_warping_golden(cuda_device, name):
    import fw_cuda
    c = golden_cases(load_golden("fw_op.npz"))[name]
    got = fw_cuda.forward_warping(_t(c["obj"], cuda_device), _t(c["safe_y"], cuda_device),
                                  _t(c["safe_x"], cuda_device), _t(c["depth"], cuda_device))
    _assert_same(got, (c["output"], c["valid"], c["collision"]), name)


@pytest.mark.parametrize("name", ["f32_c6", "f32_c2_big", "f64flow_c6", "f64obj_c4", "nearint_f64"])
def test_FW_golden_from_reference_wrapper(cuda_device, name):
    """Goldens produced by the reference alt_cuda/fw.py itself (3-D inputs)."""
    from alt_cuda.fw import FW
    c = golden_cases(load_golden("fw_wrapper.npz"))[name]
    fw = FW(cuda_device)
    got = fw(_t(c["obj"], cuda_device), _t(c["flow"], cuda_device), _t(c["depth"], cuda_device))
    assert all(g.dtype == torch.float32 and g.device.type == "cuda" for g in got)
    _assert_same(got, (c["output"], c["valid"], c["collision"]), name)


def test_FW_golden_pipeline(cuda_device):
    from opticalflowfromdepth_amd import FW
    p = load_golden("pipeline.npz")
    fw = FW(cuda_device)
    for k in ("img0", "img1"):
        d = _t(p[f"{k}/norm_depth"], cuda_device)                  # float64, as preprocess
        f01 = _t(p[f"{k}/flow01"], cuda_device)
        obj = torch.cat((_t(p[f"{k}/rgb"], cuda_device), d.float(), -f01.float()), 0)
        got = fw(obj, f01, d)
        _assert_same(got, (p[f"{k}/fw01_output"], p[f"{k}/fw01_valid"], p[f"{k}/fw01_collision"]), k + "/01")
        d32 = d.float()
        f03 = _t(p[f"{k}/flow03"], cuda_device)
        obj3 = torch.cat((_t(p[f"{k}/rgb"], cuda_device), d32, -f03), 0)
        got3 = fw(obj3, f03, d32)
        _assert_same(got3, (p[f"{k}/fw03_output"], p[f"{k}/fw03_valid"], p[f"{k}/fw03_collision"]), k + "/03")


# ------------------------------------------------------------------ seeded random vs oracle
@pytest.mark.parametrize("seed", range(12))
def test_forward_warp_flow_random_vs_oracle(cuda_device, seed):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(seed)
    B, C = int(rng.integers(1, 5)), int(rng.choice([1, 2, 4, 6, 7]))
    H, W = int(rng.integers(1, 90)), int(rng.integers(1, 120))
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = (rng.standard_normal((B, 2, H, W)) * rng.uniform(0.1, 80)).astype(
        np.float64 if seed % 3 == 0 else np.float32)
    depth = (rng.integers(0, 6, (B, 1, H, W)) * rng.choice([1.0, 0.5, 300.0])).astype(np.float32)
    depth[rng.random(depth.shape) < 0.02] = np.nan
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    _assert_same(got, oracle.fw_flow(obj, flow, depth), f"seed{seed}")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_forward_warping_random_vs_oracle(cuda_device, dtype):
    import fw_cuda
    rng = np.random.default_rng(42)
    for trial in range(6):
        B, C, H, W = 3, int(rng.integers(1, 8)), int(rng.integers(2, 70)), int(rng.integers(2, 70))
        obj = rng.standard_normal((B, C, H, W)).astype(dtype)
        flow = (rng.standard_normal((B, 2, H, W)) * 10).astype(np.float32)
        sy, sx = oracle.safe_coords(flow)
        depth = rng.integers(-2, 4, (B, 1, H, W)).astype(dtype)
        depth[rng.random(depth.shape) < 0.1] = 2000
        sy, sx = sy.astype(dtype), sx.astype(dtype)
        got = fw_cuda.forward_warping(*(_t(a, cuda_device) for a in (obj, sy, sx, depth)))
        assert got[0].dtype == (torch.float64 if dtype == np.float64 else torch.float32)
        _assert_same(got, oracle.forward_warping(obj, sy, sx, depth), f"trial{trial}")


# ------------------------------------------------------------------ edge cases
def test_hot_spot_all_sources_to_one_pixel(cuda_device):
    from opticalflowfromdepth_amd import forward_warp_flow
    B, C, H, W = 2, 6, 64, 96
    rng = np.random.default_rng(3)
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = np.full((B, 2, H, W), 1e6, np.float32)     # everything clamps to (H-1, W-1)
    depth = rng.integers(1, 3, (B, 1, H, W)).astype(np.float32)
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    exp = oracle.fw_flow(obj, flow, depth)
    _assert_same(got, exp, "hotspot")
    assert exp[1].sum() == B


def test_empty_and_degenerate(cuda_device):
    from opticalflowfromdepth_amd import forward_warp_flow
    for (B, C, H, W) in [(0, 6, 8, 8), (2, 6, 0, 8), (2, 0, 5, 7), (1, 1, 1, 1)]:
        obj = torch.randn(B, C, H, W, device=cuda_device)
        flow = torch.randn(B, 2, H, W, device=cuda_device)
        depth = torch.rand(B, 1, H, W, device=cuda_device)
        got = forward_warp_flow(obj, flow, depth)
        exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy())
        _assert_same(got, exp, f"{(B, C, H, W)}")


def test_nan_and_inf_flow(cuda_device):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(11)
    B, C, H, W = 1, 3, 16, 20
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = rng.standard_normal((B, 2, H, W)).astype(np.float32)
    flow[0, 0, 0, :5] = np.nan
    flow[0, 1, 3, :4] = np.inf
    flow[0, 0, 5, :4] = -np.inf
    depth = np.ones((B, 1, H, W), np.float32)
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    _assert_same(got, oracle.fw_flow(obj, flow, depth), "naninf")


def test_repeatable_and_workspace_reuse(cuda_device):
    """Repeated calls, and calls of every entry point / engine interleaved on
    the one cached workspace, stay bit-exact (the workspace invariants hold
    whichever path ran last)."""
    import fw_cuda
    from opticalflowfromdepth_amd import _native, forward_warp_flow, synth
    lib = _native.lib()
    obj, flow, depth = synth.stage_one_batch(list(range(4)), 96, 128, cuda_device)
    exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy())
    a = forward_warp_flow(obj, flow, depth)
    b = forward_warp_flow(obj, flow, depth)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    _assert_same(a, exp, "tile")
    rng = np.random.default_rng(9)
    o64 = rng.standard_normal((3, 2, 40, 52))
    sy, sx = oracle.safe_coords((rng.standard_normal((3, 2, 40, 52)) * 6).astype(np.float32))
    d64 = rng.integers(1, 4, (3, 1, 40, 52)).astype(np.float64)
    exp64 = oracle.forward_warping(o64, sy.astype(np.float64), sx.astype(np.float64), d64)
    prev = lib.ofd_fw_set_engine(0)
    try:
        for engine in (0, 1, 2, 0, 2, 1):
            lib.ofd_fw_set_engine(engine)
            got64 = fw_cuda.forward_warping(*(_t(x, cuda_device) for x in
                                              (o64, sy.astype(np.float64), sx.astype(np.float64), d64)))
            _assert_same(got64, exp64, f"f64 after engine {engine}")
            _assert_same(forward_warp_flow(obj, flow, depth), exp, f"engine {engine}")
    finally:
        lib.ofd_fw_set_engine(prev)


def test_non_default_stream(cuda_device):
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    obj, flow, depth = synth.stage_one_batch(list(range(3)), 64, 80, cuda_device)
    ref = forward_warp_flow(obj, flow, depth)
    s = torch.cuda.Stream(cuda_device)
    s.wait_stream(torch.cuda.current_stream(cuda_device))
    with torch.cuda.stream(s):
        got = forward_warp_flow(obj, flow, depth)
    torch.cuda.current_stream(cuda_device).wait_stream(s)
    for x, y in zip(ref, got):
        assert torch.equal(x, y)


def test_chunked_workspace_via_c_abi(cuda_device):
    """Small workspaces force several chunks; results must not change."""
    from opticalflowfromdepth_amd import _native, synth
    lib = _native.lib()
    B, H, W = 7, 48, 64
    obj, flow, depth = synth.stage_one_batch(list(range(B)), H, W, cuda_device)
    exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy())
    stream = torch.cuda.current_stream(cuda_device).cuda_stream
    one = lib.ofd_fw_workspace_bytes(1, H, W, 0)
    for images_per_chunk in (1, 2, 3, 7):
        nbytes = images_per_chunk * one
        ws = torch.empty(nbytes, dtype=torch.uint8, device=cuda_device)
        assert lib.ofd_fw_workspace_init(ws.data_ptr(), nbytes, stream) == 0
        out = torch.empty_like(obj)
        valid = torch.empty_like(depth)
        coll = torch.empty_like(depth)
        rc = lib.ofd_fw_forward_warp_flow_f32(obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(),
                                              valid.data_ptr(), coll.data_ptr(), B, obj.shape[1], H, W,
                                              ws.data_ptr(), nbytes, stream)
        assert rc == 0
        _assert_same((out, valid, coll), exp, f"chunk{images_per_chunk}")
    # a workspace smaller than one image is refused, not overrun
    ws = torch.empty(16, dtype=torch.uint8, device=cuda_device)
    rc = lib.ofd_fw_forward_warp_flow_f32(obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(),
                                          valid.data_ptr(), coll.data_ptr(), B, obj.shape[1], H, W,
                                          ws.data_ptr(), 16, stream)
    assert rc == -3


def test_vector_and_scalar_paths_agree(cuda_device):
    """H*W % 4 != 0 takes the scalar kernels; same answer as the oracle."""
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(5)
    for (H, W) in [(37, 41), (8, 8), (3, 5)]:
        obj = rng.standard_normal((2, 4, H, W)).astype(np.float32)
        flow = (rng.standard_normal((2, 2, H, W)) * 5).astype(np.float32)
        depth = rng.integers(1, 4, (2, 1, H, W)).astype(np.float32)
        got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
        _assert_same(got, oracle.fw_flow(obj, flow, depth), f"{H}x{W}")


def test_misaligned_views_take_scalar_path(cuda_device):
    """A storage offset that breaks 16-byte alignment must still be correct."""
    import fw_cuda
    rng = np.random.default_rng(8)
    B, C, H, W = 1, 2, 16, 16
    n = B * H * W
    big = torch.from_numpy(rng.standard_normal(5 * n + 1).astype(np.float32)).to(cuda_device)
    obj = big[1:1 + 2 * n].view(B, C, H, W)
    flow = (rng.standard_normal((B, 2, H, W)) * 3).astype(np.float32)
    sy, sx = oracle.safe_coords(flow)
    sy_t = big[1 + 2 * n:1 + 3 * n].view(B, 1, H, W).copy_(_t(sy, cuda_device))
    sx_t = big[1 + 3 * n:1 + 4 * n].view(B, 1, H, W).copy_(_t(sx, cuda_device))
    depth = big[1 + 4 * n:1 + 5 * n].view(B, 1, H, W).abs_()
    got = fw_cuda.forward_warping(obj, sy_t, sx_t, depth)
    exp = oracle.forward_warping(obj.cpu().numpy(), sy, sx, depth.cpu().numpy())
    _assert_same(got, exp, "misaligned")


# ------------------------------------------------------------------ headline size
def test_headline_768x1024_b64_vs_oracle(cuda_device):
    """BASELINE config 3 shape: 64 x 6 x 768 x 1024, half disparity / half
    ego-motion flows; every image checked bit-exactly against the oracle."""
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    B, H, W = 64, 768, 1024
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, cuda_device)
    got = forward_warp_flow(obj, flow, depth)
    exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy(), nthreads=16)
    _assert_same(got, exp, "768x1024x64")
    v = got[1].cpu()
    # size-independent properties: masks binary, collision == 0 for real depths
    assert torch.all((v == 0) | (v == 1)) and float(got[2].sum()) == 0


def test_FW_3d_matches_batched(cuda_device):
    from opticalflowfromdepth_amd import FW, synth
    obj, flow, depth = synth.stage_one_batch([1, 2], 40, 56, cuda_device)
    fw = FW(cuda_device)
    ob, vb, cb = fw(obj, flow, depth)
    for i in range(2):
        o, v, c = fw(obj[i], flow[i], depth[i])
        assert o.shape == (6, 40, 56) and v.shape == (1, 40, 56) and c.shape == (1, 40, 56)
        assert torch.equal(o, ob[i]) and torch.equal(v, vb[i]) and torch.equal(c, cb[i])


def test_forward_warp_autograd_function(cuda_device):
    """alt_cuda.fw.forward_warp (the autograd.Function form) == FW; no backward."""
    import alt_cuda.fw as afw
    from opticalflowfromdepth_amd import synth
    obj, flow, depth = synth.stage_one_batch([3, 4], 40, 56, cuda_device)
    a = afw.FW()(obj, flow, depth)
    b = afw.forward_warp(obj, flow, depth)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    o, v, c = afw.forward_warp(obj.clone().requires_grad_(True), flow, depth)
    assert o.requires_grad and not v.requires_grad and not c.requires_grad
    with pytest.raises(NotImplementedError):
        o.sum().backward()


def test_fused_out_validation(cuda_device):
    from opticalflowfromdepth_amd import synth, warp_disparity
    seeds = [1, 2]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, 32, 48, cuda_device))
    rgb = synth.synthetic_rgb(seeds, 32, 48, cuda_device)
    s = torch.ones(2)
    good = (torch.empty(2, 6, 32, 48, device=cuda_device), torch.empty(2, 1, 32, 48, device=cuda_device),
            torch.empty(2, 1, 32, 48, device=cuda_device))
    warp_disparity(rgb, depth, s, out=good)
    with pytest.raises(RuntimeError, match="out output"):
        warp_disparity(rgb, depth, s, out=(good[0][:, :5].contiguous(), good[1], good[2]))
    with pytest.raises(RuntimeError, match="out valid"):
        warp_disparity(rgb, depth, s, out=(good[0], good[1].double(), good[2]))


# ------------------------------------------------------------------ every engine
# 0 = TILE (fused SPLAT gathers the output), 1 = ATOMIC, 2 = TILE_SPLIT (winner map + RESOLVE)
@pytest.fixture(params=[1, 2], ids=["atomic", "split"])
def other_engine(request):
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_fw_set_engine(request.param)
    yield request.param
    lib.ofd_fw_set_engine(prev)


@pytest.mark.parametrize("seed", range(4))
def test_other_engines_random_vs_oracle(cuda_device, other_engine, seed):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(100 + seed)
    B, C, H, W = 3, int(rng.choice([2, 6, 7])), int(rng.integers(5, 90)), int(rng.integers(5, 120))
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = (rng.standard_normal((B, 2, H, W)) * rng.uniform(0.1, 60)).astype(np.float32)
    depth = rng.integers(0, 4, (B, 1, H, W)).astype(np.float32)
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    _assert_same(got, oracle.fw_flow(obj, flow, depth), f"engine {other_engine} seed{seed}")


def test_engines_agree_on_realistic_batch(cuda_device):
    from opticalflowfromdepth_amd import _native, forward_warp_flow, synth
    lib = _native.lib()
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(8)], 384, 512, cuda_device)
    prev = lib.ofd_fw_set_engine(0)
    try:
        a = forward_warp_flow(obj, flow, depth)
        for engine in (1, 2):
            lib.ofd_fw_set_engine(engine)
            b = forward_warp_flow(obj, flow, depth)
            for x, y in zip(a, b):
                assert torch.equal(x, y), engine
    finally:
        lib.ofd_fw_set_engine(prev)


def test_tile_engine_overflow_and_wide_boxes(cuda_device):
    """Border hot spots overflow tile lists; random flows give boxes wider than
    the tile budget.  Both spill to the key slab and must stay bit-exact."""
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(21)
    B, C, H, W = 2, 6, 256, 384
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = np.zeros((B, 2, H, W), np.float32)
    flow[0, 0] = 5000.0                                       # every source -> column W-1 (overflow)
    flow[0, 1] = (rng.standard_normal((H, W)) * 3).astype(np.float32)
    flow[1] = (rng.standard_normal((2, H, W)) * 150).astype(np.float32)   # non-smooth
    depth = rng.integers(1, 5, (B, 1, H, W)).astype(np.float32)
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    _assert_same(got, oracle.fw_flow(obj, flow, depth), "overflow")


# ------------------------------------------------------------------ packed targets (BIN -> SPLAT)
@pytest.fixture
def unpacked():
    """The TILE engine with SPLAT re-reading the coordinate planes instead of
    BIN's 16-bit packed targets (ofd_fw_set_pack(0)): the round-4 path, kept
    as a cross-check of the default."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_fw_set_pack(0)
    yield
    lib.ofd_fw_set_pack(prev)


@pytest.mark.parametrize("seed", range(6))
def test_unpacked_targets_random_vs_oracle(cuda_device, unpacked, seed):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(700 + seed)
    B, C = int(rng.integers(1, 4)), int(rng.choice([1, 2, 6, 7]))
    H, W = int(rng.integers(1, 90)), int(rng.integers(1, 120))
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = (rng.standard_normal((B, 2, H, W)) * rng.uniform(0.1, 80)).astype(
        np.float64 if seed % 2 else np.float32)
    depth = (rng.integers(0, 6, (B, 1, H, W)) * 0.5).astype(np.float32)
    depth[rng.random(depth.shape) < 0.02] = np.nan
    got = forward_warp_flow(_t(obj, cuda_device), _t(flow, cuda_device), _t(depth, cuda_device))
    _assert_same(got, oracle.fw_flow(obj, flow, depth), f"unpacked seed{seed}")


def test_packed_and_unpacked_targets_agree(cuda_device):
    """Every coordinate source that packs (FW on float32 / float64 flows, the
    op's safe coordinates, warp_flow_cat) gives the same bits with and without
    packed targets, on the persistent SPLAT (headline-like batch) and the
    one-workgroup-per-tile SPLAT, on rows with and without 16-byte alignment,
    with clamped border hot spots and wide (spilled) blocks."""
    import fw_cuda
    from opticalflowfromdepth_amd import _native, forward_warp_flow, synth, warp_flow_cat
    lib = _native.lib()
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(24)], 384, 512, cuda_device)
    rng = np.random.default_rng(5)
    wild = flow[:2].clone()
    wild[0, 0] += 4000.0                                                       # hot spot on column W-1
    wild[1] += torch.from_numpy((rng.standard_normal((2, 384, 512)) * 120).astype(np.float32)).to(cuda_device)
    odd = synth.stage_one_batch([999, 1000], 93, 157, cuda_device)             # W % 4 != 0: scalar path
    sy = flow[:3, 1:2].clone()
    sx = flow[:3, 0:1].clone()
    ii = torch.arange(512, device=cuda_device, dtype=torch.float32)
    jj = torch.arange(384, device=cuda_device, dtype=torch.float32)[:, None]
    sx = (sx + ii).clamp(0, 511).trunc()
    sy = (sy + jj).clamp(0, 383).trunc()
    calls = [
        lambda: forward_warp_flow(obj, flow, depth),
        lambda: forward_warp_flow(obj, flow.double(), depth),
        lambda: forward_warp_flow(obj[:2], wild, depth[:2]),
        lambda: forward_warp_flow(*odd),
        lambda: fw_cuda.forward_warping(obj[:3].contiguous(), sy.contiguous(), sx.contiguous(),
                                        depth[:3].contiguous()),
        lambda: warp_flow_cat(obj[:, 0:3].contiguous(), flow, depth.double()),
    ]
    prev = lib.ofd_fw_set_pack(-1)
    prev_pm = lib.ofd_fw_set_persist_min(-1)
    try:
        for persist_min in (prev_pm, 0, 1000):   # default split, always persistent, always one per tile
            lib.ofd_fw_set_persist_min(persist_min)
            for k, call in enumerate(calls):
                lib.ofd_fw_set_pack(1)
                a = call()
                lib.ofd_fw_set_pack(0)
                b = call()
                for x, y in zip(a, b):
                    assert torch.equal(x, y), (persist_min, k)
    finally:
        lib.ofd_fw_set_pack(prev)
        lib.ofd_fw_set_persist_min(prev_pm)
