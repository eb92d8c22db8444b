"""GPU parity of the TILE engine's PIPE variant (csrc/ofd_fw.hip
splat_pipe_kernel): BIN runs inside the persistent SPLAT launch, images
handed from their BIN items to their tile items by an agent-scope release /
acquire.  Bar: bit-exact against the oracle (the serial loop of
fw_cuda_kernel.cu:28-47) and equal to the two-launch engine on every case --
random tie-heavy batches of every size class, wide boxes and key-slab spills
(BIN's atomics and tile flags crossing the hand-off), border hot spots, row-
local images (the row path's verdict crossing the hand-off), chunked
workspaces (several pipelined launches per call), the fused coordinate
sources (disparity, ego-motion, flow planes with generated channels), bf16,
and the full headline batch.
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _same(got, exp, what):
    for g, e, n in zip(got, exp, ("output", "valid", "collision")):
        g = g.detach().cpu().numpy() if isinstance(g, torch.Tensor) else g
        e = e.detach().cpu().numpy() if isinstance(e, torch.Tensor) else e
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)
            raise AssertionError(f"{what} {n}: {len(bad)} mismatches, first at {bad[:3].tolist()}")


@pytest.fixture
def lib():
    from opticalflowfromdepth_amd import _native
    l = _native.lib()
    prev = l.ofd_fw_set_pipe(-1)
    yield l
    l.ofd_fw_set_pipe(prev)


def _both(lib, fn):
    lib.ofd_fw_set_pipe(1)
    a = fn()
    torch.cuda.synchronize()
    lib.ofd_fw_set_pipe(0)
    b = fn()
    return a, b


@pytest.mark.parametrize("seed", range(8))
def test_pipe_random_vs_oracle(cuda_device, lib, seed):
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(500 + seed)
    B, C = int(rng.integers(1, 20)), int(rng.choice([1, 2, 4, 6, 7]))
    H, W = int(rng.integers(1, 200)), int(rng.integers(1, 300))
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = (rng.standard_normal((B, 2, H, W)) * rng.uniform(0.1, 120)).astype(np.float64 if seed % 3 == 0 else np.float32)
    if seed % 4 == 1:
        flow[:, 1] = 0.0                                   # row-local images (row path behind the hand-off)
    depth = (rng.integers(0, 6, (B, 1, H, W)) * rng.choice([1.0, 0.5, 300.0])).astype(np.float32)
    depth[rng.random(depth.shape) < 0.02] = np.nan
    args = [_t(a, cuda_device) for a in (obj, flow, depth)]
    a, b = _both(lib, lambda: forward_warp_flow(*args))
    exp = oracle.fw_flow(obj, flow, depth)
    _same(a, exp, f"pipe seed{seed}")
    _same(b, exp, f"two-launch seed{seed}")


def test_pipe_wide_boxes_hot_spots_and_mixed_rows(cuda_device, lib):
    """Non-smooth flows spill to the key slab through BIN's global atomics and
    tile flags; a border hot spot overflows the lists; row-local images sit
    between them.  All of it crosses the in-launch hand-off."""
    from opticalflowfromdepth_amd import forward_warp_flow
    rng = np.random.default_rng(21)
    B, C, H, W = 11, 6, 256, 384
    obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
    flow = np.zeros((B, 2, H, W), np.float32)
    flow[0::3] = (rng.standard_normal((len(range(0, B, 3)), 2, H, W)) * 150).astype(np.float32)  # non-smooth
    flow[1::3, 0] = 5000.0                                                                    # hot spot
    flow[1::3, 1] = (rng.standard_normal((len(range(1, B, 3)), H, W)) * 3).astype(np.float32)
    flow[2::3, 0] = (rng.standard_normal((len(range(2, B, 3)), H, W)) * 40).astype(np.float32)  # row-local
    depth = rng.integers(1, 5, (B, 1, H, W)).astype(np.float32)
    args = [_t(a, cuda_device) for a in (obj, flow, depth)]
    for rep in range(3):  # repeated launches: the restored queues / counters start clean
        a, b = _both(lib, lambda: forward_warp_flow(*args))
        exp = oracle.fw_flow(obj, flow, depth)
        _same(a, exp, f"pipe rep{rep}")
        _same(b, exp, f"two-launch rep{rep}")


def test_pipe_chunked_workspace(cuda_device, lib):
    from opticalflowfromdepth_amd import synth
    B, H, W = 19, 48, 64
    obj, flow, depth = synth.stage_one_batch(list(range(B)), H, W, cuda_device)
    exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy())
    stream = torch.cuda.current_stream(cuda_device).cuda_stream
    one = lib.ofd_fw_workspace_bytes(1, H, W, 0)
    lib.ofd_fw_set_pipe(1)
    for per_chunk in (1, 3, 8, 19):
        nbytes = per_chunk * one
        ws = torch.empty(nbytes, dtype=torch.uint8, device=cuda_device)
        assert lib.ofd_fw_workspace_init(ws.data_ptr(), nbytes, stream) == 0
        for rep in range(2):
            out, valid, coll = torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth)
            rc = lib.ofd_fw_forward_warp_flow_f32(obj.data_ptr(), flow.data_ptr(), depth.data_ptr(), out.data_ptr(),
                                                  valid.data_ptr(), coll.data_ptr(), B, obj.shape[1], H, W,
                                                  ws.data_ptr(), nbytes, stream)
            assert rc == 0
            _same((out, valid, coll), exp, f"chunk {per_chunk} rep {rep}")


def test_pipe_fused_sources(cuda_device, lib):
    """The coordinate sources that generate obj channels run on the same
    pipelined launch: the disparity warp (on the TILE engine), the ego-motion
    warp, and FW on a held flow plane (warp_flow_cat)."""
    from opticalflowfromdepth_amd import _native, ego_flow, synth, warp_disparity, warp_ego, warp_flow_cat
    B, H, W = 10, 96, 128
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, cuda_device, dtype=torch.float64))
    rgb = synth.synthetic_rgb(seeds, H, W, cuda_device)
    s, T = synth.batch_camera_params(seeds)
    P, ik = synth.projection(H, W, T.to(cuda_device), cuda_device)
    plane = ego_flow(depth, P, ik)
    prev_rows = lib.ofd_fw_set_disparity_rows(0)
    try:
        for name, fn in (("disparity", lambda: warp_disparity(rgb, depth, s)),
                         ("ego", lambda: warp_ego(rgb, depth, P, ik)),
                         ("flow_cat", lambda: warp_flow_cat(rgb, plane, depth))):
            a, b = _both(lib, fn)
            for x, y in zip(a, b):
                assert torch.equal(x, y), name
    finally:
        lib.ofd_fw_set_disparity_rows(prev_rows)


def test_pipe_bf16_and_safe_coordinates(cuda_device, lib):
    import fw_cuda
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    obj, flow, depth = synth.stage_one_batch([40 + i for i in range(12)], 92, 140, cuda_device)
    objb = obj.to(torch.bfloat16)
    a, b = _both(lib, lambda: forward_warp_flow(objb, flow, depth))
    for x, y in zip(a, b):
        assert torch.equal(x.view(torch.int16) if x.dtype == torch.bfloat16 else x,
                           y.view(torch.int16) if y.dtype == torch.bfloat16 else y)
    sy, sx = oracle.safe_coords(flow.cpu().numpy())
    args = (obj, _t(sy, cuda_device), _t(sx, cuda_device), depth)
    a, b = _both(lib, lambda: fw_cuda.forward_warping(*args))
    _same(a, b, "safe coordinates")


def test_pipe_headline_768x1024_b64_vs_oracle(cuda_device, lib):
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    B, H, W = 64, 768, 1024
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, cuda_device)
    lib.ofd_fw_set_pipe(1)
    got = forward_warp_flow(obj, flow, depth)
    _same(got, oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy(), nthreads=16), "768x1024x64")
