"""BASELINE.json configs 1 and 2.

config 1 -- one 480x640 synthetic depth map through the CPU plumbing: the
  synth restatements of normalize_depth (utils.py:102-116), the disparity flow
  (preprocess.py:239-254) and the ego-motion flow (preprocess.py:265-298 with
  geometry.py:17-67) on torch-CPU, then the warp of preprocess.py:358-359 /
  :386-387 by the C oracle and by the torch-CPU scatter-min restatement, all
  checked bit for bit against tests/golden/config1.npz, which the reference's
  own utils.py / preprocess.py slice / geometry.py / fw.py produced
  (tests/golden/make_golden.py config1).
config 2 -- 480x640, B=32, C=6 fp32 on one GPU (images 0-15 disparity flow,
  16-31 ego-motion flow, seeds 12345+i): every image of the HIP warp
  bit-exact vs the oracle.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import load_golden


def _digest(a) -> str:
    a = np.ascontiguousarray(a)
    return f"{a.dtype.str}{tuple(a.shape)}:" + hashlib.sha256(a.tobytes()).hexdigest()


def _check(z, name, a):
    a = np.ascontiguousarray(a)
    if _digest(a) != str(z[f"digest/{name}"]):
        s = a.reshape(-1)[::97]
        ref = z[f"sample/{name}"]
        diff = np.abs(s.astype(np.float64) - ref.astype(np.float64)) if s.shape == ref.shape else None
        raise AssertionError(f"{name}: digest differs from the reference's "
                             f"(strided sample max |diff| = {None if diff is None else diff.max()})")


def test_config1_cpu_plumbing():
    from oracle import oracle, torch_cpu
    from opticalflowfromdepth_amd import synth
    z = load_golden("config1.npz")
    h, w = 480, 640
    raw = synth.synthetic_depth_np(h, w, 0)
    rgb = np.floor(np.random.default_rng(1000).uniform(0, 256, (3, h, w))).astype(np.float32)
    _check(z, "raw_depth", raw)
    _check(z, "rgb", rgb)
    # utils.set_seed(12345), then the first stage's draws: s (preprocess.py:240), T1 (:277)
    s, T = synth.camera_params(12345)
    assert np.array_equal(T.numpy(), z["T1"][0])
    d0 = synth.normalize_depth(torch.from_numpy(raw.copy()).view(1, 1, h, w))     # float64 like get_depth
    _check(z, "norm_depth", d0[0].numpy())
    flow01 = synth.disparity_flow(d0, s.view(1))                                   # float64 flow
    _check(z, "flow01", flow01[0].numpy())
    d0f = d0.to(torch.float32)
    flow03 = synth.ego_motion_flow(d0f, T.view(1, 4, 4))
    # geometry.py's two matmuls go through the host's CPU BLAS, whose rounding
    # differs between hosts (the fixture was made on an Intel build host; an
    # AMD host differs by ~1e-4 px even for the reference's own code): bits on
    # the fixture's host, else within 1e-3 px and the warps checked for
    # self-consistency on this host's flow
    same_host = _digest(flow03[0].numpy()) == str(z["digest/flow03"])
    if not same_host:
        diff = np.abs(flow03[0].numpy().reshape(-1)[::97] - z["sample/flow03"]).max()
        assert diff < 1e-3, diff
    rgb_t = torch.from_numpy(rgb).unsqueeze(0)
    for tag, obj, flow, depth in (("fw01", torch.cat((rgb_t, d0, flow01 * -1.0), 1), flow01, d0),
                                  ("fw03", torch.cat((rgb_t, d0f, flow03 * -1.0), 1), flow03, d0f)):
        o, v, c = oracle.fw_flow(obj.numpy(), flow.numpy(), depth.numpy())
        pinned = tag == "fw01" or same_host
        if pinned:
            for n, a in (("output", o), ("valid", v), ("collision", c)):
                _check(z, f"{tag}_{n}", a[0])
        # the torch-CPU formulation (bench.py's CPU baseline leg) gives the same bits
        for n, a, e in zip(("output", "valid", "collision"), torch_cpu.fw_flow_scatter(obj, flow, depth), (o, v, c)):
            assert np.array_equal(a.numpy(), e), (tag, n)


@pytest.mark.gpu
@pytest.mark.parametrize("short_tiles", [1, 0], ids=["tiles128x16", "tiles128x32"])
def test_config2_every_image_bit_exact(cuda_device, short_tiles):
    """Config 2 is a short call (4.7 tiles per resident SPLAT slot): by default
    on 128 x 16 target tiles (ofd_fw_set_short_tiles), else 128 x 32 -- the
    oracle's bits either way."""
    from oracle import oracle
    from opticalflowfromdepth_amd import _native, forward_warp_flow, synth
    B, H, W = 32, 480, 640
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, cuda_device)
    assert obj.shape == (B, 6, H, W)
    lib = _native.lib()
    prev = lib.ofd_fw_set_short_tiles(short_tiles)
    try:
        out = forward_warp_flow(obj, flow, depth)
        torch.cuda.synchronize()
    finally:
        lib.ofd_fw_set_short_tiles(prev)
    exp = oracle.fw_flow(obj.cpu().numpy(), flow.cpu().numpy(), depth.cpu().numpy())
    for g, e, n in zip(out, exp, ("output", "valid", "collision")):
        g = g.cpu().numpy()
        bad = [i for i in range(B) if not np.array_equal(g[i], e[i])]
        assert not bad, f"{n} differs from the oracle on images {bad}"
    # ego-motion half really clamps to the border (the config's stress case)
    assert float(out[1][16:].mean()) < float(out[1][:16].mean())
