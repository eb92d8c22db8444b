"""Hole-fill (utils.inpaint, utils.py:136-151): oracle pinning on CPU, GPU parity.

* The keep-mask algebra, the uint8 cast and the float32 return are pinned by
  tests/golden/inpaint_mask.npz (the reference's own utils.inpaint run with a
  recording stand-in for cv2; see tests/golden/make_golden.py).
* The fill values: parity with cv2.inpaint(INPAINT_TELEA) is UNPINNED (OpenCV
  is absent).  oracle/inpaint_oracle.c restates cv2's sequential Telea
  ("seq") and the GPU's layered Telea ("layered"); the GPU must match the
  layered restatement bit for bit, and the two restatements must stay close on
  smooth images (the bound below is the documented divergence).
"""
import ctypes
import os
import time

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import oracle

GOLD = os.path.join(REPO, "tests", "golden", "inpaint_mask.npz")


def _mask_cases():
    g = np.load(GOLD)
    for n in range(int(g["n"])):
        yield n, g[f"c{n}/img"], g[f"c{n}/valid"], g[f"c{n}/collision"], g[f"c{n}/img_u8_hwc"], \
            g[f"c{n}/mask"], g[f"c{n}/returned"]


def smooth_image(h, w, seed, c=3):
    """Integer-valued smooth RGB: a ramp plus one slow wave per channel."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    img = np.zeros((c, h, w))
    for k in range(c):
        gx, gy, ph = rng.uniform(-1.5, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(0, 2 * np.pi)
        img[k] = 128 + gx * (xx - w / 2) + gy * (yy - h / 2) + 60 * np.sin(2 * np.pi * xx / w + ph) * np.cos(
            2 * np.pi * yy / h)
    return np.floor(np.clip(img, 0, 255)).astype(np.float32)


def blob_masks(h, w, seed, frac=0.15):
    """valid with blob holes (disocclusions) and a border strip, collision all zero."""
    rng = np.random.default_rng(seed)
    v = np.ones((h, w), np.float32)
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    while (v == 0).mean() < frac:
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(1, 6)
        v[(yy - cy) ** 2 + (xx - cx) ** 2 < r * r] = 0
    v[:, : max(1, w // 20)] = 0  # ego-motion border strip
    return v[None], np.zeros((1, h, w), np.float32)


# ---------------------------------------------------------------- CPU: oracle pinning
def test_oracle_mask_matches_reference_fixture():
    for n, img, v, c, img_u8, mask, _ in _mask_cases():
        hole = oracle.inpaint_mask(v[None], c[None])[0]
        assert np.array_equal(hole, (mask != 0).astype(np.uint8)), n


def test_oracle_keeps_known_pixels_and_casts_like_reference():
    """Kept pixels are the uint8 cast of the input (utils.py:148), returned as float32."""
    for n, img, v, c, img_u8, mask, returned in _mask_cases():
        for layered in (False, True):
            out = oracle.inpaint(img[None], v[None], c[None], 3, layered)[0]
            keep = mask == 0
            assert np.array_equal(out[:, keep], returned[:, keep]), (n, layered)
            assert np.array_equal(returned, np.transpose(img_u8, (2, 0, 1)).astype(np.float32))
            assert out.dtype == np.float32 and np.all(out == np.round(out)) and out.min() >= 0 and out.max() <= 255


def test_layered_close_to_sequential_telea_on_smooth_images():
    """The documented divergence of the GPU's layered marching from cv2's order."""
    diffs = []
    for seed in range(3):
        h, w = 60, 80
        img = smooth_image(h, w, seed)
        v, c = blob_masks(h, w, seed)
        a = oracle.inpaint(img[None] * v[None], v[None], c[None], 3, False)[0]
        b = oracle.inpaint(img[None] * v[None], v[None], c[None], 3, True)[0]
        hole = oracle.inpaint_mask(v[None], c[None])[0] == 1
        d = np.abs(a - b)[:, hole]
        diffs.append(d.mean())
        # both fills stay near the smooth truth (the image before the holes were
        # cut), and the layered fill is no worse than cv2's order by more than a level
        err_seq, err_lay = np.abs(a - img)[:, hole].mean(), np.abs(b - img)[:, hole].mean()
        assert err_seq < 8 and err_lay < err_seq + 1.0, (err_seq, err_lay)
    assert max(diffs) < 3.0, diffs


def test_oracle_edge_cases():
    img = np.full((1, 3, 2, 2), 77.0, np.float32)
    v = np.zeros((1, 1, 2, 2), np.float32)
    c = np.zeros_like(v)
    # no known pixel at all: cv2 has an empty band and returns the input
    for layered in (False, True):
        assert np.array_equal(oracle.inpaint(img, v, c, 3, layered), img)
    with pytest.raises(ValueError):
        oracle.inpaint(np.zeros((1, 3, 1, 4), np.float32), np.ones((1, 1, 1, 4), np.float32),
                       np.zeros((1, 1, 1, 4), np.float32))


# ---------------------------------------------------------------- GPU parity
def _gpu_cases():
    rng = np.random.default_rng(7)
    cases = []
    for n, img, v, c, _, _, _ in _mask_cases():
        cases.append((f"fixture{n}", img[None], v[None], c[None], 3))
    for seed, (h, w) in enumerate([(60, 80), (33, 47), (96, 128)]):
        img = smooth_image(h, w, seed)
        v, c = blob_masks(h, w, seed, frac=0.1 + 0.1 * seed)
        cases.append((f"smooth{h}x{w}", (img * v)[None], v[None], c[None], 3))
    # batch of 3 with collisions and random holes, several radii and channel counts
    for r in (1, 3, 5):
        for C in (1, 3, 4, 6):
            B, h, w = 3, 24, 36
            img = rng.integers(0, 256, (B, C, h, w)).astype(np.float32)
            v = (rng.random((B, 1, h, w)) < 0.6).astype(np.float32)
            c = ((rng.random((B, 1, h, w)) < 0.2) & (v > 0)).astype(np.float32)
            cases.append((f"rand_r{r}_C{C}", img, v, c, r))
    # ragged / tiny shapes, a large hole, no holes, all holes
    for h, w in ((2, 2), (2, 9), (9, 2), (3, 3)):
        img = rng.integers(0, 256, (1, 3, h, w)).astype(np.float32)
        v = (rng.random((1, 1, h, w)) < 0.5).astype(np.float32)
        cases.append((f"tiny{h}x{w}", img, v, np.zeros_like(v), 3))
    # wide rows: W > 1024 takes the chunked ROWS kernel (W % 4 == 0: PREP4;
    # W % 4 != 0: the per-pixel PREP), both beside the register ROWS path
    for h, w in ((12, 1100), (10, 1030)):
        img = rng.integers(0, 256, (2, 3, h, w)).astype(np.float32)
        v = (rng.random((2, 1, h, w)) < 0.7).astype(np.float32)
        cases.append((f"wide{h}x{w}", img, v, np.zeros_like(v), 3))
    h, w = 40, 50
    img = smooth_image(h, w, 9)[None]
    v = np.ones((1, 1, h, w), np.float32)
    v[..., 5:35, 10:45] = 0
    cases.append(("bighole", img * v, v, np.zeros_like(v), 3))
    cases.append(("noholes", img, np.ones_like(v), np.zeros_like(v), 3))
    cases.append(("allholes", img, np.zeros_like(v), np.zeros_like(v), 3))
    return cases


@pytest.mark.gpu
@pytest.mark.parametrize("case", _gpu_cases(), ids=lambda c: c[0])
def test_inpaint_gpu_bit_exact_vs_layered_oracle(case):
    from opticalflowfromdepth_amd import ops
    name, img, v, c, r = case
    dev = torch.device("cuda:0")
    got = ops.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                      radius=r, order="layered").cpu().numpy()
    exp = oracle.inpaint(img, v, c, r, layered=True)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, f"{name}: {len(bad)} differing values, first {bad[:5].tolist()}"


def _seq_extra_cases():
    """Shapes that stress the bucketed march: curved and diagonal fronts (many
    distinct distances per bucket), buckets above the LDS sort capacity with
    distinct distances (scattered holes over a large image), a hole touching
    every border, thin snakes (long distance chains), a one-pixel frame of
    known pixels."""
    rng = np.random.default_rng(11)
    cases = []
    h, w = 96, 120
    yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    img = smooth_image(h, w, 3)[None]
    v = np.ones((1, 1, h, w), np.float32)
    v[0, 0][(yy - 40) ** 2 + (xx - 60) ** 2 < 30 ** 2] = 0
    v[0, 0][np.abs(yy - xx) < 4] = 0
    cases.append(("disk_diag", img * v, v, np.zeros_like(v), 3))
    h, w = 200, 300  # band ~ 20 k pixels, distances 0.707 / 0.966 / 1 ... per bucket
    img = rng.integers(0, 256, (1, 3, h, w)).astype(np.float32)
    v = (rng.random((1, 1, h, w)) < 0.55).astype(np.float32)
    cases.append(("scattered200x300", img, v, np.zeros_like(v), 3))
    h, w = 64, 80
    img = smooth_image(h, w, 4)[None]
    v = np.zeros((1, 1, h, w), np.float32)
    v[..., 20:44, 30:50] = 1  # a known island: the hole touches every border
    cases.append(("island", img * v, v, np.zeros_like(v), 3))
    v = np.ones((1, 1, h, w), np.float32)
    for k in range(4, h - 4, 6):  # snake: long thin corridors
        v[..., k:k + 2, 2:w - 2] = 0
        v[..., k:k + 6, (2 if (k // 6) % 2 else w - 4):(4 if (k // 6) % 2 else w - 2)] = 0
    cases.append(("snake", img * v, v, np.zeros_like(v), 3))
    v = np.zeros((1, 1, h, w), np.float32)
    v[..., 0, :] = v[..., -1, :] = v[..., :, 0] = v[..., :, -1] = 1
    cases.append(("frame_only", img * v, v, np.zeros_like(v), 3))
    img = rng.integers(0, 256, (2, 3, 48, 64)).astype(np.float32)
    v = np.ones((2, 1, 48, 64), np.float32)
    v[0, :, :, :25] = 0   # left border band (ego-motion strip)
    v[1, :, 30:, :] = 0   # bottom band
    cases.append(("border_bands", img * v, v, np.zeros_like(v), 3))
    return cases


@pytest.mark.gpu
@pytest.mark.parametrize("case", _gpu_cases() + _seq_extra_cases(), ids=lambda c: c[0])
def test_inpaint_gpu_bit_exact_vs_sequential_oracle(case):
    """order="sequential": cv2's heap order (the oracle's restatement of
    icvCalcFMM / icvTeleaInpaintFMM), bit for bit."""
    from opticalflowfromdepth_amd import ops
    name, img, v, c, r = case
    dev = torch.device("cuda:0")
    got = ops.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                      radius=r, order="sequential").cpu().numpy()
    exp = oracle.inpaint(img, v, c, r, layered=False)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, f"{name}: {len(bad)} differing values, first {bad[:5].tolist()}"


@pytest.mark.gpu
def test_inpaint_sequential_after_warp_headline_shape():
    """The pipeline's use at the headline shape: FW then inpaint the warped RGB
    (preprocess.py:358-366), 768x1024, disparity and ego-motion holes, cv2 order."""
    from opticalflowfromdepth_amd import forward_warp_flow, ops, synth
    dev = torch.device("cuda:0")
    obj, flow, depth = synth.stage_one_batch([12345, 12346, 12377, 12378], 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    got = ops.inpaint(rgb, valid, coll, order="sequential").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=False)
    assert np.array_equal(got, exp)


@pytest.mark.gpu
def test_inpaint_layered_deep_ego_layers_every_schedule():
    """The bench's own images (shard seeds: ego-motion border bands ~300 hole
    layers deep at 768x1024) through the layered fill: the first call at a
    shape (no statistics: every possible layer launched), the one-workgroup
    tail taking every layer past 64, and a call sized from the statistics --
    all the layered oracle's bits, no fault bit."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, shard, synth
    lib = _native.lib()
    dev = torch.device("cuda:0")
    seeds = [shard.image_seed(i) for i in range(3)]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev, ego_fraction=0.67)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=True)
    lib.ofd_inpaint_faults(1)
    try:
        for sched in ((-1, -1), (64, -1), (-1, -1)):
            lib.ofd_inpaint_set_schedule(*sched)
            got = ops.inpaint(rgb, valid, coll, order="layered")
            torch.cuda.synchronize()
            bad = np.argwhere(got.cpu().numpy() != exp)
            assert bad.size == 0, f"{sched}: {len(bad)} differing, first {bad[:5].tolist()}"
    finally:
        lib.ofd_inpaint_set_schedule(-1, -1)
    assert lib.ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
def test_inpaint_layered_deep_call_after_shallow_history():
    """the launch schedule is sized from the last 8 calls at a
    shape, so a deep call after 8 shallow ones runs its extra layers in the
    one-workgroup tail (ofd_inpaint_tail_layers counts them).  Results stay
    the layered oracle's bits; the count shows the cliff is taken, and a
    second deep call (now in the history) takes none.  tools/tail_cliff.py
    times the same sequence."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, shard, synth
    lib = _native.lib()
    dev = torch.device("cuda:0")
    H, W = 384, 512
    seeds = [shard.image_seed(i) for i in range(2)]
    shallow = synth.stage_one_batch(seeds, H, W, dev, ego_fraction=0.0)  # disparity flows: thin holes
    deep = synth.stage_one_batch(seeds, H, W, dev, ego_fraction=1.0)     # ego-motion: deep border bands

    def fill_inputs(batch):
        out, valid, coll = forward_warp_flow(*batch)
        return (out[:, 0:3] * valid).contiguous(), valid, coll

    s_in, d_in = fill_inputs(shallow), fill_inputs(deep)
    exp = oracle.inpaint(*(t.cpu().numpy() for t in d_in), 3, layered=True)
    lib.ofd_inpaint_set_schedule(-1, -1)
    for _ in range(10):
        ops.inpaint(*s_in, order="layered")
    torch.cuda.synchronize()
    time.sleep(0.05)  # let the statistics copies land (they are read only once complete)
    ops.inpaint(*s_in, order="layered")
    torch.cuda.synchronize()
    lib.ofd_inpaint_tail_layers(1)
    got = ops.inpaint(*d_in, order="layered")
    torch.cuda.synchronize()
    n_cliff = lib.ofd_inpaint_tail_layers(1)
    assert np.array_equal(got.cpu().numpy(), exp)
    assert n_cliff > 0
    time.sleep(0.05)
    ops.inpaint(*d_in, order="layered")
    torch.cuda.synchronize()
    lib.ofd_inpaint_tail_layers(1)
    got2 = ops.inpaint(*d_in, order="layered")
    torch.cuda.synchronize()
    assert lib.ofd_inpaint_tail_layers(1) == 0
    assert np.array_equal(got2.cpu().numpy(), exp)
    assert lib.ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
def test_inpaint_reference_call_shape_and_device():
    """utils.inpaint(img[3,H,W], valid[1,H,W], collision[1,H,W]) -> float32 [3,H,W] on img's device."""
    from opticalflowfromdepth_amd import utils
    _, img, v, c, _, mask, returned = next(iter(_mask_cases()))
    dev = torch.device("cuda:0")
    out = utils.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev))
    assert out.device == dev and out.dtype == torch.float32 and tuple(out.shape) == img.shape
    keep = mask == 0
    assert np.array_equal(out.cpu().numpy()[:, keep], returned[:, keep])


@pytest.mark.gpu
def test_inpaint_after_warp_headline_shape():
    """The pipeline's use: FW then inpaint the warped RGB (preprocess.py:358-366), 768x1024 x 4 images."""
    from opticalflowfromdepth_amd import forward_warp_flow, ops, synth
    dev = torch.device("cuda:0")
    seeds = [12345, 12346, 12347, 12348]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    got = ops.inpaint(rgb, valid, coll, order="layered").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=True)
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("sched", [(0, 0), (0, 1 << 30), (1, 0), (3, 64), (-1, -1)],
                         ids=["tail-only-thread", "tail-only-wave", "1-launch", "3-launches-thin64", "default"])
def test_inpaint_gpu_schedules_bit_exact(sched):
    """Every schedule of the hole layers -- one launch per layer or the
    one-workgroup deep-tail kernel, thread or wave paths --
    gives the layered oracle's bits (the schedule steers speed only)."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, synth
    lib = _native.lib()
    dev = torch.device("cuda:0")
    cases = [c for c in _gpu_cases() if c[0] in ("bighole", "smooth96x128", "rand_r3_C3", "rand_r1_C4", "wide12x1100")]
    obj, flow, depth = synth.stage_one_batch([12345, 12377], 192, 256, dev)  # disparity + ego-motion holes
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    cases.append(("warped", (out[:, 0:3] * valid).cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3))
    lib.ofd_inpaint_set_schedule(*sched)
    try:
        for name, img, v, c, r in cases:
            exp = oracle.inpaint(img, v, c, r, layered=True)
            for rep in range(2):  # the second call sees the first one's layer statistics
                got = ops.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev),
                                  torch.from_numpy(c).to(dev), radius=r, order="layered")
                torch.cuda.synchronize()
                bad = np.argwhere(got.cpu().numpy() != exp)
                assert bad.size == 0, f"{name} {sched} rep{rep}: {len(bad)} differing, first {bad[:5].tolist()}"
    finally:
        lib.ofd_inpaint_set_schedule(-1, -1)


def test_layered_vs_sequential_divergence_on_warped_images():
    """The documented divergence of the layered fill from the
    sequential (cv2-order) restatement on the real workload's kind of image:
    warped 384x512 RGB with disparity holes and ego-motion border strips,
    measured over the filled values.  The bound asserted here is the spec;
    bench.py reports the same statistics on the 768x1024 batch."""
    from opticalflowfromdepth_amd import synth
    seeds = [12345, 12346, 12377, 12378]          # 2 disparity + 2 ego-motion
    obj, flow, depth = synth.stage_one_batch(seeds, 384, 512, "cpu")
    o, v, c = oracle.fw_flow(obj.numpy(), flow.numpy(), depth.numpy())
    rgb = o[:, 0:3] * v
    seq = oracle.inpaint(rgb, v, c, 3, layered=False)
    lay = oracle.inpaint(rgb, v, c, 3, layered=True)
    hole = np.broadcast_to(oracle.inpaint_mask(v, c)[:, None] != 0, seq.shape)
    d = np.abs(seq.astype(np.int32) - lay.astype(np.int32))[hole]
    assert d.size > 0
    stats = dict(mean=float(d.mean()), p99=float(np.percentile(d, 99)), frac_over_8=float((d > 8).mean()),
                 frac_over_32=float((d > 32).mean()))
    assert stats["mean"] < 8.0 and stats["p99"] < 64 and stats["frac_over_32"] < 0.05, stats


@pytest.fixture(autouse=True)
def _no_fill_faults(request):
    """Every GPU hole-fill test ends with no invariant-violation bit raised
    (ofd_inpaint_faults: a sequential bucket
    or distance sweep past its bound); each would mean an incomplete fill."""
    yield
    if request.node.get_closest_marker("gpu") is not None and torch.cuda.is_available():
        from opticalflowfromdepth_amd import _native
        torch.cuda.synchronize()
        assert _native.lib().ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
def test_inpaint_tail_beside_a_persistent_warp():
    """The layered fill's deep-tail kernel (schedule (0, 0): every layer on it)
    runs while the FW warp's persistent SPLAT holds CUs on another stream: it
    is one workgroup that waits on no other (no co-residency
    assumed), so the bits stay the oracle's."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, synth
    lib = _native.lib()
    dev = torch.device("cuda:0")
    obj, flow, depth = synth.stage_one_batch([12345, 12377], 192, 256, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    img = (out[:, 0:3] * valid).contiguous()
    exp = oracle.inpaint(img.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=True)
    big = synth.stage_one_batch([12345 + i for i in range(32)], 768, 1024, dev)
    side = torch.cuda.Stream(dev)
    lib.ofd_inpaint_set_schedule(0, 0)
    try:
        torch.cuda.synchronize()
        for rep in range(3):
            with torch.cuda.stream(side):
                for _ in range(4):
                    forward_warp_flow(*big)
            got = ops.inpaint(img, valid, coll, order="layered")
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), exp), rep
    finally:
        lib.ofd_inpaint_set_schedule(-1, -1)
    assert lib.ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
def test_inpaint_sequential_near_the_bucket_margin():
    """The 0.7-wide distance buckets (H + W < 8000) at the largest distances
    they allow: a 6 x 7990 strip known only at its left column (plus a few
    islands in the first half for oblique fronts), so the march runs ~11 k
    buckets and T climbs to ~7990, where a float ulp of T is largest against
    the 1/sqrt(2) - 0.7 margin the bucketing relies on.  cv2 order, bit-exact,
    no fault bit (a bucket index past its bound would raise one)."""
    from opticalflowfromdepth_amd import _native, ops
    lib = _native.lib()
    rng = np.random.default_rng(33)
    h, w = 6, 7990
    img = rng.integers(0, 256, (1, 3, h, w)).astype(np.float32)
    v = np.zeros((1, 1, h, w), np.float32)
    v[..., :, 0] = 1
    isl = rng.integers(50, w // 2, 12)
    for x in isl:
        v[..., rng.integers(0, h), x:x + 2] = 1
    c = np.zeros_like(v)
    dev = torch.device("cuda:0")
    lib.ofd_inpaint_faults(1)
    got = ops.inpaint(torch.from_numpy(img * v).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                      order="sequential").cpu().numpy()
    torch.cuda.synchronize()
    assert lib.ofd_inpaint_faults(1) == 0
    assert np.array_equal(got, oracle.inpaint(img * v, v, c, 3, layered=False))


@pytest.mark.gpu
def test_inpaint_sequential_wide_image_half_unit_buckets():
    """H + W >= 8000 takes the half-unit distance buckets (the 0.7-wide ones
    need T < 8192); a long strip with holes of every kind, cv2 order, bit-exact."""
    from opticalflowfromdepth_amd import ops
    rng = np.random.default_rng(21)
    h, w = 10, 8200
    img = rng.integers(0, 256, (1, 3, h, w)).astype(np.float32)
    v = (rng.random((1, 1, h, w)) < 0.7).astype(np.float32)
    v[..., :, 100:400] = 0  # a wide hole
    v[..., :, -50:] = 0     # a border band
    c = ((rng.random((1, 1, h, w)) < 0.05) & (v > 0)).astype(np.float32)
    dev = torch.device("cuda:0")
    got = ops.inpaint(torch.from_numpy(img * v).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                      order="sequential").cpu().numpy()
    assert np.array_equal(got, oracle.inpaint(img * v, v, c, 3, layered=False))


@pytest.mark.gpu
def test_inpaint_sequential_helpers_follow_the_stream_device(cuda_device):
    """The grouped fill's helper streams are kept per device and chosen by the
    caller's stream's device: a call on a stream of device d
    forks onto helpers created on d, whichever device is current."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    for d in range(torch.cuda.device_count()):
        with torch.cuda.device(d):
            s = torch.cuda.Stream()
        with torch.cuda.device(0):  # current device 0, stream on d
            assert lib.ofd_inpaint_seq_helper_device(ctypes.c_void_p(s.cuda_stream)) == d
        with torch.cuda.device(d):
            assert lib.ofd_inpaint_seq_helper_device(None) == d  # the null stream: the current device


# ------------------------------------------------------------------ pipelined record / colour rounds
@pytest.fixture
def seq_pipeline():
    """Sets the pipelined fill's rounds for one test (ofd_inpaint_seq_set_pipeline)
    and restores the defaults afterwards."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_inpaint_seq_set_pipeline(-1, -1, -1)

    def set_(rounds, us, force):
        lib.ofd_inpaint_seq_set_pipeline(rounds, us, force)
    yield set_
    lib.ofd_inpaint_seq_set_pipeline(prev, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", _gpu_cases() + _seq_extra_cases(), ids=lambda c: c[0])
def test_inpaint_sequential_pipelined_rounds_bit_exact(case, seq_pipeline):
    """The RECORD / COLOUR3 rounds running beside the marches (forced on these
    small images, 64 rounds 2 us apart, so rounds interleave with every stage
    of the march): cv2's order bit for bit, as the unpipelined fill."""
    from opticalflowfromdepth_amd import ops
    name, img, v, c, r = case
    dev = torch.device("cuda:0")
    seq_pipeline(64, 2, 1)
    got = ops.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                      radius=r, order="sequential").cpu().numpy()
    exp = oracle.inpaint(img, v, c, r, layered=False)
    bad = np.argwhere(got != exp)
    assert bad.size == 0, f"{name}: {len(bad)} differing values, first {bad[:5].tolist()}"


@pytest.fixture
def seq_colour():
    """Sets the sequential fill's colour pass for one test
    (ofd_inpaint_seq_set_colour) and restores it afterwards."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_inpaint_seq_set_colour(-1)
    yield lambda mode: lib.ofd_inpaint_seq_set_colour(mode)
    lib.ofd_inpaint_seq_set_colour(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["levels", "levels_free"])
@pytest.mark.parametrize("case", _gpu_cases() + _seq_extra_cases(), ids=lambda c: c[0])
def test_inpaint_sequential_colour_passes_bit_exact(case, mode, seq_colour, seq_pipeline):
    """Both colour passes -- level-synchronous COLOUR3 and the levels-free pass
    (a hole starts once its last earlier neighbour has released it and waits
    for their coloured flags) -- unpipelined and in forced short rounds that
    carry their queue: cv2's order bit for bit."""
    from opticalflowfromdepth_amd import _native, ops
    name, img, v, c, r = case
    dev = torch.device("cuda:0")
    seq_colour(mode)
    exp = oracle.inpaint(img, v, c, r, layered=False)
    for rounds, us, force in ((0, 2000, 0), (64, 2, 1)):
        seq_pipeline(rounds, us, force)
        got = ops.inpaint(torch.from_numpy(img).to(dev), torch.from_numpy(v).to(dev), torch.from_numpy(c).to(dev),
                          radius=r, order="sequential").cpu().numpy()
        bad = np.argwhere(got != exp)
        assert bad.size == 0, f"{name} rounds {rounds}: {len(bad)} differing values, first {bad[:5].tolist()}"
    assert _native.lib().ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["levels", "levels_free"])
def test_inpaint_sequential_colour_passes_on_warped_images(mode, seq_colour):
    """Warped 768x1024 images (8 at once, pipelined by default): each colour
    pass gives the oracle's cv2 order."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, ops, synth
    dev = torch.device("cuda:0")
    seeds = [12345, 12346, 12377, 12378, 12401, 12402, 12433, 12434]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    seq_colour(mode)
    got = ops.inpaint(rgb, valid, coll, order="sequential").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=False)
    assert np.array_equal(got, exp)
    assert _native.lib().ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("rounds,us", [(0, 2000), (12, 2000), (48, 100), (4, 5000)])
def test_inpaint_sequential_pipeline_settings_agree_on_warped_images(rounds, us, seq_pipeline):
    """Warped 768x1024 images (disparity and ego-motion holes, 8 at once), with
    no rounds, the default rounds, many short rounds and a few long ones: the
    same bits, equal to the oracle's cv2 order."""
    from opticalflowfromdepth_amd import forward_warp_flow, ops, synth
    dev = torch.device("cuda:0")
    seeds = [12345, 12346, 12377, 12378, 12401, 12402, 12433, 12434]
    obj, flow, depth = synth.stage_one_batch(seeds, 768, 1024, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    seq_pipeline(rounds, us, 0)
    got = ops.inpaint(rgb, valid, coll, order="sequential").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=False)
    assert np.array_equal(got, exp)
    from opticalflowfromdepth_amd import _native
    assert _native.lib().ofd_inpaint_faults(1) == 0


# ------------------------------------------------------------------ several workgroups per image
@pytest.fixture
def seq_multi():
    """Sets the levels-free colour pass's workgroups per image for one test
    (ofd_inpaint_seq_set_multi) and restores the setting afterwards."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    prev = lib.ofd_inpaint_seq_set_multi(0, 0)
    yield lambda k, force=0: lib.ofd_inpaint_seq_set_multi(k, force)
    lib.ofd_inpaint_seq_set_multi(prev, 0)


def _warped_rgb(seeds, h, w):
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    dev = torch.device("cuda:0")
    obj, flow, depth = synth.stage_one_batch(seeds, h, w, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    return (out[:, 0:3] * valid).contiguous(), valid, coll


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 4, 8])
def test_inpaint_sequential_multi_workgroup_on_warped_images(k, seq_multi):
    """The levels-free colour pass with k workgroups per image (the image's
    ready holes shared through RECORD's queue, each workgroup's LDS queue and
    a shared queue of tagged granules; colours handed across CUs by
    write-through stores): warped 768x1024 images, 8 at once, pipelined as by
    default -- the oracle's cv2 order bit for bit, no fault bit."""
    from opticalflowfromdepth_amd import _native, ops
    rgb, valid, coll = _warped_rgb([12345, 12346, 12377, 12378, 12401, 12402, 12433, 12434], 768, 1024)
    seq_multi(k)
    got = ops.inpaint(rgb, valid, coll, order="sequential").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=False)
    assert np.array_equal(got, exp), f"k={k}: {int((got != exp).sum())} values differ"
    assert _native.lib().ofd_inpaint_faults(1) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("rounds,us", [(0, 2000), (48, 100), (64, 2)])
@pytest.mark.parametrize("shape", [(192, 256), (384, 512)])
def test_inpaint_sequential_multi_workgroup_rounds_and_shapes(shape, rounds, us, seq_multi, seq_pipeline):
    """k = 4 forced onto smaller warped images (fewer padded pixels per
    workgroup; each workgroup's overflow slice is smaller), with no rounds
    beside the marches, many short ones and very short ones (every round
    flushes its LDS queues into the shared queue for the next): bit for bit
    the oracle's cv2 order."""
    from opticalflowfromdepth_amd import _native, ops
    h, w = shape
    rgb, valid, coll = _warped_rgb([12345, 12346, 12377, 12378], h, w)
    seq_multi(4, 1)
    seq_pipeline(rounds, us, 1)
    got = ops.inpaint(rgb, valid, coll, order="sequential").cpu().numpy()
    exp = oracle.inpaint(rgb.cpu().numpy(), valid.cpu().numpy(), coll.cpu().numpy(), 3, layered=False)
    assert np.array_equal(got, exp), f"{shape} rounds {rounds}: {int((got != exp).sum())} values differ"
    assert _native.lib().ofd_inpaint_faults(1) == 0
