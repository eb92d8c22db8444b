"""The callers around the warp (preprocess.py:24-326, :329-450): SpecialFlow,
augment_flow, ConcatFlow, BackFlow and the PreprocessPlusAugment first stage,
against tests/golden/augment.npz (the reference's own code slices run on CPU
with the oracle as fw_cuda; see tests/golden/make_golden.py).

Bit-exact where the computation is elementwise or an FW call on identical
inputs; the special-flow and ego-motion geometry (2x2 / 3x3 products, cos /
sin) is held to the north_star's fp32 flow tolerance (1e-5 relative) because
the reference evaluates it on the GPU with unspecified summation order.
Image channels after utils.inpaint are compared on kept pixels only: the
fixture's cv2 stand-in returns the uint8 cast unchanged (fill values are the
hole-fill's own test, tests/test_inpaint.py).
"""
import os

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import oracle

G = np.load(os.path.join(REPO, "tests", "golden", "augment.npz"))
FLOW_RTOL, FLOW_ATOL = 1e-5, 1e-4  # pixel units


def _in(k):
    return torch.from_numpy(G[f"in/{k}"])


# ---------------------------------------------------------------- CPU
@pytest.mark.parametrize("kind", [5, 6, 7])
def test_special_flows_match_reference_geometry(kind):
    from opticalflowfromdepth_amd import preprocess as pp
    from opticalflowfromdepth_amd import utils
    h, w = G["in/img0"].shape[-2:]
    utils.set_seed(int(G[f"aug{kind}/seed"]))
    p = pp.draw_augment_params(kind, h, w)
    sf, bsf = pp.special_flow_from_params(h, w, kind, None if kind == 5 else (p.view(1, -1) if kind == 6 else p.view(1)),
                                          "cpu")
    if kind == 5:
        assert np.array_equal(sf[0].numpy(), G[f"aug{kind}/special"])
        assert np.array_equal(bsf[0].numpy(), G[f"aug{kind}/back_special"])
    else:
        np.testing.assert_allclose(sf[0].numpy(), G[f"aug{kind}/special"], rtol=FLOW_RTOL, atol=FLOW_ATOL)
        np.testing.assert_allclose(bsf[0].numpy(), G[f"aug{kind}/back_special"], rtol=FLOW_RTOL, atol=FLOW_ATOL)


def test_special_flow_module_state_and_draws():
    """A fresh SpecialFlow flips / shears vertically first, then alternates (preprocess.py:49, :83)."""
    from opticalflowfromdepth_amd import preprocess as pp
    from opticalflowfromdepth_amd import utils
    h, w = 6, 9
    sfm = pp.SpecialFlow("cpu")
    f1, _ = sfm((h, w), 5)
    f2, _ = sfm((h, w), 5)
    assert torch.all(f1[0] == 0) and torch.any(f1[1] != 0)  # vertical flip
    assert torch.all(f2[1] == 0) and torch.any(f2[0] != 0)  # then horizontal
    utils.set_seed(3)
    s1, _ = sfm((h, w), 7)
    utils.set_seed(3)
    shear = pp.draw_augment_params(7, h, w)
    assert torch.all(s1[0] == 0)
    np.testing.assert_allclose(s1[1].numpy(), (torch.arange(w, dtype=torch.float32) * shear).expand(h, w).numpy(),
                               rtol=1e-6, atol=1e-5)


def test_first_stage_draws_match_reference():
    """draw_image_params replays s of the reference's first stage: flow01 of group.npz."""
    from opticalflowfromdepth_amd import preprocess as pp
    from opticalflowfromdepth_amd import synth
    raw = torch.from_numpy(G["ppa/raw_depth"]).view(1, 1, *G["ppa/raw_depth"].shape)
    h, w = raw.shape[-2:]
    prm = pp.draw_image_params(int(G["ppa/seed"]), h, w)
    d0 = synth.normalize_depth(raw)
    flow01 = pp.Convert.disparity_to_flow(pp.Convert.depth_to_disparity(d0, prm["s"].view(1)), random_sign=False)
    g = G["ppa/group"]
    assert np.array_equal(flow01[0].numpy(), g[24:26])
    assert np.array_equal(d0[0].numpy(), g[3:4])


def test_augment_schedule_and_layout_constants():
    from opticalflowfromdepth_amd import preprocess as pp
    assert pp.AUGMENT_SCHEDULE == (0, 5, 6, 7, 1, 5, 6, 7, 2, 5, 6, 7)
    assert pp.N_GROUPS == 5
    assert pp.augment_flow_batch(*(torch.zeros(1, 1, 2, 2),) * 6, 3, [None]) is None


# ---------------------------------------------------------------- GPU
def _dev(t):
    return t.to("cuda:0")


def _keep(valid, coll):
    return oracle.inpaint_mask(valid.cpu().numpy()[None], coll.cpu().numpy()[None])[0] == 0


@pytest.mark.gpu
def test_concat_and_back_flow_bit_exact():
    from opticalflowfromdepth_amd import preprocess as pp
    cf, bf = pp.ConcatFlow("cuda:0"), pp.BackFlow("cuda:0")
    fBC = _dev(torch.from_numpy(G["cf/flowBC"]))
    o, v = cf(_dev(_in("flow01")), _dev(_in("back01")), fBC, _dev(_in("d1")))
    assert np.array_equal(o.cpu().numpy(), G["cf/out"]) and np.array_equal(v.cpu().numpy(), G["cf/valid"])
    o, v = bf(fBC, _dev(_in("d1")).to(torch.float32))
    assert np.array_equal(o.cpu().numpy(), G["bf/out"]) and np.array_equal(v.cpu().numpy(), G["bf/valid"])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1, 2, 5, 6, 7])
def test_augment_flow_matches_reference(kind):
    from opticalflowfromdepth_amd import FW, preprocess as pp
    from opticalflowfromdepth_amd import utils
    h, w = G["in/img0"].shape[-2:]
    args = [_dev(_in(k)) for k in ("img0", "d0", "img1", "d1", "flow01", "back01")]
    utils.set_seed(int(G[f"aug{kind}/seed"]))
    p = pp.draw_augment_params(kind, h, w)
    specials = None
    if kind >= 5:  # identical special flows: everything downstream is an FW call or elementwise
        specials = (_dev(torch.from_numpy(G[f"aug{kind}/special"]))[None],
                    _dev(torch.from_numpy(G[f"aug{kind}/back_special"]))[None])
    set1, set2, typ, _ = pp.augment_flow_batch(*[a[None] for a in args], kind, [p], specials=specials)
    assert typ == int(G[f"aug{kind}/type"])
    img_slots = {(1, 0), (2, 4)} if kind >= 5 else set()
    for si, st in ((1, set1), (2, set2)):
        for n, t in enumerate(st):
            got, exp = t[0].cpu().numpy(), G[f"aug{kind}/set{si}_{n}"]
            assert got.shape == exp.shape and got.dtype == exp.dtype, (si, n, got.dtype, exp.dtype)
            if kind == 2 and n in ((0,) if si == 1 else (4,)):
                np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-4)  # gray matmul
            elif (si, n) in img_slots:
                src = (args[0], args[1]) if si == 1 else (args[2], args[3])
                _, valid, coll = FW()(torch.cat(src, 0), specials[0][0], src[1])
                keep = _keep(valid, coll)
                assert np.array_equal(got[:, keep], exp[:, keep]), (si, n)
            else:
                assert np.array_equal(got, exp), (si, n)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [6, 7])
def test_special_flows_on_device_close_to_reference(kind):
    from opticalflowfromdepth_amd import preprocess as pp
    from opticalflowfromdepth_amd import utils
    h, w = G["in/img0"].shape[-2:]
    utils.set_seed(int(G[f"aug{kind}/seed"]))
    p = pp.draw_augment_params(kind, h, w)
    sf, bsf = pp.special_flow_from_params(h, w, kind, p.view(1, -1) if kind == 6 else p.view(1), "cuda:0")
    np.testing.assert_allclose(sf[0].cpu().numpy(), G[f"aug{kind}/special"], rtol=FLOW_RTOL, atol=FLOW_ATOL)
    np.testing.assert_allclose(bsf[0].cpu().numpy(), G[f"aug{kind}/back_special"], rtol=FLOW_RTOL, atol=FLOW_ATOL)


@pytest.mark.gpu
def test_first_stage_group_matches_reference():
    """PreprocessPlusAugment.run_batch's 44-channel group vs the reference's group.npz."""
    from opticalflowfromdepth_amd import preprocess as pp
    g = G["ppa/group"]
    raw = torch.from_numpy(G["ppa/raw_depth"]).view(1, 1, *g.shape[-2:])
    ppa = pp.PreprocessPlusAugment("cuda:0")
    got = ppa.run_batch([int(G["ppa/seed"])], _dev(_in("img0"))[None], _dev(raw), augment=False)[0].cpu().numpy()
    assert got.shape == g.shape and got.dtype == g.dtype
    # group layout (preprocess.py:437-440): img0 0:3, img0_depth 3, img1 4:7,
    # img1_depth 7, ..., flow01 24:26, back_flow01 26:28, flow12 28:30, ...,
    # flow03 36:38.  Exact: img0 / depth, the disparity warp's depth and flows
    for a, b in ((0, 4), (7, 8), (24, 28)):
        assert np.array_equal(got[a:b], g[a:b]), (a, b)
    # img1 on kept pixels (the fixture's cv2 stand-in does not fill holes)
    hole = (g[7] == 100) & (got[4:7] != g[4:7]).any(0)
    assert np.array_equal(got[4:7][:, ~hole], g[4:7][:, ~hole])
    # ego-motion flows (geometry on device): fp32 tolerance
    for a in (28, 36):  # flow12, flow03
        np.testing.assert_allclose(got[a:a + 2], g[a:a + 2], rtol=FLOW_RTOL, atol=1e-3)
    # depths and flows downstream of them (the image channels differ at holes by
    # construction: the fixture does not fill them): the same almost everywhere
    ch = [11, 15, 19, 23] + list(range(28, 44))
    agree = np.isclose(got[ch], g[ch], rtol=1e-5, atol=1e-3).mean()
    assert agree > 0.99, agree
