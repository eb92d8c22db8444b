"""CPU tests: the oracle against the golden fixtures and against itself.

The fixtures were produced by tests/golden/make_golden.py, which drives the
reference's own alt_cuda/fw.py / geometry.py / utils.py / preprocess.py slice
(see its docstring).  These tests pin the oracle before any GPU test trusts it.
"""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from oracle import oracle


@pytest.fixture(scope="module")
def op_cases():
    return golden_cases(load_golden("fw_op.npz"))


@pytest.fixture(scope="module")
def wrapper_cases():
    return golden_cases(load_golden("fw_wrapper.npz"))


def _eq(a, b):
    return np.array_equal(a, b)


def test_golden_op_cases_present(op_cases):
    assert {"ties_c1", "ties_c6", "ties_c7", "coll_c6", "negzero_c3", "hotspot_c6",
            "nonint_c2", "ties_f64_c4", "ragged_1x1"} <= set(op_cases)


@pytest.mark.parametrize("name", ["ties_c1", "ties_c2", "ties_c4", "ties_c6", "ties_c7", "coll_c6",
                                  "negzero_c3", "hotspot_c6", "nonint_c2", "ties_f64_c4",
                                  "ragged_1x1", "ragged_1xw", "ragged_hx1"])
def test_oracle_loop_matches_golden_op(op_cases, name):
    c = op_cases[name]
    out, valid, coll = oracle.forward_warping(c["obj"], c["safe_y"], c["safe_x"], c["depth"])
    assert out.dtype == c["obj"].dtype
    assert _eq(out, c["output"]) and _eq(valid, c["valid"]) and _eq(coll, c["collision"])


@pytest.mark.parametrize("name", ["ties_c6", "coll_c6", "negzero_c3", "hotspot_c6", "nonint_c2"])
def test_lexmin_formulation_matches_golden_op(op_cases, name):
    c = op_cases[name]
    out, valid, coll = oracle.forward_warping_lexmin(c["obj"], c["safe_y"], c["safe_x"], c["depth"])
    assert _eq(out, c["output"]) and _eq(valid, c["valid"]) and _eq(coll, c["collision"])


def test_collision_path_exercised(op_cases):
    c = op_cases["coll_c6"]
    assert c["collision"].sum() > 0
    # collision implies valid; a collision pixel has an all-zero output
    assert np.all(c["valid"][c["collision"] == 1] == 1)
    m = np.broadcast_to(c["collision"] == 1, c["output"].shape)
    assert np.all(c["output"][m] == 0)


@pytest.mark.parametrize("name", ["f32_c6", "f32_c2_big", "f64flow_c6", "f64obj_c4", "nearint_f64"])
def test_oracle_wrapper_matches_reference_fw_py(wrapper_cases, name):
    """Golden outputs came from the reference alt_cuda/fw.py (3-D path)."""
    c = wrapper_cases[name]
    obj, flow, depth = c["obj"][None], c["flow"][None], c["depth"][None]
    out, valid, coll = oracle.fw_flow(obj, flow, depth)
    assert _eq(out[0], c["output"]) and _eq(valid[0], c["valid"]) and _eq(coll[0], c["collision"])


def test_float64_flow_add_is_float64(wrapper_cases):
    """fw.py:31 promotes p0 + flow to float64: 0.99999999 must not round up to 1."""
    c = wrapper_cases["nearint_f64"]
    out, valid, coll = oracle.fw_flow(c["obj"][None], c["flow"][None], c["depth"][None])
    # row 0: x + 0.99999999 truncates to x, so every pixel maps onto itself
    assert _eq(out[0, 0, 0], c["obj"][0, 0])
    # the same flow in float32 rounds to 1.0 and shifts by one pixel
    out32, _, _ = oracle.fw_flow(c["obj"][None], c["flow"][None].astype(np.float32), c["depth"][None])
    assert not _eq(out32[0, 0, 0], out[0, 0, 0])


def test_pipeline_fw_outputs_match_oracle():
    p = load_golden("pipeline.npz")
    for k in ("img0", "img1"):
        obj = np.concatenate([p[f"{k}/rgb"], p[f"{k}/norm_depth"].astype(np.float32),
                              -p[f"{k}/flow01"].astype(np.float32)], 0)
        out, valid, coll = oracle.fw_flow(obj[None], p[f"{k}/flow01"][None], p[f"{k}/norm_depth"][None])
        assert _eq(out[0], p[f"{k}/fw01_output"]) and _eq(valid[0], p[f"{k}/fw01_valid"])
        assert _eq(coll[0], p[f"{k}/fw01_collision"])
        assert coll.sum() == 0  # real depths are < 1000


def test_loop_vs_lexmin_random_ties():
    rng = np.random.default_rng(7)
    for _ in range(25):
        B, C = int(rng.integers(1, 3)), int(rng.integers(1, 8))
        H, W = int(rng.integers(1, 30)), int(rng.integers(1, 40))
        obj = rng.standard_normal((B, C, H, W)).astype(np.float32)
        flow = (rng.standard_normal((B, 2, H, W)) * rng.uniform(0, 30)).astype(np.float32)
        depth = (rng.integers(0, 4, (B, 1, H, W)) * rng.choice([1, -1, 300, 400])).astype(np.float32)
        depth[rng.random(depth.shape) < 0.05] = np.nan
        sy, sx = oracle.safe_coords(flow)
        a = oracle.forward_warping(obj, sy, sx, depth)
        b = oracle.forward_warping_lexmin(obj, sy, sx, depth)
        for u, v in zip(a, b):
            assert _eq(u, v)


def test_nan_coordinates_dropped():
    obj = np.ones((1, 1, 2, 2), np.float32)
    sy = np.zeros((1, 1, 2, 2), np.float32)
    sx = np.zeros((1, 1, 2, 2), np.float32)
    sx[0, 0, 0, 0] = np.nan
    sy[0, 0, 0, 1] = 5.0  # out of range -> dropped
    depth = np.ones((1, 1, 2, 2), np.float32)
    out, valid, coll = oracle.forward_warping(obj, sy, sx, depth)
    assert valid[0, 0, 0, 0] == 1 and valid.sum() == 1  # only the two in-range sources, both -> (0,0)
