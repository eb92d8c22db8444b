"""tests/golden/make_golden.py -- generates the committed golden fixtures.

Run in the BUILD container only (it reads /root/reference, which does not exist
on the GPU box):

    python tests/golden/make_golden.py

What it does, and what each fixture pins:

* ``fw_wrapper.npz`` -- the reference's own ``alt_cuda/fw.py`` (imported from
  /root/reference, unmodified) driven with 3-D inputs exactly as preprocess.py
  calls it, with ``fw_cuda`` provided by the CPU oracle (oracle/fw_oracle.c,
  the literal restatement of fw_cuda_kernel.cu:28-47).  Pins the wrapper
  arithmetic (meshgrid, add in the flow's dtype, clamp, int64 truncation,
  casts: fw.py:27-43) with the reference's own code.
* ``fw_op.npz`` -- op-level ``forward_warping(obj, safe_y, safe_x, depth)`` cases
  (B up to 3, C in {1,2,4,6,7}, ties, depth >= 1000, -0.0, negative depths,
  hot spots, float64), expected outputs from the oracle loop, cross-checked
  here against the independent lexmin formulation before being written.
* ``pipeline.npz`` -- synthetic depth maps pushed through the reference's own
  ``utils.normalize_depth`` / ``fix_warped_depth`` / ``get_random`` /
  ``set_seed`` (function bodies taken from /root/reference/utils.py by AST,
  so cv2 is not needed), ``Plausible``/``Convert`` (verbatim text slice
  preprocess.py:184-298 -- the file as a whole does not parse, SyntaxError at
  :463) and ``geometry.py`` (imported as is): disparity and ego-motion flows
  with fixed seeds, and FW outputs on them.  Pins
  opticalflowfromdepth_amd.synth (flows within 1e-5) and realistic FW cases.
* ``inpaint_mask.npz`` -- the reference's own ``utils.inpaint`` (utils.py:136-151,
  taken by AST) run with a stand-in ``cv2`` namespace: ``dilate`` is a 3x3
  in-image maximum (what cv2.dilate with a ones(3,3) kernel computes) and
  ``inpaint`` records the uint8 image and mask it is handed and returns the
  image unchanged.  Pins the keep-mask algebra (:137-142), the HWC uint8 cast
  (:148) and the float32 return (:149-151) with the reference's own code; the
  Telea fill values themselves stay unpinned (OpenCV is absent).
* ``augment.npz`` -- the reference's own ``SpecialFlow`` / ``augment_flow``
  (verbatim text slice preprocess.py:24-182), ``ConcatFlow`` / ``BackFlow``
  (:301-326) and the first stage of ``PreprocessPlusAugment.forward``
  (:329-450, which ends at the group.npz save; the rest of the file does not
  parse), run on CPU with the oracle as ``fw_cuda`` and the recording cv2
  (its ``inpaint`` returns the uint8 image unchanged, so hole pixels are the
  cast input and only kept pixels pin image values).  Pins the flow algebra,
  the RNG draw order, the special-flow geometry and the 44-channel layout.

Nothing from /root/reference is copied into the repo: only numeric arrays.
"""
from __future__ import annotations

import ast
import importlib.util
import math
import os
import random
import sys
import types

import numpy as np
import torch

REF = os.environ.get("OFD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
# where the fixtures are written (tests/golden by default; tests/golden/check_regen.py
# regenerates into a temporary directory and compares with the committed files)
OUT = os.environ.get("OFD_GOLDEN_OUT", HERE)
sys.path.insert(0, REPO)

from oracle import oracle  # noqa: E402  (test infrastructure)


# ---------------------------------------------------------------- reference loaders
def _oracle_fw_cuda_module():
    """A module object named fw_cuda whose forward_warping is the CPU oracle."""
    m = types.ModuleType("fw_cuda")

    def forward_warping(obj, safe_y, safe_x, depth):
        out, valid, coll = oracle.forward_warping(
            obj.numpy(), safe_y.numpy(), safe_x.numpy(), depth.numpy())
        return [torch.from_numpy(out), torch.from_numpy(valid), torch.from_numpy(coll)]

    m.forward_warping = forward_warping
    return m


def load_reference_fw():
    sys.modules["fw_cuda"] = _oracle_fw_cuda_module()
    spec = importlib.util.spec_from_file_location("ref_alt_cuda_fw", os.path.join(REF, "alt_cuda", "fw.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_reference_geometry():
    spec = importlib.util.spec_from_file_location("geometry", os.path.join(REF, "geometry.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["geometry"] = mod
    return mod


def load_reference_utils_subset():
    """utils.py functions needed on the path, taken by AST (cv2 is absent here)."""
    src = open(os.path.join(REF, "utils.py")).read()
    tree = ast.parse(src)
    want = {"get_random", "normalize_depth", "fix_warped_depth", "set_seed", "smooth_closer"}
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in want]
    mod = types.ModuleType("utils")
    mod.__dict__.update(torch=torch, np=np, random=random, math=math)
    exec(compile(ast.Module(body=body, type_ignores=[]), os.path.join(REF, "utils.py"), "exec"), mod.__dict__)
    return mod


class _Cv2Recorder:
    """Stand-in cv2 namespace for utils.inpaint: dilate restated, inpaint recorded."""
    INPAINT_TELEA = 1

    def __init__(self):
        self.calls = []

    @staticmethod
    def dilate(M, kernel, iterations=1):
        assert kernel.shape == (3, 3) and kernel.all() and iterations == 1
        H, W = M.shape
        pad = np.zeros((H + 2, W + 2), M.dtype)  # uint8 >= 0: a 0 border never wins the max
        pad[1:-1, 1:-1] = M
        return np.max(np.stack([pad[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)]), axis=0)

    def inpaint(self, img, mask, radius, flags):
        self.calls.append((img.copy(), mask.copy(), radius, flags))
        return img.copy()


class _CpuImage(torch.Tensor):
    """utils.py:150 moves the result to img.get_device(), which is -1 for a CPU
    tensor; this subclass names the CPU instead (the fixture runs on CPU)."""

    def get_device(self):
        return "cpu"


class _Cv2Telea(_Cv2Recorder):
    """Stand-in cv2 whose ``inpaint`` is the oracle's restatement of OpenCV's
    sequential Telea (oracle/inpaint_oracle.c, cv2's heap order): the uint8
    HWC image and the fill mask cv2 would be handed go through it, and the
    uint8 HWC result comes back, as cv2.inpaint returns it.  The mask is fed as
    valid = (mask == 0) with no collisions, for which the oracle's mask algebra
    (utils.py:137-142) gives back exactly this mask."""

    def inpaint(self, img, mask, radius, flags):
        assert flags == self.INPAINT_TELEA and img.dtype == np.uint8 and img.ndim == 3
        self.calls.append((mask.sum(),))
        planes = np.ascontiguousarray(img.transpose(2, 0, 1)[None].astype(np.float32))
        valid = (mask == 0).astype(np.float32)[None, None]
        out = oracle.inpaint(planes, valid, np.zeros_like(valid), int(radius), layered=False)
        return np.ascontiguousarray(out[0].transpose(1, 2, 0).astype(np.uint8))


def load_reference_inpaint(cv2_cls=None):
    """utils.inpaint taken by AST with the recorder (or another stand-in) as cv2."""
    src = open(os.path.join(REF, "utils.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "inpaint"]
    rec = (cv2_cls or _Cv2Recorder)()
    mod = types.ModuleType("utils_inpaint")
    mod.__dict__.update(torch=torch, np=np, cv2=rec)
    exec(compile(ast.Module(body=body, type_ignores=[]), os.path.join(REF, "utils.py"), "exec"), mod.__dict__)
    return mod.inpaint, rec


def load_reference_plausible_convert(utils_mod, geometry_mod):
    """Verbatim text slice preprocess.py:184-298 (class Plausible, class Convert)."""
    lines = open(os.path.join(REF, "preprocess.py")).read().split("\n")
    text = "\n".join(lines[183:298])
    assert text.startswith("class Plausible"), text[:40]
    ns = dict(torch=torch, math=math, utils=utils_mod, geometry=geometry_mod)
    exec(compile(text, os.path.join(REF, "preprocess.py"), "exec"), ns)
    return ns["Plausible"], ns["Convert"]


# ---------------------------------------------------------------- synthetic inputs
def synth_depth(h, w, seed):
    """Smooth synthetic raw depth (opticalflowfromdepth_amd.synth.synthetic_depth_np)."""
    from opticalflowfromdepth_amd.synth import synthetic_depth_np
    return synthetic_depth_np(h, w, seed)


def synth_rgb(h, w, seed):
    rng = np.random.default_rng(seed + 1000)
    return np.floor(rng.uniform(0, 256, (3, h, w))).astype(np.float32)


# ---------------------------------------------------------------- fixtures
def make_op_cases():
    rng = np.random.default_rng(1234)
    cases = {}
    specs = [
        # (name, B, C, H, W, dtype, kind)
        ("ties_c1", 2, 1, 17, 23, np.float32, "ties"),
        ("ties_c2", 1, 2, 24, 32, np.float32, "ties"),
        ("ties_c4", 3, 4, 16, 20, np.float32, "ties"),
        ("ties_c6", 2, 6, 24, 32, np.float32, "ties"),
        ("ties_c7", 1, 7, 31, 29, np.float32, "ties"),
        ("coll_c6", 2, 6, 20, 24, np.float32, "collide"),
        ("negzero_c3", 1, 3, 16, 16, np.float32, "negzero"),
        ("hotspot_c6", 1, 6, 32, 48, np.float32, "hotspot"),
        ("nonint_c2", 2, 2, 18, 22, np.float32, "nonint"),
        ("ties_f64_c4", 2, 4, 20, 24, np.float64, "ties"),
        ("ragged_1x1", 1, 3, 1, 1, np.float32, "ties"),
        ("ragged_1xw", 1, 2, 1, 37, np.float32, "ties"),
        ("ragged_hx1", 2, 2, 41, 1, np.float32, "ties"),
    ]
    for name, B, C, H, W, dt, kind in specs:
        obj = rng.standard_normal((B, C, H, W)).astype(dt)
        flow = (rng.standard_normal((B, 2, H, W)) * 4).astype(np.float32)
        depth = rng.integers(1, 4, (B, 1, H, W)).astype(dt)
        if kind == "collide":
            depth[rng.random(depth.shape) < 0.3] = 1000.0
            depth[rng.random(depth.shape) < 0.2] = 5000.0
        if kind == "negzero":
            depth = rng.choice(np.array([0.0, -0.0, -1.0, 2.0], dt), size=(B, 1, H, W))
        if kind == "hotspot":
            flow = (rng.standard_normal((B, 2, H, W)) * 200).astype(np.float32)
        sy, sx = oracle.safe_coords(flow)
        if kind == "nonint":  # raw, non-integer in-range coordinates (truncated by the op)
            sx = rng.uniform(-0.99, W - 0.01, (B, 1, H, W)).astype(np.float32)
            sy = rng.uniform(-0.99, H - 0.01, (B, 1, H, W)).astype(np.float32)
        sy, sx = sy.astype(dt), sx.astype(dt)
        out, valid, coll = oracle.forward_warping(obj, sy, sx, depth)
        if dt == np.float32:
            lo, lv, lc = oracle.forward_warping_lexmin(obj, sy, sx, depth)
            assert np.array_equal(lo, out) and np.array_equal(lv, valid) and np.array_equal(lc, coll), name
        cases.update({f"{name}/obj": obj, f"{name}/safe_y": sy, f"{name}/safe_x": sx, f"{name}/depth": depth,
                      f"{name}/output": out, f"{name}/valid": valid, f"{name}/collision": coll})
    return cases


def make_wrapper_cases(ref_fw):
    """Drive the reference FW.forward (3-D inputs, as preprocess.py does)."""
    rng = np.random.default_rng(99)
    fw = ref_fw.FW("cpu")
    cases = {}
    specs = [
        ("f32_c6", 6, 24, 32, torch.float32, 6.0),
        ("f32_c2_big", 2, 20, 28, torch.float32, 60.0),
        ("f64flow_c6", 6, 24, 32, torch.float64, 6.0),
        ("f64obj_c4", 4, 16, 24, torch.float64, 3.0),
    ]
    for name, C, H, W, fdt, scale in specs:
        obj = torch.from_numpy(rng.standard_normal((C, H, W))).to(torch.float64 if "f64obj" in name else torch.float32)
        flow = torch.from_numpy(rng.standard_normal((2, H, W)) * scale).to(fdt)
        depth = torch.from_numpy(rng.integers(1, 6, (1, H, W)).astype(np.float64)).to(fdt)
        out, valid, coll = fw(obj, flow, depth)
        cases.update({f"{name}/obj": obj.numpy(), f"{name}/flow": flow.numpy(), f"{name}/depth": depth.numpy(),
                      f"{name}/output": out.numpy(), f"{name}/valid": valid.numpy(), f"{name}/collision": coll.numpy()})
    # float64 flow within rounding of an integer: add done in float64 (fw.py:31)
    H, W = 4, 8
    flow = torch.zeros(2, H, W, dtype=torch.float64)
    flow[0] = 0.99999999
    flow[1, 1] = -0.99999999
    flow[1, 2] = 1.0 - 1e-9
    obj = torch.arange(3 * H * W, dtype=torch.float32).reshape(3, H, W)
    depth = torch.ones(1, H, W, dtype=torch.float64)
    out, valid, coll = fw(obj, flow, depth)
    cases.update({"nearint_f64/obj": obj.numpy(), "nearint_f64/flow": flow.numpy(),
                  "nearint_f64/depth": depth.numpy(), "nearint_f64/output": out.numpy(),
                  "nearint_f64/valid": valid.numpy(), "nearint_f64/collision": coll.numpy()})
    return cases


def make_pipeline_cases(ref_fw, Plausible, Convert, utils_mod):
    """preprocess.py:348-359 / :372-374 first-stage calls on synthetic depth."""
    fw = ref_fw.FW("cpu")
    cases = {}
    for k, (h, w) in enumerate([(48, 64), (60, 80)]):
        seed = 12345 + k
        depth_np = synth_depth(h, w, seed)
        rgb = torch.from_numpy(synth_rgb(h, w, seed))
        # (a) disparity flow, depth float64 as utils.get_depth returns it (utils.py:47-59)
        utils_mod.set_seed(seed)
        d0 = utils_mod.normalize_depth(torch.from_numpy(depth_np.copy()).unsqueeze(0))
        disp0 = Convert.depth_to_disparity(d0)
        flow01 = Convert.disparity_to_flow(disp0, device="cpu", random_sign=False)
        img0_all = torch.cat((rgb, d0, flow01 * -1.0), axis=0)       # preprocess.py:358
        o, v, c = fw(img0_all, flow01, d0)                            # preprocess.py:359
        # (b) ego-motion flow on float32 depth (preprocess.py:372, 385)
        utils_mod.set_seed(seed + 7)
        d0f = d0.to(torch.float32)
        flow03, T1 = Convert.depth_to_random_flow(d0f, "cpu")
        img0_all3 = torch.cat((rgb, d0f, flow03 * -1.0), axis=0)      # preprocess.py:386
        o3, v3, c3 = fw(img0_all3, flow03, d0f)                       # preprocess.py:387
        fixed = utils_mod.fix_warped_depth((o3[3:4] * v3).clone())    # preprocess.py:391,394
        p = f"img{k}"
        cases.update({
            f"{p}/raw_depth": depth_np, f"{p}/rgb": rgb.numpy(), f"{p}/seed": np.array(seed),
            f"{p}/norm_depth": d0.numpy(), f"{p}/flow01": flow01.numpy(),
            f"{p}/fw01_output": o.numpy(), f"{p}/fw01_valid": v.numpy(), f"{p}/fw01_collision": c.numpy(),
            f"{p}/T1": T1.numpy(), f"{p}/flow03": flow03.numpy(),
            f"{p}/fw03_output": o3.numpy(), f"{p}/fw03_valid": v3.numpy(), f"{p}/fw03_collision": c3.numpy(),
            f"{p}/fw03_fixed_depth": fixed.numpy(),
        })
    # Plausible.K and a batch of camera parameters drawn from the reference RNG
    K, invK = Plausible.K((768, 1024))
    cases["K_768x1024"] = K.numpy()
    cases["invK_768x1024"] = invK.numpy()
    Ts, ss = [], []
    for i in range(8):
        utils_mod.set_seed(12345 + i)
        s = utils_mod.get_random(0.3, 0.8, random_sign=False)
        T, _, _ = Plausible.random_motion(1. / 36., 1. / 36., 0.1, 0.1)
        ss.append(float(s))
        Ts.append(T.numpy()[0])
    cases["camera_seeds"] = np.arange(12345, 12353)
    cases["camera_s"] = np.array(ss, np.float32)
    cases["camera_T"] = np.stack(Ts)
    return cases


def load_reference_preprocess_slices(utils_mod, ref_fw, Convert):
    """SpecialFlow + augment_flow (:24-182), ConcatFlow + BackFlow (:301-326) and
    PreprocessPlusAugment through its group save (:329-450), as text slices."""
    import torch.nn as nn
    lines = open(os.path.join(REF, "preprocess.py")).read().split("\n")
    ns = dict(torch=torch, nn=nn, np=np, os=os, sys=sys, time=__import__("time"), math=math,
              utils=utils_mod, FW=ref_fw.FW, Convert=Convert, device="cpu")
    for a, b in ((301, 326), (24, 182), (329, 450)):
        exec(compile("\n".join(lines[a - 1:b]), os.path.join(REF, "preprocess.py"), "exec"), ns)
    return ns


def make_augment_cases(ns, utils_mod):
    """augment_flow per type, ConcatFlow / BackFlow, and the first stage's group tensor."""
    import tempfile
    cases = {}
    h, w = 40, 56
    raw = synth_depth(h, w, 4242)
    d64 = utils_mod.normalize_depth(torch.from_numpy(raw.copy()).unsqueeze(0))        # float64, as get_depth
    img0 = torch.from_numpy(synth_rgb(h, w, 4242))
    utils_mod.set_seed(4242)
    flow01 = ns["Convert"].disparity_to_flow(ns["Convert"].depth_to_disparity(d64), device="cpu", random_sign=False)
    fw = ns["FW"]("cpu")
    o, v, c = fw(torch.cat((img0, d64, flow01 * -1.0), 0), flow01, d64)
    img1, d1, back01 = o[0:3] * v, utils_mod.fix_warped_depth(o[3:4] * v), o[4:6] * v
    base = {"img0": img0, "d0": d64, "img1": img1, "d1": d1, "flow01": flow01, "back01": back01}
    for k, t in base.items():
        cases[f"in/{k}"] = t.numpy()
    for kind in (0, 1, 2, 5, 6, 7):
        seed = 777 + kind
        utils_mod.set_seed(seed)
        set1, set2, typ, spec = ns["augment_flow"](img0, d64, img1, d1, flow01, back01, device="cpu",
                                                     augment_flow_type=kind)
        cases[f"aug{kind}/seed"] = np.array(seed)
        cases[f"aug{kind}/type"] = np.array(typ)
        for n, t in enumerate(set1):
            cases[f"aug{kind}/set1_{n}"] = t.numpy()
        for n, t in enumerate(set2):
            cases[f"aug{kind}/set2_{n}"] = t.numpy()
        if spec is not None:
            cases[f"aug{kind}/special"] = spec[0].numpy()
            cases[f"aug{kind}/back_special"] = spec[1].numpy()
    # ConcatFlow / BackFlow on the disparity pair and a float32 rotation-like flow
    cf, bf = ns["ConcatFlow"]("cpu"), ns["BackFlow"]("cpu")
    yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    fBC = torch.stack((0.05 * (yy - h / 2), -0.04 * (xx - w / 2)), 0)
    cfo, cfv = cf(flow01, back01, fBC, d1)
    bfo, bfv = bf(fBC, d1.to(torch.float32))
    cases.update({"cf/flowBC": fBC.numpy(), "cf/out": cfo.numpy(), "cf/valid": cfv.numpy(),
                  "bf/out": bfo.numpy(), "bf/valid": bfv.numpy()})
    # PreprocessPlusAugment first stage (7 FW calls, 5 hole-fills, ConcatFlow) -> group.npz
    ppa = ns["PreprocessPlusAugment"]("cpu")
    with tempfile.TemporaryDirectory() as td:
        utils_mod.set_seed(12399)
        ppa((img0, torch.from_numpy(raw.copy()).unsqueeze(0)), os.path.join(td, "img"), False)
        g = np.load(os.path.join(td, "img", "group.npz"))["img_depth_flow"]
    cases["ppa/seed"] = np.array(12399)
    cases["ppa/raw_depth"] = raw
    cases["ppa/group"] = g
    return cases


def make_inpaint_mask_cases(ref_inpaint, rec):
    """utils.inpaint's mask algebra and casts on FW outputs and on masks with collisions."""
    pl = np.load(os.path.join(HERE, "pipeline.npz"))
    rng = np.random.default_rng(99)
    inputs = []
    for k in range(2):  # realistic: the warped RGB and masks of pipeline.npz
        for tag in ("fw01", "fw03"):
            o = pl[f"img{k}/{tag}_output"]
            v, c = pl[f"img{k}/{tag}_valid"], pl[f"img{k}/{tag}_collision"]
            inputs.append((o[0:3] * v, v, c))
    for h, w in ((17, 23), (32, 40)):  # synthetic: collisions, isolated pixels, non-integer values
        v = (rng.random((1, h, w)) < 0.7).astype(np.float32)
        c = ((rng.random((1, h, w)) < 0.3) & (v > 0)).astype(np.float32)
        img = (rng.uniform(-20, 300, (3, h, w))).astype(np.float32)
        inputs.append((img, v, c))
    cases = {}
    for n, (img, v, c) in enumerate(inputs):
        rec.calls.clear()
        got = ref_inpaint(torch.from_numpy(np.ascontiguousarray(img)).as_subclass(_CpuImage),
                          torch.from_numpy(v), torch.from_numpy(c))
        got = got.as_subclass(torch.Tensor)
        (img_u8, mask, radius, flags), = rec.calls
        assert radius == 3 and flags == _Cv2Recorder.INPAINT_TELEA
        assert got.dtype == torch.float32 and tuple(got.shape) == img.shape
        cases.update({f"c{n}/img": img, f"c{n}/valid": v, f"c{n}/collision": c,
                      f"c{n}/img_u8_hwc": img_u8, f"c{n}/mask": mask, f"c{n}/returned": got.numpy()})
    cases["n"] = np.array(len(inputs))
    return cases


def _digest(a) -> str:
    import hashlib
    a = np.ascontiguousarray(a)
    return f"{a.dtype.str}{tuple(a.shape)}:" + hashlib.sha256(a.tobytes()).hexdigest()


def make_config1_cases(ref_fw, Convert, utils_mod):
    """BASELINE config 1: one 480x640 synthetic depth map (seed
    0) through the reference's normalize_depth (utils.py:102-116), its
    disparity flow (preprocess.py:239-254, s drawn after utils.set_seed(12345))
    and ego-motion flow (:265-298 with geometry.py, the next draws), each
    warped by the reference's fw.py (oracle as fw_cuda) with the :358 / :386
    obj.  Full planes at this size would be megabytes, so the fixture holds a
    SHA-256 digest of every array plus a strided sample of its values (for
    readable failures) and the scalar draws."""
    h, w = 480, 640
    fw = ref_fw.FW("cpu")
    raw = synth_depth(h, w, 0)
    rgb = torch.from_numpy(synth_rgb(h, w, 0))
    utils_mod.set_seed(12345)
    d0 = utils_mod.normalize_depth(torch.from_numpy(raw.copy()).unsqueeze(0))   # float64 (utils.get_depth)
    flow01 = Convert.disparity_to_flow(Convert.depth_to_disparity(d0), device="cpu", random_sign=False)
    o1, v1, c1 = fw(torch.cat((rgb, d0, flow01 * -1.0), 0), flow01, d0)          # preprocess.py:358-359
    d0f = d0.to(torch.float32)
    flow03, T1 = Convert.depth_to_random_flow(d0f, "cpu")                         # preprocess.py:372 / :385
    o3, v3, c3 = fw(torch.cat((rgb, d0f, flow03 * -1.0), 0), flow03, d0f)        # preprocess.py:386-387
    arrays = {"raw_depth": raw, "rgb": rgb.numpy(), "norm_depth": d0.numpy(), "flow01": flow01.numpy(),
              "fw01_output": o1.numpy(), "fw01_valid": v1.numpy(), "fw01_collision": c1.numpy(),
              "flow03": flow03.numpy(), "fw03_output": o3.numpy(), "fw03_valid": v3.numpy(),
              "fw03_collision": c3.numpy()}
    cases = {"T1": T1.numpy()}
    for k, a in arrays.items():
        cases[f"digest/{k}"] = np.array(_digest(a))
        cases[f"sample/{k}"] = np.ascontiguousarray(a).reshape(-1)[::97].copy()
    return cases


def make_ppa_forward_cases(utils_mod, ref_fw, Convert):
    """The whole of PreprocessPlusAugment.forward for one small image: the
    reference's text slices preprocess.py:24-182 (SpecialFlow, augment_flow),
    :301-326 (ConcatFlow, BackFlow) and :329-476 (forward through the last
    augment save) exec'd with the oracle as fw_cuda and the recording cv2
    (its inpaint returns the uint8 cast unchanged).  The slice needs one
    repair: :463 leaves its parenthesis open (the SyntaxError that makes the
    file unparseable); the generator closes it.  Every
    file forward writes -- group.npz and the 120 {g}_{a}_{1,2}.npz -- is
    stored (16 x 24 pixels keeps the fixture small)."""
    import tempfile
    import torch.nn as nn
    lines = open(os.path.join(REF, "preprocess.py")).read().split("\n")
    assert lines[462].rstrip().endswith("axis=0"), lines[462]
    body = lines[328:476]
    body[462 - 328] = lines[462] + ")"  # the missing parenthesis of :463
    ns = dict(torch=torch, nn=nn, np=np, os=os, sys=sys, time=__import__("time"), math=math,
              utils=utils_mod, FW=ref_fw.FW, Convert=Convert, device="cpu")
    for a, b in ((301, 326), (24, 182)):
        exec(compile("\n".join(lines[a - 1:b]), os.path.join(REF, "preprocess.py"), "exec"), ns)
    exec(compile("\n".join(body), os.path.join(REF, "preprocess.py"), "exec"), ns)
    h, w, seed = 16, 24, 4711
    raw = synth_depth(h, w, seed)
    img0 = torch.from_numpy(synth_rgb(h, w, seed))
    ppa = ns["PreprocessPlusAugment"]("cpu")
    cases = {"seed": np.array(seed), "raw_depth": raw, "img0": img0.numpy()}
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "img")
        utils_mod.set_seed(seed)
        ppa((img0, torch.from_numpy(raw.copy()).unsqueeze(0)), out, False)
        cases["group"] = np.load(os.path.join(out, "group.npz"))["img_depth_flow"]
        for g in range(5):
            for a in range(12):
                for k in (1, 2):
                    z = np.load(os.path.join(out, f"{g}_{a}_{k}.npz"))
                    cases[f"aug/{g}_{a}_{k}"] = z["img_depth_flow"]
                    cases[f"type/{g}_{a}_{k}"] = z["augment_flow_type"]
        assert len(os.listdir(out)) == 121
    return cases


# the flows of files that pass through geometry evaluated on the device: the
# group's ego-motion flows and the flows composed from them (channels 28:44),
# every augmentation of groups 1-4 (their flowAB / back_flowAB are those
# flows, copied or composed) and the rotation augmentations (type 6) of every
# group; everything else must match bit for bit (tests/test_preprocess.py)
FILL_TOL_GROUP_CH = tuple(range(28, 44))


def _tol_channels(key, kind):
    if key == "group":
        return FILL_TOL_GROUP_CH
    if kind != 6 and key.startswith("0_"):
        return ()
    return (4, 5, 6, 7) if key.endswith("_1") else (0, 1, 2, 3)


def _rotation_base(rot, c0, h, w):
    """numpy evaluation of SpecialFlow._rotate's flow, (p0 - c0) @ rot + c0 -
    p0 (preprocess.py:63-77), in float32 with the 2-term product rounded as a
    GEMM accumulates it: the k = 0 product, then a fused multiply-add of the
    k = 1 term (emulated in float64: the product is exact there, the sum
    rounds once before the float32 rounding).  The base that
    ppa_fill_large.npz's rotation flows are stored against; the pixels where
    the reference's matmul differs from it (none were found) are stored as
    patches.  tests/test_preprocess.py restates it."""
    x = np.broadcast_to(np.arange(w, dtype=np.float32)[None, :], (h, w))
    y = np.broadcast_to(np.arange(h, dtype=np.float32)[:, None], (h, w))
    dx, dy = (x - c0[0]).astype(np.float32), (y - c0[1]).astype(np.float32)
    px = (dy.astype(np.float64) * np.float64(rot[1, 0]) + (dx * rot[0, 0]).astype(np.float64)).astype(np.float32)
    py = (dy.astype(np.float64) * np.float64(rot[1, 1]) + (dx * rot[0, 1]).astype(np.float64)).astype(np.float32)
    return np.stack(((px + c0[0]) - x, (py + c0[1]) - y)).astype(np.float32)


def make_ppa_fill_cases(utils_mod, ref_fw, Convert, h=32, w=40, seeds=(5150, 5151), sample=(5, 7), tol_full=True,
                        store_flows=False):
    """PreprocessPlusAugment.forward (:329-476) of two 32x40 images with the
    real hole-fill: the reference's text slices run with utils.inpaint backed
    by _Cv2Telea (cv2's sequential Telea, restated by the oracle), the oracle
    as fw_cuda.  Every file forward writes is pinned per channel: a SHA-256
    digest of the channel (bit-exact bar), plus the float32 values of the
    channels held to the 1e-5 px geometry tolerance, and a strided sample of
    every channel for readable failures.  ``holes`` counts the pixels each
    image's 95 fills actually filled (the fill is not idle).

    ``tol_full=False`` (the larger-image fixture, ppa_fill_large.npz) keeps
    the tolerance channels as a strided sample plus their sum and absolute
    sum instead of whole planes, so the fixture stays a few MB.

    ``store_flows`` (ppa_fill_large.npz) also stores every device-geometry
    flow the reference drew, exactly: the two ego-motion flows (flow12 of
    :372, flow03 of :385, whole planes) and each rotation's special / back
    special flow (:31-41, :63-77) as its rotation matrices and centre plus the
    pixels where the reference's CPU matmul differs from the float32 numpy
    base (_rotation_base).  tests/test_preprocess.py feeds them to the product
    in place of its device geometry: everything downstream must then be bit
    for bit the reference's (the causal check of the target-index flips)."""
    import tempfile
    import torch.nn as nn
    lines = open(os.path.join(REF, "preprocess.py")).read().split("\n")
    assert lines[462].rstrip().endswith("axis=0"), lines[462]
    body = lines[328:476]
    body[462 - 328] = lines[462] + ")"  # the missing parenthesis of :463
    ns = dict(torch=torch, nn=nn, np=np, os=os, sys=sys, time=__import__("time"), math=math,
              utils=utils_mod, FW=ref_fw.FW, Convert=Convert, device="cpu")
    for a, b in ((301, 326), (24, 182)):
        exec(compile("\n".join(lines[a - 1:b]), os.path.join(REF, "preprocess.py"), "exec"), ns)
    exec(compile("\n".join(body), os.path.join(REF, "preprocess.py"), "exec"), ns)
    cases = {"h": np.array(h), "w": np.array(w), "sample_stride": np.array(sample)}
    ref_inpaint, tel = load_reference_inpaint(_Cv2Telea)
    utils_mod.inpaint = lambda img, valid, coll: ref_inpaint(img.as_subclass(_CpuImage), valid, coll).as_subclass(
        torch.Tensor)
    cases["seeds"] = np.array(seeds)
    cap = {"ego": [], "rot": []}
    if store_flows:
        d2rf = Convert.depth_to_random_flow
        SF = ns["SpecialFlow"]
        sf_fwd, sf_rot = SF.forward, SF._rotate

        def cap_d2rf(*a, **k):
            r = d2rf(*a, **k)
            cap["ego"].append(r[0].detach().clone())
            return r

        def cap_rotate(self, size):
            # the matrices _rotate builds, rebuilt from its own draws: wrap
            # utils.get_random for the call to see c0 and theta
            draws = []
            gr = utils_mod.get_random

            def rec(*a, **k):
                v = gr(*a, **k)
                draws.append(v)
                return v
            ns_utils = ns["utils"]
            ns_utils.get_random = rec
            try:
                p1, p_prev = sf_rot(self, size)
            finally:
                ns_utils.get_random = gr
            hh, ww = size
            c0 = torch.tensor((draws[0] + ww / 2, draws[1] + hh / 2)).to(torch.float32)
            theta = torch.deg2rad(draws[2])
            rot = torch.tensor([[torch.cos(theta), -torch.sin(theta)], [torch.sin(theta), torch.cos(theta)]]
                               ).type(torch.float32)
            rrot = torch.tensor([[torch.cos(-theta), -torch.sin(-theta)], [torch.sin(-theta), torch.cos(-theta)]]
                                ).type(torch.float32)
            cap["rot"].append({"c0": c0.numpy(), "rot": rot.numpy(), "rrot": rrot.numpy()})
            return p1, p_prev

        def cap_fwd(self, size, kind):
            r = sf_fwd(self, size, kind)
            if 6. <= kind < 7.:
                cap["rot"][-1]["flows"] = (r[0].detach().numpy().copy(), r[1].detach().numpy().copy())
            return r
        Convert.depth_to_random_flow = staticmethod(cap_d2rf)
        SF._rotate, SF.forward = cap_rotate, cap_fwd
    for n, seed in enumerate(seeds):
        raw = synth_depth(h, w, seed)
        img0 = torch.from_numpy(synth_rgb(h, w, seed))
        cases[f"i{n}/raw_depth"] = raw
        cases[f"i{n}/img0"] = img0.numpy()
        ppa = ns["PreprocessPlusAugment"]("cpu")
        tel.calls.clear()
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "img")
            utils_mod.set_seed(seed)
            ppa((img0, torch.from_numpy(raw.copy()).unsqueeze(0)), out, False)
            assert len(os.listdir(out)) == 121
            files = {"group": (np.load(os.path.join(out, "group.npz"))["img_depth_flow"], None)}
            for g in range(5):
                for a in range(12):
                    for k in (1, 2):
                        z = np.load(os.path.join(out, f"{g}_{a}_{k}.npz"))
                        files[f"{g}_{a}_{k}"] = (z["img_depth_flow"], int(z["augment_flow_type"]))
        cases[f"i{n}/holes"] = np.array([c[0] for c in tel.calls], np.int64)
        if store_flows:
            # the reference draws flow12 (:372) before flow03 (:385)
            assert len(cap["ego"]) == 2 and len(cap["rot"]) == 15, (len(cap["ego"]), len(cap["rot"]))
            cases[f"i{n}/ref_flow12"] = cap["ego"][0].numpy().astype(np.float32)
            cases[f"i{n}/ref_flow03"] = cap["ego"][1].numpy().astype(np.float32)
            for r, rc in enumerate(cap["rot"]):
                pre = f"i{n}/rot{r}"
                cases[pre + "/c0"], cases[pre + "/rot"], cases[pre + "/rrot"] = rc["c0"], rc["rot"], rc["rrot"]
                for nm, m, flow in (("sf", rc["rot"], rc["flows"][0]), ("bsf", rc["rrot"], rc["flows"][1])):
                    base = _rotation_base(m, rc["c0"], h, w)
                    assert flow.dtype == np.float32 and flow.shape == base.shape
                    idx = np.flatnonzero(base.view(np.uint32) != flow.view(np.uint32)).astype(np.int32)
                    cases[f"{pre}/{nm}_idx"] = idx
                    cases[f"{pre}/{nm}_val"] = flow.reshape(-1)[idx]
            cap["ego"].clear()
            cap["rot"].clear()
        for key, (arr, kind) in files.items():
            pre = f"i{n}/{key}"
            cases[pre + "/dtype"] = np.array(arr.dtype.str)
            cases[pre + "/shape"] = np.array(arr.shape)
            if kind is not None:
                cases[pre + "/type"] = np.array(kind)
            cases[pre + "/digest"] = np.array([_digest(arr[c]) for c in range(arr.shape[0])])
            cases[pre + "/sample"] = np.ascontiguousarray(arr[:, ::sample[0], ::sample[1]]).astype(np.float32)
            for c in _tol_channels(key, kind):
                if tol_full:
                    cases[f"{pre}/tol{c}"] = arr[c].astype(np.float32)
                else:
                    cases[f"{pre}/tolsum{c}"] = np.array([arr[c].astype(np.float64).sum(),
                                                         np.abs(arr[c].astype(np.float64)).sum()])
    if store_flows:
        Convert.depth_to_random_flow = staticmethod(d2rf)
        SF._rotate, SF.forward = sf_rot, sf_fwd
    return cases


def make_loss_cases():
    """The two training losses the on-the-fly step restates, run as the
    reference has them: adjusted_RAFT/train.py's sequence_loss (taken by AST
    with its MAX_FLOW; the module imports the RAFT network) and
    adjusted_gmflow/loss.py's flow_loss_func (imported as is), on seeded
    predictions, ground truth with some |flow| >= 400 and a ragged valid mask."""
    src = open(os.path.join(REF, "adjusted_RAFT", "train.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if (isinstance(n, ast.Assign) and any(getattr(t, "id", "") == "MAX_FLOW"
                                                                       for t in n.targets))
            or (isinstance(n, ast.FunctionDef) and n.name == "sequence_loss")]
    ns = {"torch": torch}
    exec(compile(ast.Module(body=body, type_ignores=[]), os.path.join(REF, "adjusted_RAFT", "train.py"), "exec"), ns)
    spec = importlib.util.spec_from_file_location("ref_gmflow_loss", os.path.join(REF, "adjusted_gmflow", "loss.py"))
    gml = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gml)
    g = torch.Generator().manual_seed(7)
    cases = {}
    for n_pred, key in ((4, "raft"), (2, "gmflow")):
        gt = torch.randn(2, 2, 12, 16, generator=g) * 60.0
        gt[0, 0, :2, :3] = 450.0  # |flow| >= max_flow: excluded
        preds = [gt + torch.randn(2, 2, 12, 16, generator=g) * (3.0 / (i + 1)) for i in range(n_pred)]
        valid = (torch.rand(2, 12, 16, generator=g) > 0.2).float()
        if key == "raft":
            loss, m = ns["sequence_loss"](preds, gt, valid)
        else:
            loss, m = gml.flow_loss_func(preds, gt, valid)
        cases[f"{key}/gt"] = gt.numpy()
        cases[f"{key}/preds"] = torch.stack(preds).numpy()
        cases[f"{key}/valid"] = valid.numpy()
        cases[f"{key}/loss"] = np.float32(float(loss))
        for k in ("epe", "1px", "3px", "5px"):
            cases[f"{key}/{k}"] = np.float64(m[k])
    return cases


def main():
    if sys.argv[1:] == ["losses"]:  # only the training-loss fixture
        lc = make_loss_cases()
        np.savez_compressed(os.path.join(OUT, "losses.npz"), **lc)
        print("losses.npz", os.path.getsize(os.path.join(OUT, "losses.npz")), "bytes")
        return
    ref_fw = load_reference_fw()
    geometry_mod = load_reference_geometry()
    utils_mod = load_reference_utils_subset()
    Plausible, Convert = load_reference_plausible_convert(utils_mod, geometry_mod)

    if sys.argv[1:] == ["config1"]:  # only the config-1 fixture (the others are unchanged)
        c1 = make_config1_cases(ref_fw, Convert, utils_mod)
        np.savez_compressed(os.path.join(OUT, "config1.npz"), **c1)
        print("config1.npz", os.path.getsize(os.path.join(OUT, "config1.npz")), "bytes")
        return
    if sys.argv[1:] == ["ppa_fill"]:  # only the forward fixture with the real (oracle-Telea) fill
        pf = make_ppa_fill_cases(utils_mod, ref_fw, Convert)
        np.savez_compressed(os.path.join(OUT, "ppa_fill.npz"), **pf)
        print("ppa_fill.npz", os.path.getsize(os.path.join(OUT, "ppa_fill.npz")), "bytes")
        return
    if sys.argv[1:] == ["ppa_fill_large"]:  # one 192x256 image: ego-motion border bands, larger fills
        pf = make_ppa_fill_cases(utils_mod, ref_fw, Convert, h=192, w=256, seeds=(5160,), sample=(8, 8),
                                 tol_full=False, store_flows=True)
        np.savez_compressed(os.path.join(OUT, "ppa_fill_large.npz"), **pf)
        print("ppa_fill_large.npz", os.path.getsize(os.path.join(OUT, "ppa_fill_large.npz")), "bytes")
        return
    if sys.argv[1:] == ["ppa_forward"]:  # only the per-image forward fixture
        ref_inpaint, rec = load_reference_inpaint()
        utils_mod.inpaint = lambda img, valid, coll: ref_inpaint(img.as_subclass(_CpuImage), valid, coll).as_subclass(
            torch.Tensor)
        pf = make_ppa_forward_cases(utils_mod, ref_fw, Convert)
        np.savez_compressed(os.path.join(OUT, "ppa_forward.npz"), **pf)
        print("ppa_forward.npz", os.path.getsize(os.path.join(OUT, "ppa_forward.npz")), "bytes")
        return
    op = make_op_cases()
    np.savez_compressed(os.path.join(OUT, "fw_op.npz"), **op)
    wr = make_wrapper_cases(ref_fw)
    np.savez_compressed(os.path.join(OUT, "fw_wrapper.npz"), **wr)
    pl = make_pipeline_cases(ref_fw, Plausible, Convert, utils_mod)
    np.savez_compressed(os.path.join(OUT, "pipeline.npz"), **pl)
    ref_inpaint, rec = load_reference_inpaint()
    im = make_inpaint_mask_cases(ref_inpaint, rec)
    np.savez_compressed(os.path.join(OUT, "inpaint_mask.npz"), **im)
    # utils with inpaint = the reference's, behind the CPU-device shim
    utils_mod.inpaint = lambda img, valid, coll: ref_inpaint(img.as_subclass(_CpuImage), valid, coll).as_subclass(
        torch.Tensor)
    ns = load_reference_preprocess_slices(utils_mod, ref_fw, Convert)
    au = make_augment_cases(ns, utils_mod)
    np.savez_compressed(os.path.join(OUT, "augment.npz"), **au)
    for f in ("fw_op.npz", "fw_wrapper.npz", "pipeline.npz", "inpaint_mask.npz", "augment.npz"):
        print(f, os.path.getsize(os.path.join(OUT, f)), "bytes")


if __name__ == "__main__":
    main()
