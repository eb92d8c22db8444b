"""The C ABI from a plain C host (tests/c_host/ofd_host.c, built by
opticalflowfromdepth_amd.build with gcc against libofd_fw.so and
libamdhip64): no Python and no torch on the product side -- the shape of a
cgo / JNI / C++ integration.  The C program warps a batch
(ofd_fw_forward_warp_flow_f32) and fills the warped RGB in cv2's order
(ofd_inpaint_telea_seq_f32); both are checked bit-exactly against the oracle."""
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import oracle

HOST = os.path.join(REPO, "opticalflowfromdepth_amd", "_build", "ofd_host")


def test_c_host_is_built():
    """The C host links against the library and the HIP runtime (gcc, no GPU needed)."""
    from opticalflowfromdepth_amd import build
    build.build_native()  # no-op when up to date
    if not os.access(HOST, os.X_OK):
        build.build_c_host()
    assert os.access(HOST, os.X_OK)


@pytest.mark.gpu
def test_c_host_warp_and_fill_match_oracle(tmp_path):
    from opticalflowfromdepth_amd import synth
    obj, flow, depth = synth.stage_one_batch([12345, 12377], 96, 128, "cpu")
    obj, flow, depth = (t.contiguous().numpy().astype(np.float32) for t in (obj, flow, depth))
    B, C, H, W = obj.shape
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(src, "wb") as f:
        np.array([B, C, H, W], np.int64).tofile(f)
        for a in (obj, flow, depth):
            a.tofile(f)
    r = subprocess.run([HOST, str(src), str(dst)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(dst, np.float32)
    n_o, n_m, n_f = B * C * H * W, B * H * W, B * 3 * H * W
    out = got[:n_o].reshape(B, C, H, W)
    valid = got[n_o:n_o + n_m].reshape(B, 1, H, W)
    coll = got[n_o + n_m:n_o + 2 * n_m].reshape(B, 1, H, W)
    filled = got[n_o + 2 * n_m:n_o + 2 * n_m + n_f].reshape(B, 3, H, W)
    e_out, e_valid, e_coll = oracle.fw_flow(obj, flow, depth)
    assert np.array_equal(out, e_out) and np.array_equal(valid, e_valid) and np.array_equal(coll, e_coll)
    rgb = out[:, :3] * valid
    assert np.array_equal(filled, oracle.inpaint(rgb, valid, coll, 3, layered=False))
    assert (valid == 0).mean() > 0.01  # there were holes to fill
