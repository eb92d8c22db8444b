"""PreprocessPlusAugment.forward on the GPU vs tests/golden/ppa_forward.npz, per file and channel.

Runs forward with the fixture's hole-fill stand-in (the uint8 cast, see
tests/golden/make_golden.py make_ppa_forward_cases) and prints, for every one
of the 121 files, the channels that differ: count of differing pixels and the
max |diff|.  Diagnostic companion of tests/test_preprocess.py
test_forward_all_files_match_reference.

usage: python tools/ppa_forward_diff.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def cast_only(img, valid, coll):
    """The fixture's utils.inpaint with cv2.inpaint returning its input: float32(uint8(img))."""
    a = img.permute(0, 2, 3, 1).cpu().numpy().astype(np.uint8)
    return torch.from_numpy(a).to(img.device).permute(0, 3, 1, 2).to(torch.float32).contiguous()


def run_forward(z, device="cuda:0"):
    from opticalflowfromdepth_amd import preprocess as pp, utils
    ppa = pp.PreprocessPlusAugment(device, inpaint_fn=cast_only)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "img")
        utils.set_seed(int(z["seed"]))
        ppa((torch.from_numpy(z["img0"]), torch.from_numpy(z["raw_depth"].copy()).unsqueeze(0)), d, False)
        names = sorted(os.listdir(d))
        for n in names:
            f = np.load(os.path.join(d, n))
            out[n[:-4]] = {k: f[k] for k in f.files}
    return out


def main():
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "ppa_forward.npz"))
    got = run_forward(z)
    print("files written:", len(got))
    g = got["group"]["img_depth_flow"]
    e = z["group"]
    for c in range(44):
        n = int((g[c] != e[c]).sum())
        if n:
            print(f"group ch {c:2d}: {n:4d} px differ, max |diff| {np.abs(g[c] - e[c]).max():.4g}")
    for gi in range(5):
        for a in range(12):
            for k in (1, 2):
                key = f"{gi}_{a}_{k}"
                x = got[key]
                assert int(x["augment_flow_type"]) == int(z[f"type/{key}"]), key
                g, e = x["img_depth_flow"], z[f"aug/{key}"]
                bad = [(c, int((g[c] != e[c]).sum()), float(np.abs(g[c] - e[c]).max())) for c in range(8)
                       if (g[c] != e[c]).any()]
                if bad:
                    print(f"{key} type {int(x['augment_flow_type'])}: " +
                          " ".join(f"c{c}:{n}/{m:.3g}" for c, n, m in bad))


if __name__ == "__main__":
    main()
