"""Device geometry vs the reference's own runs (diagnostic, GPU only).

Counts the float32 elements where the product's device flows differ from the
reference's (tests/golden/pipeline.npz flow03, ppa_fill_large.npz flow03 and
the rotation special flows), and how many of the 968 channels of the
192x256 pipeline run differ from the reference's (digests).
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def rot_base(rot, c0, h, w):
    x = np.broadcast_to(np.arange(w, dtype=np.float32)[None, :], (h, w))
    y = np.broadcast_to(np.arange(h, dtype=np.float32)[:, None], (h, w))
    dx, dy = x - c0[0], y - c0[1]
    px = (dx * rot[0, 0] + dy * rot[1, 0]) + c0[0]
    py = (dx * rot[0, 1] + dy * rot[1, 1]) + c0[1]
    return np.stack((px - x, py - y)).astype(np.float32)


def main():
    from opticalflowfromdepth_amd import ego_flow, ops, synth, preprocess as pp, utils
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(REPO, "tests", "golden", "pipeline.npz"))
    for img in ("img0", "img1"):
        d = torch.from_numpy(g[f"{img}/norm_depth"]).float()[None]
        h, w = d.shape[-2:]
        P, ik = synth.projection(h, w, torch.from_numpy(g[f"{img}/T1"]), dev)
        got = ego_flow(d.to(dev), P, ik)[0].cpu().numpy()
        print(f"pipeline.npz {img} flow03: {(got != g[f'{img}/flow03']).sum()} of {got.size} differ")
    z = np.load(os.path.join(REPO, "tests", "golden", "ppa_fill_large.npz"))
    h, w = int(z["h"]), int(z["w"])
    seed = int(z["seeds"][0])
    s, T = synth.camera_params(seed)
    d0 = synth.normalize_depth(torch.from_numpy(z["i0/raw_depth"].copy())[None, None])
    P, ik = synth.projection(h, w, T[None], dev)
    got = ego_flow(d0.to(dev), P, ik)[0].cpu().numpy()
    print(f"ppa_fill_large flow03: {(got != z['i0/ref_flow03']).sum()} of {got.size} differ")
    for r in range(15):
        pre = f"i0/rot{r}"
        prm = torch.from_numpy(np.concatenate([z[pre + "/c0"], z[pre + "/rot"].reshape(-1), z[pre + "/rrot"].reshape(-1)]))
        f, b = ops.rotation_flow(prm[None], h, w, dev)
        nd = 0
        for nm, m, out in (("sf", "rot", f), ("bsf", "rrot", b)):
            ref = rot_base(z[pre + "/" + m], z[pre + "/c0"], h, w).reshape(-1)
            ref[z[f"{pre}/{nm}_idx"]] = z[f"{pre}/{nm}_val"]
            nd += int((out[0].cpu().numpy().reshape(-1) != ref).sum())
        print(f"rotation {r}: {nd} differ")
    import tempfile
    import test_preprocess as tp
    with tempfile.TemporaryDirectory() as td:
        ppa = pp.PreprocessPlusAugment("cuda:0")
        out = os.path.join(td, "img")
        utils.set_seed(seed)
        ppa((torch.from_numpy(z["i0/img0"]), torch.from_numpy(z["i0/raw_depth"].copy()).unsqueeze(0)), out, False)
        torch.cuda.synchronize()
        bad = []
        for key in ["group"] + [f"{g_}_{a}_{k}" for g_ in range(5) for a in range(12) for k in (1, 2)]:
            arr = np.load(os.path.join(out, key + ".npz"))["img_depth_flow"]
            dig = z[f"i0/{key}/digest"]
            for c in range(arr.shape[0]):
                if tp._digest(arr[c]) != str(dig[c]):
                    bad.append(f"{key}:{c}")
        print(f"192x256 pipeline: {len(bad)} of 968 channels differ: {bad[:40]}")


if __name__ == "__main__":
    main()
