"""Per-hole chain anatomy of the hole-fill layer launches (diagnostic, GPU only).

Runs tools/probe_ip.hip (the product hole-fill TU with OFD_IP_STAMPS) on the
headline batch's warped RGB and prints, for sampled layers, the shader-clock
cycles thread 0 of the first block of each path spends between: kernel entry,
list entry read, patch loaded, colour computed, stores done.
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from opticalflowfromdepth_amd import forward_warp_flow, synth  # noqa: E402

SO = os.path.join(REPO, "tools", "_build", "libprobe_ip.so")


def main():
    dev = torch.device("cuda:0")
    B, H, W = int(os.environ.get("B", "64")), 768, 1024
    obj, flow, depth = synth.stage_one_batch([12345 + i for i in range(B)], H, W, dev)
    out, valid, coll = forward_warp_flow(obj, flow, depth)
    rgb = (out[:, 0:3] * valid).contiguous()
    lib = ctypes.CDLL(SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.ofd_inpaint_workspace_bytes.argtypes = [I64] * 3
    lib.ofd_inpaint_workspace_bytes.restype = ctypes.c_size_t
    lib.ofd_inpaint_telea_f32.argtypes = [P] * 4 + [I64] * 4 + [ctypes.c_int, P, ctypes.c_size_t, P]
    lib.probe_ip_set_stamps.argtypes = [P]
    ws = torch.empty(lib.ofd_inpaint_workspace_bytes(B, H, W), dtype=torch.uint8, device=dev)
    res = torch.empty_like(rgb)
    st = torch.cuda.current_stream().cuda_stream
    nL = H + W + 8
    stamps = torch.zeros(2 * nL * 8, dtype=torch.int64, device=dev)

    def call():
        rc = lib.ofd_inpaint_telea_f32(rgb.data_ptr(), valid.data_ptr(), coll.data_ptr(), res.data_ptr(), B, 3, H, W,
                                       3, ws.data_ptr(), ws.numel(), st)
        assert rc == 0, rc

    lib.probe_ip_set_stamps(None)
    call()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    call()
    b.record()
    torch.cuda.synchronize()
    print(f"unstamped call {a.elapsed_time(b):.3f} ms")
    assert lib.probe_ip_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
    a.record()
    call()
    b.record()
    torch.cuda.synchronize()
    print(f"stamped call {a.elapsed_time(b):.3f} ms")
    lib.probe_ip_set_stamps(None)
    s = stamps.view(nL, 2, 8).cpu().numpy().astype(np.int64)
    names = ["list", "patch", "compute", "store"]
    for path, pn in ((0, "interior thread"), (1, "border wave")):
        rows = []
        for L in range(1, nL):
            r = s[L, path]
            if r[0] == 0 or r[4] == 0:
                continue
            d = [r[k + 1] - r[k] if r[k + 1] and r[k] else -1 for k in range(4)]
            rows.append((L, d, r[4] - r[0]))
        print(f"{pn}: {len(rows)} layers stamped")
        if not rows:
            continue
        tot = np.array([t for _, _, t in rows])
        ds = np.array([d for _, d, _ in rows])
        print("   median cycles: " + "  ".join(f"{n}={np.median(ds[:, k]):.0f}" for k, n in enumerate(names)) +
              f"  entry->done={np.median(tot):.0f}")
        for L, d, t in rows[:4] + rows[len(rows) // 2:len(rows) // 2 + 2] + rows[-3:]:
            print(f"   L={L:4d} " + "  ".join(f"{n}={v:6d}" for n, v in zip(names, d)) + f"  total={t}")


if __name__ == "__main__":
    main()
