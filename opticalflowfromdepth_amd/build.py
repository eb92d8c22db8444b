"""In-tree build of the native forward-warp library for gfx950.

``python -m opticalflowfromdepth_amd.build`` or ``build_native()`` compiles
csrc/ofd_fw.hip (forward warp), csrc/ofd_inpaint.hip (layered hole-fill) and
csrc/ofd_inpaint_seq.hip (the default hole-fill, cv2's sequential Telea order)
and csrc/ofd_deflate.hip (the npz product's GPU deflate) with hipcc into
``_build/libofd_fw.so`` (C ABI, include/ofd_fw.h, ofd_inpaint.h, ofd_deflate.h).
The .so is git-ignored but travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
SRCS = [os.path.join(_HERE, "csrc", f) for f in ("ofd_fw.hip", "ofd_inpaint.hip", "ofd_inpaint_seq.hip",
                                                  "ofd_deflate.hip")]
HDRS = [os.path.join(REPO, "include", f) for f in ("ofd_fw.h", "ofd_inpaint.h", "ofd_deflate.h")] + [
    os.path.join(_HERE, "csrc", "ip_common.h")]
OUT_DIR = os.path.join(_HERE, "_build")
OUT = os.path.join(OUT_DIR, "libofd_fw.so")
ARCH = os.environ.get("OFD_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found (set HIPCC or install ROCm)")


ID_FILE = OUT + ".id"


def compile_flags() -> list:
    """hipcc's flags for the library, without the compiler path, the output
    name and the build id.  -ffp-contract=off: the hole-fill's float / double
    sequence must be the oracle's bit for bit (the warp has no contractible
    arithmetic)."""
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
            "-I", "include"]


def source_hash() -> str:
    """The build id: first 16 hex digits of the SHA-256 over every source
    the library is compiled from (name and bytes, in a fixed order) and the
    compile flags (target arch included), so a flag or arch change yields a
    new id and a rebuild.  The library embeds it (ofd_fw_build_id) and a
    sidecar file records it, so a binary can be tied to the sources -- i.e.
    the commit -- it came from."""
    import hashlib
    h = hashlib.sha256()
    h.update(" ".join(compile_flags()).encode() + b"\0")
    for p in SRCS + HDRS:
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def built_id() -> str | None:
    """The build id the in-tree library was built with (its sidecar), or None."""
    try:
        with open(ID_FILE) as f:
            return f.read().strip() or None
    except OSError:
        return None


def needs_build() -> bool:
    """True unless the in-tree library exists and was built from the current
    sources (content hash, not mtimes: a copied tree keeps its verdict)."""
    return not os.path.exists(OUT) or built_id() != source_hash()


def build_native(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = OUT + f".tmp{os.getpid()}"
    bid = source_hash()
    flags = [os.path.join(REPO, "include") if f == "include" else f for f in compile_flags()]
    cmd = [hipcc()] + flags + [f'-DOFD_BUILD_ID="{bid}"', "-o", tmp] + SRCS
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)  # atomic: concurrent builders never expose a half-written .so
    with open(ID_FILE + f".tmp{os.getpid()}", "w") as f:
        f.write(bid + "\n")
    os.replace(ID_FILE + f".tmp{os.getpid()}", ID_FILE)
    build_c_host()
    return OUT


HOST_SRC = os.path.join(REPO, "tests", "c_host", "ofd_host.c")
HOST_OUT = os.path.join(OUT_DIR, "ofd_host")


def build_c_host() -> str:
    """tests/c_host/ofd_host.c: the C ABI driven from plain C (gcc, libamdhip64), for tests/test_c_host.py."""
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = HOST_OUT + f".tmp{os.getpid()}"
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(REPO, "include"),
                    "-I", os.path.join(rocm, "include"), "-o", tmp, HOST_SRC, "-L", OUT_DIR, "-lofd_fw",
                    "-L", os.path.join(rocm, "lib"), "-lamdhip64", f"-Wl,-rpath,{OUT_DIR}",
                    f"-Wl,-rpath,{os.path.join(rocm, 'lib')}", "-Wl,-rpath,$ORIGIN"], check=True)
    os.replace(tmp, HOST_OUT)
    return HOST_OUT


if __name__ == "__main__":
    print(build_native(force="--force" in sys.argv, verbose=True))
