"""npz files deflated on the GPU: the product writer of preprocess.py:446, :471-476.

np.savez_compressed writes a zip of .npy members, each deflated by host zlib:
at 768x1024 that is ~6.3 GB of float64 planes per image, and one host core
per file bounds the pipeline (~0.3 images/s on the lease's 16 cores).
GpuNpzWriter deflates the arrays where they are (include/ofd_deflate.h:
dynamic-Huffman literal blocks, RFC 1951) and only assembles the zip on the
host:

* member ``<key>.npy`` = the .npy header (deflated by host zlib, closed by a
  sync flush so it ends on a byte boundary) followed by the GPU's stream of
  the array's bytes (which ends the deflate stream);
* its CRC-32 is the header's combined with the GPU's (zlib's crc32_combine);
* small extra members (``augment_flow_type``) are written by zlib as usual.

The files are ordinary zips that np.load / zipfile read and CRC-check; the
arrays come back bit for bit.  The compressed bytes differ from zlib's (no
LZ77 matches: ~2.3x on these planes against zlib level 6's ~2.9x).
"""
from __future__ import annotations

import contextlib
import io
import os
import struct
import threading
import zlib
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _native

_POLY = 0xEDB88320


# ---------------------------------------------------------------- CRC-32 combine (zlib's multmodp / x2nmodp)
def _multmodp(a: int, b: int) -> int:
    m, p = 1 << 31, 0
    while True:
        if a & m:
            p ^= b
            if (a & (m - 1)) == 0:
                break
        m >>= 1
        b = (b >> 1) ^ _POLY if b & 1 else b >> 1
    return p


_shift_cache: Dict[int, int] = {}


def _x8nmodp(n: int) -> int:
    """x^(8n) mod P: the operator that moves a CRC past n more bytes (cached per n)."""
    v = _shift_cache.get(n)
    if v is None:
        p, sq, k = 1 << 31, 1 << 23, n
        while k:
            if k & 1:
                p = _multmodp(sq, p)
            sq = _multmodp(sq, sq)
            k >>= 1
        _shift_cache[n] = v = p
    return v


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """zlib.crc32(A + B) from zlib.crc32(A), zlib.crc32(B) and len(B)."""
    return _multmodp(_x8nmodp(len2), crc1) ^ crc2


# ---------------------------------------------------------------- zip container
def npy_header(shape, dtype) -> bytes:
    """The .npy header np.save writes for a C-contiguous array of this shape and dtype."""
    f = io.BytesIO()
    np.lib.format.write_array_header_1_0(
        f, {"descr": np.lib.format.dtype_to_descr(np.dtype(dtype)), "fortran_order": False, "shape": tuple(shape)})
    return f.getvalue()


def _raw_deflate(data: bytes, level: int, final: bool) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    return c.compress(data) + c.flush(zlib.Z_FINISH if final else zlib.Z_SYNC_FLUSH)


class _Member:
    __slots__ = ("name", "crc", "usize", "parts")

    def __init__(self, name, crc, usize, parts):
        self.name, self.crc, self.usize, self.parts = name, crc, usize, parts


def member_from_gpu_stream(key: str, shape, dtype, stream: memoryview, crc_data: int, nbytes: int,
                           level: int = 6) -> _Member:
    """``<key>.npy``: the host-deflated .npy header, then the GPU stream of the data."""
    hdr = npy_header(shape, dtype)
    crc = crc32_combine(zlib.crc32(hdr), crc_data, nbytes)
    return _Member(key + ".npy", crc, len(hdr) + nbytes, [_raw_deflate(hdr, level, final=False), stream])


def member_from_array(key: str, value, level: int = 6) -> _Member:
    f = io.BytesIO()
    np.lib.format.write_array(f, np.asanyarray(value), allow_pickle=False)
    raw = f.getvalue()
    return _Member(key + ".npy", zlib.crc32(raw), len(raw), [_raw_deflate(raw, level, final=True)])


@contextlib.contextmanager
def atomic_path(path: str):
    """A temporary name beside ``path``, renamed onto it (os.replace) only
    once the body has written it completely: an interrupted run leaves no
    truncated product file for ``--skip-existing`` to count as done."""
    tmp = f"{path}.tmp{os.getpid()}.{threading.get_ident()}"
    try:
        yield tmp
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except FileNotFoundError:
            pass
        raise


def zip_complete(path: str) -> bool:
    """The file ends with a zip end-of-central-directory record (22 bytes, no
    comment: every writer here and np.savez_compressed end so), i.e. its
    writer finished it."""
    try:
        with open(path, "rb") as f:
            f.seek(0, os.SEEK_END)
            if f.tell() < 22:
                return False
            f.seek(-22, os.SEEK_END)
            return f.read(4) == b"PK\x05\x06"
    except OSError:
        return False


def write_zip(path: str, members: Sequence[_Member]) -> int:
    """A zip (deflate method) of the members, as zipfile writes one; returns
    the bytes written.  Written under a temporary name and renamed."""
    with atomic_path(path) as tmp:
        return _write_zip(tmp, members)


def _write_zip(path: str, members: Sequence[_Member]) -> int:
    with open(path, "wb") as f:
        central = []
        for m in members:
            name = m.name.encode()
            csize = sum(len(p) for p in m.parts)
            if csize >= 0xFFFFFFFF or m.usize >= 0xFFFFFFFF:
                raise ValueError("member of 4 GiB or more: zip64 is not written by this writer")
            off = f.tell()
            f.write(struct.pack("<IHHHHHIIIHH", 0x04034B50, 20, 0, 8, 0, 0x21, m.crc, csize, m.usize, len(name), 0))
            f.write(name)
            for p in m.parts:
                f.write(p)
            central.append(struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 20, 20, 0, 8, 0, 0x21, m.crc, csize,
                                       m.usize, len(name), 0, 0, 0, 0, 0, off) + name)
        cd_off = f.tell()
        for c in central:
            f.write(c)
        cd_size = f.tell() - cd_off
        f.write(struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, len(members), len(members), cd_size, cd_off, 0))
        return f.tell()


# ---------------------------------------------------------------- the writer
class GpuNpzWriter:
    """Drop-in for NpzWriter (preprocess.py's product files) with the arrays
    deflated on the GPU.  ``save_batch(paths, x, key, extra)`` writes one npz
    per leading index of the device tensor x (one ofd_deflate_batch call for
    all of them) and returns without waiting for the GPU: the stream sizes
    and CRCs go to pinned host memory behind an event; a pool thread waits
    for that event, copies the compressed streams to pinned memory on a side
    stream, and hands the zips to the other pool threads.  The caller's
    stream therefore keeps its queue full (augmentations already queued on
    it, or on side streams, keep running while earlier files deflate)."""

    def __init__(self, workers: int = 8, header_level: int = 6, max_pending_bytes: int = 8 << 30):
        self.pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="gnpz")
        # one fetch thread: waits for each batch's deflate, then for room under
        # max_pending_bytes, then copies the streams; it never occupies a
        # writer thread, so the writes that free room always make progress
        self.fetcher = ThreadPoolExecutor(max_workers=1, thread_name_prefix="gnpz-fetch")
        self.level = header_level
        self.cap = max_pending_bytes
        self.pending = 0
        self.cv = threading.Condition()
        self.futures = []
        self.bytes_written = 0       # compressed bytes on disk
        self.bytes_in = 0            # array bytes deflated
        self._ws = {}                # (device, stream) -> deflate workspace
        self._copy_streams = {}      # device -> side stream of the D2H copies
        self._lock = threading.Lock()

    def _workspace(self, dev, stream, nbytes):
        # keyed by (device, stream): two deflates in flight on different
        # streams never share scratch; calls on one stream are ordered by it
        k = (dev, stream.cuda_stream)
        with self._lock:
            ws = self._ws.get(k)
            if ws is None or ws.numel() < nbytes:
                ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=dev)
                self._ws[k] = ws
            return ws

    def _copy_stream(self, dev):
        with self._lock:
            s = self._copy_streams.get(dev)
            if s is None:
                s = self._copy_streams[dev] = torch.cuda.Stream(dev)
            return s

    def save_batch(self, paths: Sequence[str], x: torch.Tensor, key: str = "img_depth_flow",
                   extra: Optional[Dict[str, object]] = None) -> None:
        if not x.is_cuda:
            raise RuntimeError("GpuNpzWriter.save_batch expects a device tensor")
        x = x.detach().contiguous()
        count = x.shape[0]
        if len(paths) != count:
            raise ValueError(f"{len(paths)} paths for {count} arrays")
        if count == 0:
            return
        lib = _native.lib()
        each = int(x[0].numel() * x.element_size())
        bound = int(lib.ofd_deflate_bound(each))
        dev = x.device
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            out = torch.empty(count * bound, dtype=torch.uint8, device=dev)
            sizes = torch.empty(count, dtype=torch.int64, device=dev)
            crcs = torch.empty(count, dtype=torch.int32, device=dev)
            nws = int(lib.ofd_deflate_workspace_bytes(count, each))
            ws = self._workspace(dev, stream, nws) if nws else None
            rc = lib.ofd_deflate_batch(x.data_ptr(), count, each, out.data_ptr(), sizes.data_ptr(), crcs.data_ptr(),
                                       ws.data_ptr() if ws is not None else None, nws, stream.cuda_stream)
            _native.check(rc, "ofd_deflate_batch")
            sz_h = torch.empty(count, dtype=torch.int64, pin_memory=True)
            cr_h = torch.empty(count, dtype=torch.int32, pin_memory=True)
            sz_h.copy_(sizes, non_blocking=True)
            cr_h.copy_(crcs, non_blocking=True)
            ev_sizes = torch.cuda.Event()
            ev_sizes.record(stream)
            side = self._copy_stream(dev)
            out.record_stream(side)  # the D2H copies below read it on the side stream
        shape, dtype = tuple(x.shape[1:]), np.dtype(str(x.dtype).replace("torch.", ""))
        extra = dict(extra or {})
        self.bytes_in += each * count

        def write_one(host, i, off, n, crc):
            mv = memoryview(host.numpy())[off:off + n]
            mem = [member_from_gpu_stream(key, shape, dtype, mv, crc, each, self.level)]
            mem += [member_from_array(k, v, self.level) for k, v in extra.items()]
            return write_zip(paths[i], mem)

        def done(f, n):
            with self.cv:
                self.pending -= n
                if f.exception() is None:
                    self.bytes_written += f.result()
                self.cv.notify_all()

        def fetch():
            # runs on the fetch thread: only it waits for the deflate
            ev_sizes.synchronize()
            sz = sz_h.tolist()
            cr = [c & 0xFFFFFFFF for c in cr_h.tolist()]
            total = sum(sz)
            with self.cv:
                while self.pending > 0 and self.pending + total > self.cap:
                    self.cv.wait()
                self.pending += total
            handed = 0  # bytes whose write job owns their share of `pending`
            try:
                host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
                with torch.cuda.device(dev), torch.cuda.stream(side):
                    side.wait_event(ev_sizes)
                    o = 0
                    for i, n in enumerate(sz):  # the streams, back to back, one D2H each
                        host[o:o + n].copy_(out[i * bound:i * bound + n], non_blocking=True)
                        o += n
                    ev = torch.cuda.Event()
                    ev.record(side)
                ev.synchronize()
                o = 0
                for i, n in enumerate(sz):
                    fut = self.pool.submit(write_one, host, i, o, n, cr[i])
                    handed += n
                    fut.add_done_callback(lambda f, n=n: done(f, n))
                    with self._lock:
                        self.futures.append(fut)
                    o += n
            except BaseException:
                # give back the share no write job will release, so later
                # fetches and flush() never wait on it
                with self.cv:
                    self.pending -= total - handed
                    self.cv.notify_all()
                raise

        fut = self.fetcher.submit(fetch)
        with self._lock:
            self.futures.append(fut)

    def save(self, path: str, **arrays) -> None:
        """NpzWriter.save's interface: the first device array is deflated on the
        GPU, the others (small) by zlib."""
        dev_keys = [k for k, v in arrays.items() if isinstance(v, torch.Tensor) and v.is_cuda]
        if not dev_keys:
            raise RuntimeError("GpuNpzWriter.save needs a device array")
        k0 = dev_keys[0]
        extra = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in arrays.items() if k != k0}
        self.save_batch([path], arrays[k0].unsqueeze(0), k0, extra)

    def flush(self) -> None:
        """Wait for every pending file, then re-raise the first error.  A
        fetch job appends its files' jobs before it completes, so drain until
        no job is left; a failed job never stops the wait for the others."""
        first = None
        while True:
            with self._lock:
                futs, self.futures = self.futures, []
            if not futs:
                break
            for f in futs:
                try:
                    f.result()
                except BaseException as e:  # noqa: BLE001 - re-raised below
                    if first is None:
                        first = e
        if first is not None:
            raise first

    def close(self) -> None:
        self.flush()
        self.fetcher.shutdown()
        self.pool.shutdown()
