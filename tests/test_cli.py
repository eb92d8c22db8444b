"""The product CLI, ``python -m opticalflowfromdepth_amd.preprocess`` (the
reference's ``__main__``, preprocess.py:508-561).

Bar: sharding never changes a product file.  Two runs on one card with
``--split 2 --split_id 0 / 1`` write, between them, exactly the files of one
``--split 1`` run, every array ``np.load``-equal (the reference's per-image
seed 12345 + img_idx + epoch * N, :555, makes each image independent of its
shard).  The same holds for two ranks under torch.distributed.run, where the
camera parameters reach rank 1 through the broadcast from rank 0
(shard.broadcast_camera_params; gloo here, both ranks on cuda:0).  The files
are written by the default GPU deflate writer; a resumed run skips complete
images.  CPU tests cover the file inventory and the writer choice.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from opticalflowfromdepth_amd import preprocess as pp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--n-images", "3", "--height", "32", "--width", "48", "--epochs", "1", "--batch", "2"]


def _files(root):
    out = {}
    for d, _, fs in os.walk(root):
        for f in fs:
            p = os.path.join(d, f)
            out[os.path.relpath(p, root)] = p
    return out


def _assert_same_tree(a, b):
    fa, fb = _files(a), _files(b)
    assert sorted(fa) == sorted(fb)
    for k in fa:
        za, zb = np.load(fa[k], allow_pickle=False), np.load(fb[k], allow_pickle=False)
        assert sorted(za.files) == sorted(zb.files), k
        for m in za.files:
            x, y = za[m], zb[m]
            assert x.dtype == y.dtype and x.shape == y.shape, (k, m)
            assert np.array_equal(x.reshape(-1).view(np.uint8), y.reshape(-1).view(np.uint8)), (k, m)


def test_file_inventory_matches_reference_layout(tmp_path):
    # preprocess.py:446 (group.npz) and :471-476 ({g}_{a}_{1,2}.npz, 5 groups x 12 augments)
    assert pp.N_FILES_PER_IMAGE == 121
    d = tmp_path / "7"
    d.mkdir()
    assert not pp.image_complete(str(d))
    pp.savez_compressed(str(d / "group.npz"), img_depth_flow=np.zeros((44, 2, 3), np.float32))
    assert pp.image_complete(str(d), augment=False)
    assert not pp.image_complete(str(d))
    for g in range(pp.N_GROUPS):
        for a in range(len(pp.AUGMENT_SCHEDULE)):
            for k in (1, 2):
                pp.write_npz(str(d / f"{g}_{a}_{k}.npz"), 1, img_depth_flow=np.ones((8, 2, 3)),
                             augment_flow_type=np.array(a))
    assert pp.image_complete(str(d))
    assert sorted(os.listdir(d)) == sorted(["group.npz"] + [f"{g}_{a}_{k}.npz" for g in range(pp.N_GROUPS)
                                                            for a in range(len(pp.AUGMENT_SCHEDULE)) for k in (1, 2)])
    # a truncated file (a writer killed mid-write before the atomic rename existed)
    # or an empty one makes the image incomplete, so --skip-existing redoes it
    f = d / "3_5_2.npz"
    data = f.read_bytes()
    f.write_bytes(data[:-30])
    assert not pp.image_complete(str(d))
    f.write_bytes(b"")
    assert not pp.image_complete(str(d))
    f.write_bytes(data)
    assert pp.image_complete(str(d))


def test_writers_never_leave_a_partial_file(tmp_path):
    from opticalflowfromdepth_amd import npz_gpu
    path = tmp_path / "x.npz"
    # a write that fails midway leaves neither the file nor its temporary
    with pytest.raises(RuntimeError):
        with npz_gpu.atomic_path(str(path)) as tmp:
            open(tmp, "wb").write(b"PK partial")
            raise RuntimeError("killed")
    assert os.listdir(tmp_path) == []

    class Boom:  # np.lib.format.write_array raises on it after the zip is opened
        def __array__(self, *a, **k):
            raise RuntimeError("array failed")
    with pytest.raises(RuntimeError):
        pp.write_npz(str(path), 1, img_depth_flow=Boom())
    assert os.listdir(tmp_path) == []
    # the zip writer of the GPU writer: a complete file under the final name only
    m = npz_gpu.member_from_array("a", np.arange(10))
    n = npz_gpu.write_zip(str(path), [m])
    assert os.listdir(tmp_path) == ["x.npz"] and os.path.getsize(path) == n and npz_gpu.zip_complete(str(path))
    assert np.array_equal(np.load(path)["a"], np.arange(10))


def test_writer_choice():
    assert pp.make_writer("sync") is None
    w = pp.make_writer("zlib")
    assert isinstance(w, pp.NpzWriter) and w.level == 6
    w.close()
    with pytest.raises(ValueError):
        pp.make_writer("lz4")


@pytest.mark.gpu
def test_split_runs_union_equals_one_run(tmp_path, cuda_device):
    split = str(tmp_path / "split")
    one = str(tmp_path / "one")
    r0 = pp.main(SMALL + ["--split", "2", "--split_id", "0", "--out", split])
    r1 = pp.main(SMALL + ["--split", "2", "--split_id", "1", "--out", split])
    r = pp.main(SMALL + ["--split", "1", "--split_id", "0", "--out", one])
    assert (r0["shard"], r1["shard"], r["shard"]) == ([0, 2], [2, 3], [0, 3])
    assert r0["images"] + r1["images"] == r["images"] == 3
    assert r["files"] == 3 * 121 and len(_files(one)) == 3 * 121
    assert r["writer"] == "gpu"
    _assert_same_tree(split, one)
    # resume: every image is complete, nothing is recomputed
    again = pp.main(SMALL + ["--split", "1", "--split_id", "0", "--out", one, "--skip-existing"])
    assert again["images"] == 0 and again["skipped"] == 3


@pytest.mark.gpu
def test_gpu_writer_equals_sync_writer(tmp_path, cuda_device):
    a, b = str(tmp_path / "gpu"), str(tmp_path / "sync")
    args = ["--n-images", "1", "--height", "24", "--width", "32", "--epochs", "1"]
    pp.main(args + ["--out", a, "--writer", "gpu"])
    pp.main(args + ["--out", b, "--writer", "sync"])
    _assert_same_tree(a, b)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_two_ranks_under_torchrun_equal_one_run(tmp_path, cuda_device):
    """Two ranks (gloo, both on cuda:0): --split / --split_id from the world
    size / rank, (s, T) from rank 0's broadcast."""
    ranks = str(tmp_path / "ranks")
    one = str(tmp_path / "one")
    env = dict(os.environ, OFD_PPA_BACKEND="gloo", PYTHONPATH=REPO)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "opticalflowfromdepth_amd.preprocess",
           *SMALL, "--gpu", "0", "--out", ranks]
    res = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 2
    pp.main(SMALL + ["--split", "1", "--split_id", "0", "--out", one])
    _assert_same_tree(ranks, one)
