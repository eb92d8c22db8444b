"""CPU tests of the multi-GPU sharding path: gloo, world_size 2 (and 3)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opticalflowfromdepth_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,ws", [(512, 8), (64, 2), (10, 3), (5, 4), (1505, 7), (0, 2)])
def test_shard_range_partitions(n, ws):
    seen = []
    for r in range(ws):
        a, b = shard.shard_range(n, ws, r)
        assert 0 <= a <= b <= n
        seen.extend(range(a, b))
    assert seen == list(range(n))


def test_shard_range_matches_reference_formula():
    # preprocess.py:543-547 for a split the reference handles (no overrun)
    n, split = 1698, 8
    split_len = int((n + split - 1) // split)
    for sid in range(split):
        start, end = sid * split_len, (sid + 1) * split_len
        if sid == split - 1:
            end = n
        assert shard.shard_range(n, split, sid) == (start, end)


def test_image_seed():
    assert shard.image_seed(0) == 12345
    assert shard.image_seed(7, epoch=1, n_images=1505) == 12345 + 7 + 1505


def _worker(rank, ws, port, n_images, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        seeds = [shard.image_seed(i) for i in range(n_images)]
        s, T = shard.broadcast_camera_params(seeds, device="cpu")
        a, b = shard.shard_range(n_images, ws, rank)
        # the shard's inputs, built from broadcast params, on CPU
        obj, flow, depth = synth.stage_one_batch(seeds[a:b], 16, 24, "cpu", camera=(s[a:b], T[a:b]))
        t = torch.tensor([float(b - a)])
        dist.all_reduce(t)
        q.put((rank, s.numpy(), T.numpy(), (a, b), float(obj.sum()), float(t)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_broadcast_camera_params_gloo(ws):
    n = 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, n, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_s, ref_T = synth.batch_camera_params([shard.image_seed(i) for i in range(n)])
    ranges = sorted(r[3] for r in res)
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for rank, s, T, rng, osum, total in res:
        assert (s == ref_s.numpy()).all() and (T == ref_T.numpy()).all()  # bit-identical to the redraw
        assert total == n
        # sharded inputs equal the unsharded ones (per-image seeding)
        a, b = rng
        if b > a:
            obj, _, _ = synth.stage_one_batch([shard.image_seed(i) for i in range(a, b)], 16, 24, "cpu")
            assert abs(float(obj.sum()) - osum) < 1e-3 * max(1.0, abs(osum))
