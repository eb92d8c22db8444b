"""Image-shard partitioning across GPUs for the preprocess batch loop.

The reference shards its dataset loop by hand across processes with
``--split/--split_id`` (preprocess.py:511-515, :543-547): contiguous ranges of
``ceil(N / split)`` images, the last shard taking the remainder, and a
per-image seed ``12345 + img_idx + epoch * N`` (:555) so results do not depend
on the sharding.  Here one process per GPU (torch.distributed, RCCL = backend
"nccl" on ROCm) plays the role of one ``split_id``.

Every image is independent, so the data path has no collective.  The only
communication is one broadcast of the per-image camera parameters (scale s and
ego-motion T1, 17 floats per image) from rank 0 over RCCL/xGMI per batch --
optional, because every rank could redraw them from the seeds (the broadcast
result is bit-identical to the redraw; tests/test_shard.py checks that).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch
import torch.distributed as dist

from . import synth


def shard_range(n_items: int, world_size: int, rank: int) -> Tuple[int, int]:
    """[start, end) of ``rank``'s contiguous shard (preprocess.py:543-547).

    Differs from the reference only where the reference would index past the
    end (a rank whose ceil-sized range starts beyond N): such a shard is empty.
    """
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world size {world_size}")
    split_len = (n_items + world_size - 1) // world_size
    start = min(rank * split_len, n_items)
    end = min((rank + 1) * split_len, n_items)
    if rank == world_size - 1:
        end = n_items
    return start, max(start, end)


def image_seed(img_idx: int, epoch: int = 0, n_images: int = 0, base: int = 12345) -> int:
    """preprocess.py:555: 12345 + img_idx + epoch * len(dataset)."""
    return base + img_idx + epoch * n_images


def pack_camera(s: torch.Tensor, T: torch.Tensor) -> torch.Tensor:
    """(s [N], T [N,4,4]) -> [N,17] float32."""
    return torch.cat([s.view(-1, 1).to(torch.float32), T.reshape(-1, 16).to(torch.float32)], 1)


def unpack_camera(p: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    return p[:, 0].contiguous(), p[:, 1:].reshape(-1, 4, 4).contiguous()


def broadcast_camera_params(seeds: Sequence[int], device=None, group=None, src: int = 0
                            ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rank ``src`` draws (s, T) for all ``seeds``; one broadcast hands them to
    every rank.  ``device`` is where the broadcast buffer lives (a GPU for
    RCCL, CPU for gloo).  Returns CPU tensors (s [N], T [N,4,4])."""
    n = len(seeds)
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return synth.batch_camera_params(seeds)
    buf = torch.empty(n, 17, dtype=torch.float32, device=device)
    if dist.get_rank(group) == src:
        s, T = synth.batch_camera_params(seeds)
        buf.copy_(pack_camera(s, T))
    dist.broadcast(buf, src=src, group=group)
    return unpack_camera(buf.cpu())
