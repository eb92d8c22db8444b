"""bench.py's N-rank launch, on CPU: ``python bench.py --gpus 2``
with no torchrun environment starts 2 ranks itself (a torch.distributed.run
child), and exactly one JSON line -- rank 0's, with n_gpus = 2 -- reaches
stdout.  --dry-run swaps the GPU work for a CPU no-op and RCCL for gloo; the
launcher, the shard split, the camera broadcast, the barrier-bracketed timing
and the max over ranks are the product code."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_n_ranks(n):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--dry-run",
                        "--steps", "3", "--warmup", "1", "--batch", "4"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["dry_run"] is True and rec["steps"] == 3
    assert rec["shard_images"] == [0, 4]  # rank 0's contiguous shard of 4 * n images
    # what the process group itself saw: its size, its backend, every rank's own time
    ranks = rec["ranks"]
    assert ranks["world_size"] == n and ranks["backend"] == "gloo"
    assert len(ranks["ms_per_step"]) == n and all(t >= 0 for t in ranks["ms_per_step"])
    # every rank exited cleanly after the final barrier (rank 0 sleeps before it)
    assert "Traceback" not in r.stderr


def test_bench_single_rank_does_not_relaunch():
    from bench import parse
    a = parse(["--gpus", "1"])
    assert a.gpus == 1 and a.steps == 50 and a.warmup == 5
