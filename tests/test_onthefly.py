"""On-the-fly bf16 warp inside a RAFT-style DDP train step (SURVEY.md 8(d)
config 5, 8(f) rank 4; opticalflowfromdepth_amd/onthefly.py, following
adjusted_RAFT/train.py:184-211) and a GMFlow-style one
(adjusted_gmflow/main.py:450-494).  Both losses are pinned by the reference's
own functions (tests/golden/losses.npz).

CPU: the pair builder with the oracle's ops, and DDP over gloo at world size 2
(two processes, each on its shard) against one process stepping the union of
the two shards -- the gradient all-reduce must make the ranks identical and
equal to the single-process step.
GPU: the HIP pair builder (bf16 warp, device ego flow, hole-fill) against the
oracle ops, a gloo world-2 DDP run on the card, and a loss that falls.
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from opticalflowfromdepth_amd import onthefly as otf

H, W = 48, 72  # a multiple of 4 like 368x560 (the network's 1/4 encoder)


def _cpu_ops():
    """PairOps with CPU restatements (test infrastructure): the oracle's warp
    (bf16 obj warped as float32 then rounded back: exact, every value came
    from a bf16), synth's ego flow, and the fixtures' cast-only hole-fill."""
    from oracle import torch_cpu
    from opticalflowfromdepth_amd import synth

    def warp(obj, flow, depth):
        o, v, c = torch_cpu.fw_flow_scatter(obj.float(), flow, depth)
        return o.to(obj.dtype), v, c

    def fill(img, valid, coll):
        return torch.floor(img).clamp(0, 255)  # integer-valued images: the uint8 cast

    return otf.PairOps(warp=warp, ego_flow=lambda d, T: synth.ego_motion_flow(d, T), fill=fill)


def _batches(rank, world, per_rank, steps):
    it = iter(otf.shard_loader(per_rank * world * steps, H, W, per_rank, rank, world))
    return [next(it) for _ in range(steps)]


def _run(rank, world, per_rank, steps, out, port, device="cpu", ops=None):
    import torch.distributed as dist
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = otf.IterativeFlowNet(dim=16).to(device)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model)
    opt, sched = otf.fetch_optimizer(model, num_steps=steps)
    args = otf.StepArgs(iters=3, amp=False)
    ops = ops or _cpu_ops()
    losses = []
    for b in _batches(rank, world, per_rank, steps) if world > 1 else _union(per_rank, steps):
        loss, m = otf.train_step(model, opt, sched, b, device, args, ops)
        losses.append(float(loss))
    sd = {k: v.detach().cpu() for k, v in (model.module if world > 1 else model).state_dict().items()}
    torch.save({"params": sd, "losses": losses}, out)
    if world > 1:
        dist.destroy_process_group()


def _union(per_rank, steps, world=2):
    """The single-process equivalent: step i sees every rank's step-i batch."""
    shards = [_batches(r, world, per_rank, steps) for r in range(world)]
    return [[torch.cat([shards[r][i][k] for r in range(world)]) for k in range(5)] for i in range(steps)]


def _spawn_target(rank, world, per_rank, steps, outdir, port, device):
    ops = _cpu_ops() if device == "cpu" else otf.PairOps()
    _run(rank, world, per_rank, steps, os.path.join(outdir, f"r{rank}.pt"), port, device, ops)


# ---------------------------------------------------------------- CPU
def test_make_pairs_cpu_ops():
    b = _batches(0, 1, 4, 1)[0]
    assert b[4].tolist() == [0, 1, 0, 1]  # disparity and ego-motion images
    img1, img2, flow, valid = otf.make_pairs(*b, ops=_cpu_ops())
    assert img1.dtype == img2.dtype == torch.bfloat16 and flow.dtype == torch.float32
    assert torch.equal(img1.float(), b[0])  # integer values are exact in bf16
    # adjusted_RAFT/core/datasets.py:282-288: |flow| < 1000 per component and img1_depth != 100
    from opticalflowfromdepth_amd import synth
    depth = synth.normalize_depth(b[1].to(torch.float32))
    exp_valid = (flow[:, 0].abs() < 1000) & (flow[:, 1].abs() < 1000) & (depth[:, 0] != 100)
    assert torch.equal(valid.bool(), exp_valid) and 0 < valid.mean() < 1
    # disparity images: horizontal flow only (preprocess.py:251-254)
    assert torch.all(flow[0::2, 1] == 0) and torch.all(flow[0::2, 0] < 0)
    # a source pixel that won its target shows up in image2 there
    from oracle import torch_cpu
    from opticalflowfromdepth_amd import synth
    d = synth.normalize_depth(b[1])
    o, v, c = torch_cpu.fw_flow_scatter(b[0], flow, d)
    won = (v > 0).expand_as(o)
    assert torch.equal(img2.float()[won], o[won])


def test_sequence_loss_follows_reference():
    """adjusted_RAFT/train.py:51-76 on a hand-sized case."""
    gt = torch.zeros(1, 2, 2, 2)
    gt[0, 0, 0, 0] = 500.0  # beyond MAX_FLOW: excluded
    preds = [torch.ones(1, 2, 2, 2), torch.full((1, 2, 2, 2), 2.0)]
    valid = torch.tensor([[[1.0, 1.0], [0.0, 1.0]]])
    loss, m = otf.sequence_loss(preds, gt, valid, gamma=0.5)
    keep = torch.tensor([[[0.0, 1.0], [0.0, 1.0]]])
    exp = 0.5 * (keep[:, None] * 1.0).expand(1, 2, 2, 2).mean() + 1.0 * (keep[:, None] * 2.0).expand(1, 2, 2, 2).mean()
    assert torch.isclose(loss, exp)
    assert torch.isclose(m["epe"], torch.tensor(2.0 * 2 ** 0.5))


def _loss_fixture(key):
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "losses.npz"))
    preds = [torch.from_numpy(p) for p in z[f"{key}/preds"]]
    return preds, torch.from_numpy(z[f"{key}/gt"]), torch.from_numpy(z[f"{key}/valid"]), z


@pytest.mark.parametrize("key", ["raft", "gmflow"])
def test_losses_match_reference_fixture(key):
    """sequence_loss (adjusted_RAFT/train.py:51-76) and flow_loss_func
    (adjusted_gmflow/loss.py:4-37) against the reference's own functions run
    on the same tensors (tests/golden/make_golden.py losses)."""
    preds, gt, valid, z = _loss_fixture(key)
    fn = otf.sequence_loss if key == "raft" else otf.flow_loss_func
    loss, m = fn(preds, gt, valid)
    assert float(loss) == pytest.approx(float(z[f"{key}/loss"]), rel=1e-6)
    for k in ("epe", "1px", "3px", "5px"):
        assert float(m[k]) == pytest.approx(float(z[f"{key}/{k}"]), rel=1e-6, abs=1e-12), k


def _run_gm(steps, per_rank, device, ops, model_dim=16):
    torch.manual_seed(0)
    model = otf.GlobalMatchFlowNet(dim=model_dim).to(device)
    opt, sched = otf.fetch_gmflow_optimizer(model, num_steps=steps)
    args = otf.StepArgs(gamma=0.9, amp=False)
    out = []
    for b in _batches(0, 1, per_rank, steps):
        r = otf.gmflow_train_step(model, opt, sched, b, device, args, ops)
        out.append(r)
    return model, opt, sched, out


def test_gmflow_step_cpu_ops():
    """adjusted_gmflow/main.py:450-494 on on-the-fly pairs: two predictions
    per step (matching, refined), the OneCycle schedule advances once per
    step, every parameter moves."""
    torch.manual_seed(0)
    init = otf.GlobalMatchFlowNet(dim=16).state_dict()
    model, opt, sched, out = _run_gm(2, 2, "cpu", _cpu_ops())
    assert all(r is not None and np.isfinite(float(r[0])) for r in out)
    assert sched.last_epoch == 2
    for k, v in model.state_dict().items():
        assert not torch.equal(v, init[k]), k
    b = _batches(0, 1, 2, 1)[0]
    r = model(b[0], b[0])
    assert set(r) == {"flow_preds"} and len(r["flow_preds"]) == 2 and r["flow_preds"][0].shape == (2, 2, H, W)


def test_gmflow_step_skips_nan_loss():
    """main.py:479-480: a NaN loss skips the step -- no update, no scheduler step."""
    torch.manual_seed(0)
    model = otf.GlobalMatchFlowNet(dim=16)
    opt, sched = otf.fetch_gmflow_optimizer(model, num_steps=4)
    before = {k: v.clone() for k, v in model.state_dict().items()}
    nan_ops = otf.PairOps(warp=_cpu_ops().warp, ego_flow=lambda d, T: torch.full_like(d.expand(-1, 2, -1, -1),
                                                                                       float("nan")),
                          fill=_cpu_ops().fill)
    b = _batches(0, 1, 2, 1)[0]
    b[4][:] = 1  # ego-motion images only: every flow is NaN
    r = otf.gmflow_train_step(model, opt, sched, b, "cpu", otf.StepArgs(gamma=0.9, amp=False), nan_ops)
    assert r is None and sched.last_epoch == 0
    for k, v in model.state_dict().items():
        assert torch.equal(v, before[k]), k


def _nan_skip_target(rank, world, outdir, port):
    """Rank 1's first batch makes a NaN loss, rank 0's does not: under DDP both
    must skip that step together, then both take the next one."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.parallel.DistributedDataParallel(otf.GlobalMatchFlowNet(dim=16))
    opt, sched = otf.fetch_gmflow_optimizer(model, num_steps=4)
    nan_ops = otf.PairOps(warp=_cpu_ops().warp,
                          ego_flow=lambda d, T: torch.full_like(d.expand(-1, 2, -1, -1), float("nan")),
                          fill=_cpu_ops().fill)
    bs = _batches(rank, world, 2, 2)
    if rank == 1:
        bs[0][4][:] = 1  # ego-motion images only: every flow is NaN
    r1 = otf.gmflow_train_step(model, opt, sched, bs[0], "cpu", otf.StepArgs(gamma=0.9, amp=False),
                               nan_ops if rank == 1 else _cpu_ops())
    r2 = otf.gmflow_train_step(model, opt, sched, bs[1], "cpu", otf.StepArgs(gamma=0.9, amp=False), _cpu_ops())
    sd = {k: v.detach().cpu() for k, v in model.module.state_dict().items()}
    torch.save({"params": sd, "first": r1 is None, "second": r2 is not None, "epoch": sched.last_epoch},
               os.path.join(outdir, f"nan{rank}.pt"))
    dist.destroy_process_group()


def test_gmflow_nan_skip_is_collective_under_ddp(tmp_path):
    mp.spawn(_nan_skip_target, args=(2, str(tmp_path), 29737), nprocs=2, join=True)
    r0, r1 = (torch.load(tmp_path / f"nan{r}.pt", weights_only=True) for r in range(2))
    assert r0["first"] and r1["first"]          # both skipped the step rank 1's NaN poisoned
    assert r0["second"] and r1["second"]        # and both took the next one
    assert r0["epoch"] == r1["epoch"] == 1
    for k in r0["params"]:
        assert torch.equal(r0["params"][k], r1["params"][k]), k


def test_ddp_gloo_world2_matches_single_process(tmp_path):
    per_rank, steps = 2, 2
    mp.spawn(_spawn_target, args=(2, per_rank, steps, str(tmp_path), 29731, "cpu"), nprocs=2, join=True)
    r0, r1 = (torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2))
    _run(0, 1, per_rank, steps, str(tmp_path / "single.pt"), 0)
    one = torch.load(tmp_path / "single.pt", weights_only=True)
    torch.manual_seed(0)
    init = otf.IterativeFlowNet(dim=16).state_dict()
    for k in r0["params"]:
        assert torch.equal(r0["params"][k], r1["params"][k]), k  # all-reduced gradients: identical ranks
        torch.testing.assert_close(r0["params"][k], one["params"][k], rtol=1e-5, atol=1e-6)
        assert not torch.equal(r0["params"][k], init[k]), k  # the step moved every parameter
    assert all(np.isfinite(r0["losses"])) and r0["losses"] != r1["losses"]  # each rank saw its own shard


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_make_pairs_gpu_matches_cpu_ops():
    """The HIP pair (bf16 warp, device ego flow, GPU hole-fill) vs the oracle ops:
    disparity flows exact, ego-motion flows within 1e-4 px (device geometry),
    image2 bit-exact wherever a source won (the fill only touches holes)."""
    dev = torch.device("cuda:0")
    b = _batches(0, 1, 4, 1)[0]
    g = otf.make_pairs(*[x.to(dev) for x in b])
    c = otf.make_pairs(*b, ops=_cpu_ops())
    gi1, gi2, gf, gv = (x.cpu() for x in g)
    ci1, ci2, cf, cv = c
    assert gi2.dtype == torch.bfloat16
    assert torch.equal(gi1, ci1)
    assert torch.equal(gf[0::2], cf[0::2])
    torch.testing.assert_close(gf[1::2], cf[1::2], rtol=0, atol=1e-4)
    # recompute the warp from the GPU flow with the oracle; the fill keeps the
    # pixels utils.py:137-142's mask keeps
    from oracle import oracle, torch_cpu
    from opticalflowfromdepth_amd import synth
    o, v, cl = torch_cpu.fw_flow_scatter(b[0], gf, synth.normalize_depth(b[1]))
    keep = torch.from_numpy(oracle.inpaint_mask(v.numpy(), cl.numpy()) == 0).unsqueeze(1).expand_as(o)
    assert 0.5 < keep.float().mean() < 1
    assert torch.equal(gi2.float()[keep], o[keep])


@pytest.mark.gpu
def test_ddp_gloo_world2_on_gpu(tmp_path):
    """Two ranks on the card, DDP over gloo, the HIP pair builder in the loop."""
    per_rank, steps = 2, 3
    mp.spawn(_spawn_target, args=(2, per_rank, steps, str(tmp_path), 29733, "cuda:0"), nprocs=2, join=True)
    r0, r1 = (torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2))
    for k in r0["params"]:
        assert torch.equal(r0["params"][k], r1["params"][k]), k
    assert all(np.isfinite(r0["losses"]))


@pytest.mark.gpu
def test_gmflow_step_on_gpu_loss_falls():
    """The GMFlow-style step with the HIP pair builder at 368x560 under bf16
    autocast, one batch repeated: finite and falling."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = otf.GlobalMatchFlowNet().to(dev)
    opt, _ = otf.fetch_gmflow_optimizer(model, lr=1e-3)
    b = next(iter(otf.shard_loader(2, 368, 560, 2, 0, 1)))
    losses = []
    for _ in range(30):
        r = otf.gmflow_train_step(model, opt, None, b, dev, otf.StepArgs(gamma=0.9))
        assert r is not None
        losses.append(float(r[0]))
    assert all(np.isfinite(losses)) and max(losses[-5:]) < losses[0], losses


def test_prefetched_pair_equals_inline_pair_cpu():
    """PairPrefetcher (no side stream on CPU) hands over the pair make_pairs builds."""
    b = _batches(0, 1, 2, 1)[0]
    pf = otf.PairPrefetcher("cpu", ops=_cpu_ops())
    pf.put(b)
    got = pf.get(b)
    exp = otf.make_pairs(*b, ops=_cpu_ops())
    assert all(torch.equal(x, y) for x, y in zip(got, exp))


@pytest.mark.gpu
def test_prefetched_pair_on_side_stream_equals_inline():
    """The pair built on the side stream while another step runs is the same
    pair, and the train step on it matches the step that builds its own."""
    dev = torch.device("cuda:0")
    bs = [next(iter(otf.shard_loader(2, 368, 560, 2, 0, 1, base=k))) for k in range(2)]
    pf = otf.PairPrefetcher(dev)
    pf.put(bs[0])
    p0 = pf.get(bs[0])
    pf.put(bs[1])
    torch.cuda.synchronize()
    e0 = otf.make_pairs(*[x.to(dev) for x in bs[0]])
    p1 = pf.get(bs[1])
    e1 = otf.make_pairs(*[x.to(dev) for x in bs[1]])
    torch.cuda.synchronize()
    for got, exp in ((p0, e0), (p1, e1)):
        assert all(torch.equal(x, y) for x, y in zip(got, exp))


@pytest.mark.gpu
def test_train_step_loss_falls_on_a_fixed_batch():
    """bf16 autocast step at 368x560 (config 5 size) on one batch repeated: the loss falls."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = otf.IterativeFlowNet().to(dev)
    opt, _ = otf.fetch_optimizer(model, lr=1e-3)
    b = next(iter(otf.shard_loader(2, 368, 560, 2, 0, 1)))
    losses = [float(otf.train_step(model, opt, None, b, dev, otf.StepArgs())[0]) for _ in range(30)]
    # the flows are tens of px, the step clipped to norm 1: a steady fall, not a collapse
    assert all(np.isfinite(losses)) and max(losses[-5:]) < losses[0] and losses[-1] < losses[10], losses
