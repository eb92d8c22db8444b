#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X forward-warp hot path.

Metric (BASELINE.json): Mpix/s forward-warped (768x1024, B=64) + %HBM roofline.
One "step" = one FW pass (flow -> z-buffered splat -> resolve) over one batch
of 64 synthetic 768x1024 images with C=6 channels per image ([RGB, depth,
-flow], the preprocess.py:358/:386 call), inputs already resident in HBM.
Half the images carry a disparity flow, half an ego-motion flow (per-image
seeds 12345+i, camera parameters broadcast from rank 0 over RCCL).

Multi-GPU: one process per GPU (torchrun), each rank warps its own 64-image
shard (weak scaling, no data-path collective); timing is barrier-bracketed and
the max over ranks is taken.  Rank 0 prints ONE JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpix/s forward-warped (768×1024, B=64) + %HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--ego-fraction", type=float, default=0.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline wall budget")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    ap.add_argument("--check", action="store_true", help="verify one image against the oracle")
    ap.add_argument("--engine", choices=["tile", "split", "atomic"], default="tile")
    ap.add_argument("--no-hole-fill", action="store_true", help="skip the config-3 hole-fill phase")
    ap.add_argument("--hole-fill-steps", type=int, default=5)
    ap.add_argument("--no-fused", action="store_true", help="skip the fused disparity-warp phase")
    ap.add_argument("--no-bf16", action="store_true", help="skip the config-5 bf16 warp phase")
    return ap.parse_args()


def cpu_baseline(obj, flow, depth, budget_s, threads):
    """Oracle (C restatement of fw_cuda_kernel.cu:28-47 + fw.py:27-43, OpenMP
    over (image, channel) planes like the reference's <<<B, C>>> grid), timed
    on this box's host cores over a bounded sample of the same workload."""
    from oracle import oracle  # test infrastructure: baseline leg only
    n_img = min(8, obj.shape[0])
    half = n_img // 2
    B = obj.shape[0]
    idx = list(range(half)) + list(range(B - (n_img - half), B))  # both flow kinds
    o = obj[idx].cpu().numpy()
    f = flow[idx].cpu().numpy()
    d = depth[idx].cpu().numpy()
    oracle.fw_flow(o[:1], f[:1], d[:1], nthreads=threads)  # warm (build + page-in)
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.fw_flow(o, f, d, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    px = reps * n_img * o.shape[2] * o.shape[3]
    return {"value": px / el / 1e6, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{n_img} images (of the {B}-image batch, both flow kinds) x {reps} reps, "
                      f"C={o.shape[1]}, {o.shape[2]}x{o.shape[3]}, oracle/fw_oracle.c serial-per-plane "
                      f"loop, {el:.1f} s wall on {platform.processor() or platform.machine()}"}


def hole_fill_phase(out, valid, coll, steps, stream):
    """BASELINE config 3's hole-fill, reported as its own phase:
    utils.inpaint on the warped RGB of this batch (preprocess.py:362-366),
    batched on the GPU.  28 algorithmic B/px (RGB + valid in, RGB out)."""
    from opticalflowfromdepth_amd import ops
    rgb = (out[:, 0:3] * valid).contiguous()
    res = ops.inpaint(rgb, valid, coll)  # warm-up (workspace, code paging)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for s, e in ev:
        s.record(stream)
        res = ops.inpaint(rgb, valid, coll)
        e.record(stream)
    torch.cuda.synchronize()
    ms = sum(s.elapsed_time(e) for s, e in ev) / steps
    B, _, H, W = rgb.shape
    px = B * H * W
    gbs = px * 28 / (ms / 1e3) / 1e9
    return rgb, res, {
        "metric": "Mpix/s hole-filled (utils.inpaint, layered Telea r=3, same batch)",
        "value": round(px / (ms / 1e3) / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(ms, 3), "steps": steps,
        "hole_fraction": round(float((valid == 0).float().mean()), 4),
        "roofline": {"bound": "latency (one launch per hole layer)", "achieved": round(gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
                     "algorithmic_bytes_per_px": 28},
        "parity": "bit-exact vs oracle/inpaint_oracle.c layered mode; cv2 Telea parity unpinned (no OpenCV)"}


def fused_disparity_phase(B, H, W, steps, dev, stream):
    """preprocess.py:356-359 as one fused warp (depth ->
    disparity -> flow -> splat, obj's depth / flow channels generated in the
    gather) over B disparity images, next to the same call unfused (torch
    builds the flow and the 6-channel obj, then forward_warp_flow).
    Algorithmic bytes: RGB 12 + depth 4 in, 6 channels 24 + valid 4 + coll 4
    out = 48 B/px."""
    from opticalflowfromdepth_amd import forward_warp_flow, preprocess as pp, synth, warp_disparity
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev))
    rgb = synth.synthetic_rgb(seeds, H, W, dev)
    s = synth.batch_camera_params(seeds)[0].to(dev)

    def unfused():
        flow = pp.Convert.disparity_to_flow(pp.Convert.depth_to_disparity(depth, s), random_sign=False)
        return forward_warp_flow(torch.cat((rgb, depth, flow * -1.0), 1), flow, depth)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / steps

    ms = timed(lambda: warp_disparity(rgb, depth, s))
    ms_unfused = timed(unfused)
    px = B * H * W
    gbs = px * 48 / (ms / 1e3) / 1e9
    return {"metric": "Mpix/s fused depth->disparity->flow->splat (preprocess.py:356-359), C=6 out",
            "value": round(px / (ms / 1e3) / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(ms, 4),
            "unfused_ms_per_step": round(ms_unfused, 4), "images": B, "steps": steps,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_px": 48},
            "parity": "bit-exact vs the unfused FW call and the oracle (tests/test_fused.py)"}


def fused_ego_phase(B, H, W, steps, dev, stream):
    """SURVEY §8f row 1 (ego-motion half): preprocess.py:385-387 as one fused
    warp (depth -> ego-motion flow -> splat) over B images with float64 depth,
    next to the unfused sequence (the torch restatement of geometry.py's
    flow, the concatenation, then forward_warp_flow) and to the one-kernel
    flow plane (ops.ego_flow).  Algorithmic bytes of the fused call: RGB 12 +
    depth 8 in, 6 channels 24 + valid 4 + coll 4 out = 52 B/px."""
    from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, synth, warp_ego
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64))
    rgb = synth.synthetic_rgb(seeds, H, W, dev)
    T = synth.batch_camera_params(seeds)[1].to(dev)
    P, ik = synth.projection(H, W, T, dev)

    def unfused():
        flow = synth.ego_motion_flow(depth, T)
        d32 = depth.float()
        return forward_warp_flow(torch.cat((rgb, d32, flow * -1.0), 1), flow, d32)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / steps

    ms = timed(lambda: warp_ego(rgb, depth, P, ik))
    ms_unfused = timed(unfused)
    ms_flow = timed(lambda: ego_flow(depth, P, ik))
    ms_flow_torch = timed(lambda: synth.ego_motion_flow(depth, T))
    px = B * H * W
    gbs = px * 52 / (ms / 1e3) / 1e9
    return {"metric": "Mpix/s fused depth->ego-motion flow->splat (preprocess.py:385-387), C=6 out",
            "value": round(px / (ms / 1e3) / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(ms, 4),
            "unfused_ms_per_step": round(ms_unfused, 4), "images": B, "steps": steps,
            "ego_flow_plane_ms": round(ms_flow, 4), "ego_flow_torch_ms": round(ms_flow_torch, 4),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_px": 52},
            "parity": "bit-exact vs FW on ego_flow's plane; flow within 8 ulp of the reference's (tests/test_ego.py)"}


def bf16_warp_phase(B, H, W, steps, dev, stream):
    """the training-loop warp on bf16
    planes (no reference counterpart), at 368x560, next to the float32 warp of
    the same batch.  Algorithmic bytes at C=6: obj 12 + flow 8 + depth 4 in,
    output 12 + valid 4 + coll 4 out = 44 B/px (68 for the float32 op)."""
    from opticalflowfromdepth_amd import forward_warp_flow, synth
    seeds = [7000 + i for i in range(B)]
    obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev)
    objb = obj.to(torch.bfloat16)
    C = obj.shape[1]
    outb = (torch.empty_like(objb), torch.empty_like(depth), torch.empty_like(depth))
    outf = (torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / steps

    ms = timed(lambda: forward_warp_flow(objb, flow, depth, out=outb))
    ms_f32 = timed(lambda: forward_warp_flow(obj, flow, depth, out=outf))
    same = bool(torch.equal(outb[0].view(torch.int16), outf[0].to(torch.bfloat16).view(torch.int16)))
    px = B * H * W
    bpp = 4 * C + 20
    gbs = px * bpp / (ms / 1e3) / 1e9
    return {"metric": f"Mpix/s bf16 forward warp (config 5, {H}x{W}), C={C}", "value": round(px / (ms / 1e3) / 1e6, 1),
            "unit": "Mpix/s", "ms_per_step": round(ms, 4), "f32_ms_per_step": round(ms_f32, 4), "images": B,
            "steps": steps, "dtype": "bf16 planes, f32 flow / depth",
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_px": bpp,
                         "scope": "whole call (BIN + SPLAT)"},
            "equals_f32_path": same,
            "parity": "bit-exact vs the oracle and the float32 path (tests/test_bf16.py)"}


def hole_fill_cpu_baseline(rgb, valid, coll, budget_s, threads):
    """The reference's hole-fill runs cv2.inpaint(TELEA) per image on the CPU
    (utils.py:149); timed here as the sequential restatement of that algorithm
    (oracle/inpaint_oracle.c), OpenMP over images, on a bounded sample."""
    from oracle import oracle  # test infrastructure: baseline leg only
    B = rgb.shape[0]
    n = min(max(threads, 1), B)
    idx = list(range(n // 2)) + list(range(B - (n - n // 2), B))  # both flow kinds
    r, v, c = rgb[idx].cpu().numpy(), valid[idx].cpu().numpy(), coll[idx].cpu().numpy()
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.inpaint(r, v, c, 3, layered=False, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    px = reps * n * r.shape[2] * r.shape[3]
    return {"value": px / el / 1e6, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{n} warped images (of the {B}-image batch, both flow kinds) x {reps} reps, 768x1024 RGB, "
                      f"oracle/inpaint_oracle.c sequential Telea (cv2.inpaint restatement), one image per thread, "
                      f"{el:.1f} s wall"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OFD_BENCH_BACKEND=gloo + OFD_BENCH_SAME_DEVICE=1 rehearse the N>1 path on
    # a one-GPU box (all ranks on cuda:0, CPU collectives); the default is one
    # rank per GPU with RCCL ("nccl" on ROCm).
    backend = os.environ.get("OFD_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("OFD_BENCH_SAME_DEVICE") == "1" else local
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    from opticalflowfromdepth_amd import forward_warp_flow, shard, synth
    from opticalflowfromdepth_amd import _native

    B, H, W = args.batch, args.height, args.width
    n_total = B * world
    seeds = [shard.image_seed(i) for i in range(n_total)]
    s_all, T_all = shard.broadcast_camera_params(seeds, device=coll_dev)  # RCCL broadcast (setup)
    a, b = shard.shard_range(n_total, world, rank)
    obj, flow, depth = synth.stage_one_batch(seeds[a:b], H, W, dev, ego_fraction=args.ego_fraction,
                                             camera=(s_all[a:b], T_all[a:b]))
    C = obj.shape[1]
    out = (torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth))
    _native.lib().ofd_fw_set_engine({"tile": 0, "atomic": 1, "split": 2}[args.engine])
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        forward_warp_flow(obj, flow, depth, out=out)
    torch.cuda.synchronize()

    if args.check and rank == 0:
        from oracle import oracle
        exp = oracle.fw_flow(obj[:1].cpu().numpy(), flow[:1].cpu().numpy(), depth[:1].cpu().numpy())
        ok = all((g[:1].cpu().numpy() == e).all() for g, e in zip(out, exp))
        print(f"# check vs oracle (image 0): {'OK' if ok else 'MISMATCH'}", file=sys.stderr)

    stream = torch.cuda.current_stream(dev)
    mk = lambda: [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    starts, ends, rstarts, rends = mk(), mk(), mk(), mk()
    for ev in rstarts + rends:  # torch creates events lazily: force the HIP handles to exist
        ev.record(stream)
    torch.cuda.synchronize()
    lib = _native.lib()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # Per-step events: the library's pair around the dominant kernel (the
    # roofline's launch duration).  Each extra event record costs the stream
    # ~5-10 us, so the call time is the wall clock of the K steps; the probe
    # knob OFD_BENCH_EVENTS=2 adds events around each call, 0 drops all.
    evmode = int(os.environ.get("OFD_BENCH_EVENTS", "1"))
    for k in range(args.steps):
        # events around the dominant kernel, recorded by the library
        # on the launch stream (include/ofd_fw.h: ofd_fw_set_profile_events)
        if evmode >= 1:
            lib.ofd_fw_set_profile_events(rstarts[k].cuda_event, rends[k].cuda_event)
        if evmode >= 2:
            starts[k].record(stream)
        forward_warp_flow(obj, flow, depth, out=out)
        if evmode >= 2:
            ends[k].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    lib.ofd_fw_set_profile_events(None, None)
    ev_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)] if evmode >= 2 else [wall * 1e3 / args.steps]
    dev_ms = sum(ev_ms) / len(ev_ms)
    rv_ms = [s.elapsed_time(e) for s, e in zip(rstarts, rends)] if evmode >= 1 else [dev_ms]
    resolve_ms = sum(rv_ms) / len(rv_ms)

    t = torch.tensor([wall, dev_ms], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, dev_ms_max = float(t[0]), float(t[1])

    px_step_rank = B * H * W
    bytes_per_px = (2 * C + 5) * 4  # algorithmic: obj C + flow 2 + depth in; out C + valid + coll
    value = n_total * H * W * args.steps / wall / 1e6
    achieved_gbs = px_step_rank * bytes_per_px / (dev_ms / 1e3) / 1e9
    # dominant kernel and its algorithmic bytes per source pixel:
    #   tile  : SPLAT reads flow, depth and obj, writes output, valid and
    #           collision -- every algorithmic byte of the op, (2C+5)*4
    #           (BIN's flow read is the one re-read)
    #   split : RESOLVE gathers obj and writes the C output planes, 2C*4
    #   atomic: the resolve pass also writes valid / collision, (2C+2)*4
    kern_bpp, kern_name = {"tile": ((2 * C + 5) * 4, "splat_persist_kernel"),
                           "split": (2 * C * 4, "resolve2d_kernel"),
                           "atomic": ((2 * C + 2) * 4, "resolve_atomic_kernel")}[args.engine]
    kern_gbs = px_step_rank * kern_bpp / (resolve_ms / 1e3) / 1e9

    traffic = traffic_step = None
    traffic_note = None
    pmc_file = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_file) and args.engine != "atomic":
        try:
            pm = json.load(open(pmc_file))
            if pm.get("config") == [B, C, H, W] and pm.get("engine", "split") == args.engine:
                traffic_step = pm.get("hbm_bytes_per_step")
                for kk in pm.get("kernels", []):
                    if kk["kernel"] == kern_name:
                        traffic = kk["fetch_bytes_x2"] + kk["write_bytes"]
                traffic_note = pm.get("source")
        except Exception:
            pass

    cpu = None
    threads = args.cpu_threads if args.cpu_threads > 0 else min(16, os.cpu_count() or 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(obj, flow, depth, args.cpu_seconds, threads)

    fused = fused_ego = None
    if rank == 0 and not args.no_fused:
        fused = fused_disparity_phase(B, H, W, 10, dev, stream)
        fused_ego = fused_ego_phase(B, H, W, 10, dev, stream)

    bf16 = None
    if rank == 0 and not args.no_bf16:
        bf16 = bf16_warp_phase(64, 368, 560, 20, dev, stream)

    hole = None
    if rank == 0 and not args.no_hole_fill:  # untimed by the driver's clock contract: after the K steps
        rgb, _, hole = hole_fill_phase(out[0], out[1], out[2], args.hole_fill_steps, stream)
        if world == 1 and not args.no_cpu_baseline:
            hole["cpu_baseline"] = hole_fill_cpu_baseline(rgb, out[1], out[2], args.cpu_seconds, threads)

    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded depth fields -> normalize_depth -> disparity / ego-motion flow)",
            "config": {"workload": f"FW forward warp, {H}x{W}, B={B} per GPU, C={C} "
                                   f"(BASELINE config 3/4)", "global_batch": n_total, "height": H,
                       "width": W, "channels": C, "ego_fraction": args.ego_fraction,
                       "parallelism": f"shard{world} (images, no data-path collective)"},
            "roofline": {"bound": "hbm", "achieved": round(kern_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(kern_gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": f"{kern_name} ({args.engine} engine), dominant kernel of the call",
                         "algorithmic_bytes_per_px": kern_bpp,
                         "event_ms_per_launch": round(resolve_ms, 4),
                         "traffic_source": traffic_note},
            "op_roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                            "traffic": traffic_step,
                            "scope": f"whole forward_warp_flow call ({args.engine} engine, all launches)",
                            "algorithmic_bytes_per_px": bytes_per_px,
                            ("event_ms_per_call" if evmode >= 2 else "wall_ms_per_call"): round(dev_ms, 4)},
            "cpu_baseline": cpu,
            "hole_fill": hole,
            "fused_disparity": fused,
            "fused_ego": fused_ego,
            "bf16_warp": bf16,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
