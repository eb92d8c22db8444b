#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X forward-warp hot path.

Metric (BASELINE.json): Mpix/s forward-warped (768x1024, B=64) + %HBM roofline.
One "step" = one FW pass (flow -> z-buffered splat -> resolve) over one batch
of 64 synthetic 768x1024 images with C=6 channels per image ([RGB, depth,
-flow], the preprocess.py:358/:386 call), inputs already resident in HBM.
Half the images carry a disparity flow, half an ego-motion flow (per-image
seeds 12345+i, camera parameters broadcast from rank 0 over RCCL).

Multi-GPU: one process per GPU, each rank warps its own 64-image shard (weak
scaling, no data-path collective; the reference's --split/--split_id sharding,
preprocess.py:540-547); timing is barrier-bracketed and the max over ranks is
taken.  Rank 0 prints ONE JSON line.  ``python bench.py --gpus N`` with no
torchrun environment starts the N ranks itself (a torch.distributed.run child
process, launched before anything touches the GPU) and exits with the worst
rank's status; under torchrun (WORLD_SIZE set) it is one rank.

Besides the headline, rank 0 reports (after the timed steps, outside the
driver's clock contract): BASELINE config 2 (480x640, B=32), the config-3
hole-fill, the fused first-stage warps, the config-5 bf16 warp, and the CPU
baselines of BASELINE.md §3 (the C loop, the torch-CPU scatter-min warp and
the torch-CPU geometry flow) on this box's host cores.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpix/s forward-warped (768×1024, B=64) + %HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--ego-fraction", type=float, default=0.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline wall budget (headline leg)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    ap.add_argument("--check", action="store_true", help="verify one image against the oracle")
    ap.add_argument("--engine", choices=["tile", "split", "atomic"], default="tile")
    ap.add_argument("--no-hole-fill", action="store_true", help="skip the config-3 hole-fill phase")
    ap.add_argument("--hole-fill-steps", type=int, default=5)
    ap.add_argument("--no-fused", action="store_true", help="skip the fused disparity-warp phase")
    ap.add_argument("--no-bf16", action="store_true", help="skip the config-5 bf16 warp phase")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (480x640, B=32) phase")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / collective / timing skeleton only, on CPU with gloo (tests)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start n ranks of this script as one torch.distributed.run child (never
    an exec: nothing in this process has touched the GPU) and return the worst
    exit status.  Each rank reads RANK / LOCAL_RANK / WORLD_SIZE from torchrun
    and runs main() on cuda:LOCAL_RANK; rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL on this host driver)
    env.setdefault("OMP_NUM_THREADS", str(max(1, min(16, (os.cpu_count() or 1) // max(n, 1)))))
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- helpers
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def lease_cores(threads: int) -> dict:
    """How many host cores the baseline may use, and why: the one-GPU lease's
    CPU share is 16 cores (OMP_NUM_THREADS on the box); host_cpus counts the
    whole machine, which the lease does not own."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"affinity_cpus": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cores_note": f"{threads} threads = the lease's CPU share (OMP_NUM_THREADS); "
                          f"host_cpus is the whole machine, shared with other leases"}


def timed_events(fn, steps, stream):
    """Mean ms per call of fn over `steps` calls, HIP events on `stream`."""
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / steps


def sample_idx(B, n):
    """n image indices of a B-image batch covering both flow kinds (first
    half disparity, second half ego-motion)."""
    n = min(n, B)
    return list(range(n // 2)) + list(range(B - (n - n // 2), B))


def cpu_baseline(obj, flow, depth, budget_s, threads):
    """BASELINE.md §3 on this box's host cores, over a bounded sample of the
    same workload (images of both flow kinds):
      value      -- the C loop (oracle/fw_oracle.c: the serial raster loop of
                    fw_cuda_kernel.cu:28-47 + fw.py:27-43, OpenMP over
                    (image, channel) planes like the reference's <<<B, C>>> grid)
      torch_cpu  -- the torch-CPU scatter_reduce('amin') warp (oracle/torch_cpu.py)
                    and the torch-CPU geometry.py-equivalent depth -> flow
                    (synth.disparity_flow / ego_motion_flow on CPU tensors)."""
    from oracle import oracle, torch_cpu  # test infrastructure: baseline leg only
    from opticalflowfromdepth_amd import synth
    B, C, H, W = obj.shape
    idx = sample_idx(B, 8)
    n_img = len(idx)
    o, f, d = obj[idx].cpu(), flow[idx].cpu(), depth[idx].cpu()
    on, fn_, dn = o.numpy(), f.numpy(), d.numpy()
    oracle.fw_flow(on[:1], fn_[:1], dn[:1], nthreads=threads)  # warm (build + page-in)
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.fw_flow(on, fn_, dn, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    px = reps * n_img * H * W
    loop = px / el / 1e6

    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch_cpu.fw_flow_scatter(o[:1], f[:1], d[:1])
        reps_t, t0 = 0, time.perf_counter()
        while True:
            torch_cpu.fw_flow_scatter(o, f, d)
            reps_t += 1
            el_t = time.perf_counter() - t0
            if el_t >= budget_s / 2:
                break
        # flow synthesis on torch-CPU: the same images' depth -> flow (both kinds)
        seeds = [12345 + i for i in idx]
        s, T = synth.batch_camera_params(seeds)
        h = n_img // 2

        def flows():
            synth.disparity_flow(d[:h].double(), s[:h])
            synth.ego_motion_flow(d[h:].double(), T[h:])
        flows()
        reps_f, t0 = 0, time.perf_counter()
        while True:
            flows()
            reps_f += 1
            el_f = time.perf_counter() - t0
            if el_f >= budget_s / 4:
                break
    finally:
        torch.set_num_threads(prev)
    warp_t = reps_t * n_img * H * W / el_t / 1e6
    flow_t = reps_f * n_img * H * W / el_f / 1e6
    return {"value": round(loop, 2), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), **lease_cores(threads),
            "sample": f"{n_img} images (of the {B}-image batch, both flow kinds) x {reps} reps, C={C}, "
                      f"{H}x{W}, oracle/fw_oracle.c serial-per-plane loop, {el:.1f} s wall",
            "torch_cpu": {"warp_scatter_amin_mpix_s": round(warp_t, 2),
                          "flow_geometry_mpix_s": round(flow_t, 2),
                          "flow_then_warp_mpix_s": round(1.0 / (1.0 / warp_t + 1.0 / flow_t), 2),
                          "threads": threads,
                          "sample": f"same {n_img} images: oracle/torch_cpu.py scatter_reduce('amin') warp "
                                    f"x {reps_t} reps ({el_t:.1f} s); synth.disparity_flow / ego_motion_flow "
                                    f"(geometry.py:17-67, preprocess.py:239-298) on float64 CPU depth "
                                    f"x {reps_f} reps ({el_f:.1f} s)"}}


def hole_fill_phase(out, valid, coll, steps, stream):
    """BASELINE config 3's hole-fill, reported as its own phase:
    utils.inpaint on the warped RGB of this batch (preprocess.py:362-366),
    batched on the GPU, in both orders ops.inpaint offers: "sequential" (the
    default: cv2's heap order, ofd_inpaint_telea_seq_f32) is ``value``;
    "layered" (ofd_inpaint_telea_f32, the faster re-specification) is
    reported beside it.  28 algorithmic B/px (RGB + valid in, RGB out)."""
    from opticalflowfromdepth_amd import ops
    rgb = (out[:, 0:3] * valid).contiguous()
    B, _, H, W = rgb.shape
    px = B * H * W
    res = {}

    def rec(order, ms, bound, parity):
        gbs = px * 28 / (ms / 1e3) / 1e9
        return {"value": round(px / (ms / 1e3) / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(ms, 3),
                "steps": steps, "order": order,
                "roofline": {"bound": bound, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_px": 28},
                "parity": parity}

    recs = {}
    for order in ("sequential", "layered"):
        ops.inpaint(rgb, valid, coll, order=order)  # warm-up (workspace, code paging, launch statistics)
        ms = timed_events(lambda: ops.inpaint(rgb, valid, coll, order=order), steps, stream)
        res[order] = ops.inpaint(rgb, valid, coll, order=order)
        recs[order] = ms
    torch.cuda.synchronize()
    top = rec("sequential", recs["sequential"], "latency (dependent fast-march levels)",
              "bit-exact vs oracle/inpaint_oracle.c sequential mode (OpenCV's Telea restated; "
              "cv2 itself absent, so parity with cv2 is pinned only through that restatement)")
    top["metric"] = "Mpix/s hole-filled (utils.inpaint, cv2-order Telea r=3, same batch)"
    top["hole_fraction"] = round(float((valid == 0).float().mean()), 4)
    top["layered"] = rec("layered", recs["layered"], "latency (dependent hole layers)",
                         "bit-exact vs oracle/inpaint_oracle.c layered mode; differs from the sequential "
                         "order by the specified divergence (divergence_vs_sequential)")
    return rgb, res, top


def hole_fill_cpu_baseline(rgb, valid, coll, gpu_res, budget_s, threads):
    """The reference's hole-fill runs cv2.inpaint(TELEA) per image on the CPU
    (utils.py:149); timed here as the sequential restatement of that algorithm
    (oracle/inpaint_oracle.c), OpenMP over images, on a bounded sample.  The
    same sample checks the GPU's sequential fill against it (mismatches, expected
    0) and measures how far the layered fill sits from it."""
    import numpy as np
    from oracle import oracle  # test infrastructure: baseline leg only
    B = rgb.shape[0]
    idx = sample_idx(B, max(threads, 1))
    n = len(idx)
    r, v, c = rgb[idx].cpu().numpy(), valid[idx].cpu().numpy(), coll[idx].cpu().numpy()
    reps, t0 = 0, time.perf_counter()
    seq = None
    while True:
        seq = oracle.inpaint(r, v, c, 3, layered=False, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    px = reps * n * r.shape[2] * r.shape[3]
    hole = np.broadcast_to(oracle.inpaint_mask(v, c)[:, None] != 0, seq.shape)
    seq_mis = int((gpu_res["sequential"][idx].cpu().numpy() != seq).sum())
    g = gpu_res["layered"][idx].cpu().numpy()
    dif = np.abs(g.astype(np.int32) - seq.astype(np.int32))[hole]
    div = {"hole_values": int(dif.size), "max_abs": int(dif.max()) if dif.size else 0,
           "p99_abs": float(np.percentile(dif, 99)) if dif.size else 0.0,
           "mean_abs": round(float(dif.mean()), 3) if dif.size else 0.0,
           "frac_differing": round(float((dif != 0).mean()), 4) if dif.size else 0.0,
           "frac_over_8": round(float((dif > 8).mean()), 4) if dif.size else 0.0,
           "images": n, "of": "layered GPU fill vs the sequential restatement"}
    return {"value": px / el / 1e6, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{n} warped images (of the {B}-image batch, both flow kinds) x {reps} reps, "
                      f"{r.shape[2]}x{r.shape[3]} RGB, oracle/inpaint_oracle.c sequential Telea (cv2.inpaint "
                      f"restatement), one image per thread, {el:.1f} s wall"}, div, \
        {"images": n, "values_differing": seq_mis}


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

    ms = timed_events(lambda: warp_disparity(rgb, depth, s), steps, stream)
    ms_unfused = timed_events(unfused, steps, stream)
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
    from opticalflowfromdepth_amd import ego_flow, forward_warp_flow, synth, warp_ego, warp_flow_cat
    seeds = [12345 + i for i in range(B)]
    depth = synth.normalize_depth(synth.synthetic_depth(seeds, H, W, dev, dtype=torch.float64))
    rgb = synth.synthetic_rgb(seeds, H, W, dev)
    T = synth.batch_camera_params(seeds)[1].to(dev)
    P, ik = synth.projection(H, W, T, dev)

    def unfused():
        flow = synth.ego_motion_flow(depth, T)
        d32 = depth.float()
        return forward_warp_flow(torch.cat((rgb, d32, flow * -1.0), 1), flow, d32)

    ms = timed_events(lambda: warp_ego(rgb, depth, P, ik), steps, stream)
    ms_unfused = timed_events(unfused, steps, stream)
    ms_flow = timed_events(lambda: ego_flow(depth, P, ik), steps, stream)
    ms_flow_torch = timed_events(lambda: synth.ego_motion_flow(depth, T), steps, stream)
    # the honest comparator, and what the pipeline runs (the flow plane is a
    # group output there): the HIP plane, then FW on it with obj's depth / flow
    # channels generated (warp_flow_cat)
    plane = ego_flow(depth, P, ik)
    ms_cat = timed_events(lambda: warp_flow_cat(rgb, plane, depth), steps, stream)
    px = B * H * W
    gbs = px * 52 / (ms / 1e3) / 1e9
    gbs_cat = px * 60 / (ms_cat / 1e3) / 1e9
    return {"metric": "Mpix/s fused depth->ego-motion flow->splat (preprocess.py:385-387), C=6 out",
            "value": round(px / (ms / 1e3) / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(ms, 4),
            "unfused_ms_per_step": round(ms_unfused, 4), "images": B, "steps": steps,
            "ego_flow_plane_ms": round(ms_flow, 4), "ego_flow_torch_ms": round(ms_flow_torch, 4),
            "plane_then_warp_flow_cat": {
                "warp_ms_per_step": round(ms_cat, 4), "plane_plus_warp_ms": round(ms_flow + ms_cat, 4),
                "roofline": {"bound": "hbm", "achieved": round(gbs_cat, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs_cat / HBM_PEAK_GBS, 4),
                             "algorithmic_bytes_per_px": 60,
                             "bytes": "RGB 12 + flow 8 + depth 8 in, 6 channels 24 + valid 4 + coll 4 out"},
                "parity": "bit-exact vs FW on the materialised concatenation (tests/test_flow_cat.py)"},
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_px": 52},
            "parity": "bit-exact vs FW on ego_flow's plane; the plane bit-exact vs the reference's CPU run (tests/test_ego.py)"}


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
    ms = timed_events(lambda: forward_warp_flow(objb, flow, depth, out=outb), steps, stream)
    ms_f32 = timed_events(lambda: forward_warp_flow(obj, flow, depth, out=outf), steps, stream)
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


def config2_phase(steps, dev, stream, threads, cpu_budget):
    """BASELINE config 2: 480x640, B=32, C=6, fp32 on one GPU (images 0-15
    disparity flow, 16-31 ego-motion flow, seeds 12345+i; the
    preprocess.py:358-359 / :385-387 call shape), with its roofline at 68 B/px
    and its CPU baseline.  Parity is tests/test_configs.py (every image
    bit-exact vs the oracle)."""
    from opticalflowfromdepth_amd import _native, forward_warp_flow, synth
    B, H, W = 32, 480, 640
    seeds = [12345 + i for i in range(B)]
    obj, flow, depth = synth.stage_one_batch(seeds, H, W, dev)
    C = obj.shape[1]
    out = (torch.empty_like(obj), torch.empty_like(depth), torch.empty_like(depth))
    lib = _native.lib()
    for _ in range(3):
        forward_warp_flow(obj, flow, depth, out=out)
    torch.cuda.synchronize()
    ks = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ks:  # force the HIP event handles to exist
        a.record(stream)
        b.record(stream)
    torch.cuda.synchronize()
    every = max(1, int(os.environ.get("OFD_BENCH_EVENT_EVERY", "4")))  # as the headline: sampled launches
    sampled = [k for k in range(steps) if k % every == every - 1 or steps < every]
    t0 = time.perf_counter()
    for k, (a, b) in enumerate(ks):
        if k in sampled:
            lib.ofd_fw_set_profile_events(a.cuda_event, b.cuda_event)
        else:
            lib.ofd_fw_set_profile_events(None, None)
        forward_warp_flow(obj, flow, depth, out=out)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    lib.ofd_fw_set_profile_events(None, None)
    kern_ms = sum(ks[k][0].elapsed_time(ks[k][1]) for k in sampled) / len(sampled)
    px = B * H * W
    bpp = (2 * C + 5) * 4
    rec = {"metric": "Mpix/s forward-warped (480×640, B=32) + %HBM roofline, BASELINE config 2",
           "value": round(px / wall / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(wall * 1e3, 4),
           "steps": steps, "images": B, "height": H, "width": W, "channels": C, "dtype": "f32",
           "roofline": {"bound": "hbm", "achieved": round(px * bpp / (kern_ms / 1e3) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(px * bpp / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                        "kernel": "splat_persist_kernel", "event_ms_per_launch": round(kern_ms, 4),
                        "algorithmic_bytes_per_px": bpp},
           "op_roofline": {"bound": "hbm", "achieved": round(px * bpp / wall / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(px * bpp / wall / 1e9 / HBM_PEAK_GBS, 4),
                           "scope": "whole call, wall clock"},
           "parity": "every image bit-exact vs the oracle (tests/test_configs.py)"}
    if cpu_budget > 0:
        rec["cpu_baseline"] = cpu_baseline(obj, flow, depth, cpu_budget, threads)
    return rec


# ---------------------------------------------------------------- multi-rank record
def rank_report(ms_per_step: float, world: int, coll_dev) -> dict:
    """What the process group saw: its size (dist.get_world_size(), not the
    launcher's WORLD_SIZE), its backend, and every rank's own ms per step
    (all_gather; the line's ms_per_step is the max-rank wall clock)."""
    if not dist.is_initialized():
        return {"world_size": 1, "backend": None, "ms_per_step": [round(ms_per_step, 4)]}
    n = dist.get_world_size()
    mine = torch.tensor([ms_per_step], dtype=torch.float64, device=coll_dev)
    got = [torch.zeros_like(mine) for _ in range(n)]
    dist.all_gather(got, mine)
    return {"world_size": n, "backend": dist.get_backend(), "ms_per_step": [round(float(x[0]), 4) for x in got]}


def finish(world: int) -> None:
    """Final barrier, then teardown: rank 0 runs its extra phases after the
    timed steps, and no rank may tear the process group down while another
    still uses it."""
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------- main
def dry_run(args, world, rank):
    """The launcher / collective / timing skeleton without a GPU (tests): gloo
    collectives, barrier-bracketed timing, max over ranks, one JSON line."""
    if world > 1:
        dist.init_process_group("gloo")
    from opticalflowfromdepth_amd import shard
    n_total = args.batch * world
    seeds = [shard.image_seed(i) for i in range(n_total)]
    s_all, _ = shard.broadcast_camera_params(seeds, device="cpu")
    a, b = shard.shard_range(n_total, world, rank)
    x = torch.zeros(b - a)
    for _ in range(args.warmup):
        x += 1
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x += s_all[a:b]
    if world > 1:
        dist.barrier()
    own = time.perf_counter() - t0
    t = torch.tensor([own], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ranks = rank_report(own * 1e3 / max(args.steps, 1), world, "cpu")
    if rank == 0:
        time.sleep(0.2)  # stands in for rank 0's extra phases: the others wait at the final barrier
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpix/s", "n_gpus": ranks["world_size"],
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                          "shard_images": [a, b], "wall_s": float(t[0]), "ranks": ranks}), flush=True)
    finish(world)


_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """One line per phase on stderr (stdout carries only the JSON line), so a
    watchdog on silent output never mistakes the later phases for a hang."""
    print(f"# bench {time.perf_counter() - _T0:7.1f}s: {msg}", file=sys.stderr, flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    # OFD_BENCH_BACKEND=gloo + OFD_BENCH_SAME_DEVICE=1 rehearse the N>1 path on
    # a one-GPU box (all ranks on cuda:0, CPU collectives); the default is one
    # rank per GPU with RCCL ("nccl" on ROCm).
    backend = os.environ.get("OFD_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("OFD_BENCH_SAME_DEVICE") == "1" else local
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    # a process group whenever a launcher started this process (WORLD_SIZE set),
    # so `torchrun --nproc-per-node 1 bench.py` runs the RCCL path at one rank
    pg = world > 1 or "WORLD_SIZE" in os.environ
    if pg:
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

    progress(f"inputs ready ({B}x{C}x{H}x{W}); warmup")
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
    starts, ends, rstarts, rends, bstarts = mk(), mk(), mk(), mk(), mk()
    for ev in rstarts + rends + bstarts:  # torch creates events lazily: force the HIP handles to exist
        ev.record(stream)
    torch.cuda.synchronize()
    lib = _native.lib()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # Events: the library's pair around the dominant kernel (the roofline's
    # launch duration), on every EVERY-th step of the timed region.  A pair
    # costs the stream ~6 us (0.730 vs 0.724 ms per step with a pair on every
    # step, tools/ab_env.sh), so the call time is the wall clock of the K steps
    # and the kernel time the mean over the sampled launches.  The probe knob
    # OFD_BENCH_EVENTS=2 adds events around each call, 0 drops all.
    evmode = int(os.environ.get("OFD_BENCH_EVENTS", "1"))
    every = max(1, int(os.environ.get("OFD_BENCH_EVENT_EVERY", "4")))
    sampled = [k for k in range(args.steps) if k % every == every - 1 or args.steps < every] if evmode >= 1 else []
    for k in range(args.steps):
        # events around the dominant kernel, recorded by the library
        # on the launch stream (include/ofd_fw.h: ofd_fw_set_profile_events)
        if evmode >= 1:
            if k in sampled:
                lib.ofd_fw_set_profile_events(rstarts[k].cuda_event, rends[k].cuda_event)
                lib.ofd_fw_set_profile_bin_event(bstarts[k].cuda_event)
            else:
                lib.ofd_fw_set_profile_events(None, None)
                lib.ofd_fw_set_profile_bin_event(None)
        if evmode >= 2:
            starts[k].record(stream)
        forward_warp_flow(obj, flow, depth, out=out)
        if evmode >= 2:
            ends[k].record(stream)
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    wall = time.perf_counter() - t0
    lib.ofd_fw_set_profile_events(None, None)
    lib.ofd_fw_set_profile_bin_event(None)
    ev_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)] if evmode >= 2 else [wall * 1e3 / args.steps]
    dev_ms = sum(ev_ms) / len(ev_ms)
    rv_ms = [rstarts[k].elapsed_time(rends[k]) for k in sampled] if evmode >= 1 else [dev_ms]
    resolve_ms = sum(rv_ms) / len(rv_ms)
    bin_ms = None
    if evmode >= 1 and args.engine != "atomic" and sampled:
        bv = [bstarts[k].elapsed_time(rstarts[k]) for k in sampled]
        bin_ms = sum(bv) / len(bv)

    ranks = rank_report(wall / args.steps * 1e3, world, coll_dev)
    t = torch.tensor([wall, dev_ms], dtype=torch.float64, device=coll_dev)
    if pg:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, dev_ms_max = float(t[0]), float(t[1])

    px_step_rank = B * H * W
    bytes_per_px = (2 * C + 5) * 4  # algorithmic: obj C + flow 2 + depth in; out C + valid + coll
    value = n_total * H * W * args.steps / wall / 1e6
    achieved_gbs = px_step_rank * bytes_per_px / (dev_ms / 1e3) / 1e9
    # dominant kernel and the bytes it moves per source pixel (its own, not
    # the op's: the split of the op's 68 B/px between the launches)
    #   tile  : SPLAT.  With BIN's packed targets (the default for a flow) it
    #           reads obj C*4 (the winners' gather), depth 4 and the 2-byte
    #           target code, and writes output C*4, valid 4, collision 4;
    #           BIN reads the flow (8) and writes the code (2).  Unpacked,
    #           SPLAT re-reads the flow itself: (2C+5)*4, every byte of the op.
    #   split : RESOLVE gathers obj and writes the C output planes, 2C*4
    #   atomic: the resolve pass also writes valid / collision, (2C+2)*4
    packed = args.engine == "tile" and lib.ofd_fw_set_pack(-1) == 1
    splat_bpp = (8 * C + 14) if packed else (2 * C + 5) * 4
    bin_bpp = 10 if packed else 8
    kern_bpp, kern_name = {"tile": (splat_bpp, "splat_persist_kernel"),
                           "split": (2 * C * 4, "resolve2d_kernel"),
                           "atomic": ((2 * C + 2) * 4, "resolve_atomic_kernel")}[args.engine]
    kern_gbs = px_step_rank * kern_bpp / (resolve_ms / 1e3) / 1e9
    bin_rec = None
    if bin_ms is not None:
        bin_gbs = px_step_rank * bin_bpp / (bin_ms / 1e3) / 1e9
        bin_rec = {"kernel": "bin_kernel", "event_ms_per_launch": round(bin_ms, 4), "bytes_per_px": bin_bpp,
                   "bytes": "flow 8 in" + (", target code 2 out" if packed else ""),
                   "achieved": round(bin_gbs, 1), "frac": round(bin_gbs / HBM_PEAK_GBS, 4)}

    # PMC traffic (profiles/pmc_traffic.json, tools/profile_round.sh): only
    # for the build that was profiled -- a file from other sources says
    # nothing about this library's traffic
    traffic = traffic_step = bin_traffic = None
    traffic_note = "no PMC file for this configuration"
    pmc_file = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_file) and args.engine != "atomic":
        try:
            pm = json.load(open(pmc_file))
            if pm.get("config") == [B, C, H, W] and pm.get("engine", "split") == args.engine:
                if pm.get("build_id") != _native.build_id():
                    traffic_note = (f"null: profiles/pmc_traffic.json is from build {pm.get('build_id')}, "
                                    f"this run is build {_native.build_id()}")
                else:
                    traffic_step = pm.get("hbm_bytes_per_step")
                    for kk in pm.get("kernels", []):
                        if kk["kernel"] == kern_name:
                            traffic = kk["fetch_bytes_x2"] + kk["write_bytes"]
                        if kk["kernel"] == "bin_kernel":
                            bin_traffic = kk["fetch_bytes_x2"] + kk["write_bytes"]
                    traffic_note = f"profiles/pmc_traffic.json (build {pm.get('build_id')}): " + str(pm.get("source"))
        except Exception as e:  # a malformed file is reported, not fatal
            traffic_note = f"null: profiles/pmc_traffic.json unreadable ({e})"
    if bin_rec is not None:
        bin_rec["traffic"] = bin_traffic

    cpu = None
    threads = args.cpu_threads if args.cpu_threads > 0 else min(16, os.cpu_count() or 1)
    cpu_on = rank == 0 and world == 1 and not args.no_cpu_baseline
    progress(f"headline {wall / args.steps * 1e3:.4f} ms/step")
    if cpu_on:
        progress("cpu baseline")
        cpu = cpu_baseline(obj, flow, depth, args.cpu_seconds, threads)

    cfg2 = None
    if rank == 0 and not args.no_config2:
        progress("config 2")
        cfg2 = config2_phase(60, dev, stream, threads, args.cpu_seconds / 2 if cpu_on else 0)

    fused = fused_ego = None
    if rank == 0 and not args.no_fused:
        progress("fused warps")
        fused = fused_disparity_phase(B, H, W, 10, dev, stream)
        fused_ego = fused_ego_phase(B, H, W, 10, dev, stream)

    bf16 = None
    if rank == 0 and not args.no_bf16:
        progress("bf16 warp")
        bf16 = bf16_warp_phase(64, 368, 560, 20, dev, stream)

    hole = None
    if rank == 0 and not args.no_hole_fill:  # untimed by the driver's clock contract: after the K steps
        progress("hole-fill")
        rgb, res, hole = hole_fill_phase(out[0], out[1], out[2], args.hole_fill_steps, stream)
        if cpu_on:
            progress("hole-fill cpu baseline")
            (hole["cpu_baseline"], hole["layered"]["divergence_vs_sequential"],
             hole["sequential_vs_oracle"]) = hole_fill_cpu_baseline(rgb, out[1], out[2], res, args.cpu_seconds,
                                                                    threads)

    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": ranks["world_size"],
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
                         "event_launches": len(sampled) if evmode >= 1 else 0,
                         "traffic_source": traffic_note,
                         "bytes": (f"obj {4 * C} (winners' gather) + depth 4 + target code 2 in, output {4 * C} "
                                   f"+ valid 4 + collision 4 out" if packed and args.engine == "tile" else None)},
            "bin": bin_rec,
            "op_roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                            "traffic": traffic_step,
                            "scope": f"whole forward_warp_flow call ({args.engine} engine, all launches)",
                            "algorithmic_bytes_per_px": bytes_per_px,
                            ("event_ms_per_call" if evmode >= 2 else "wall_ms_per_call"): round(dev_ms, 4)},
            "cpu_baseline": cpu,
            "config2": cfg2,
            "hole_fill": hole,
            "fused_disparity": fused,
            "fused_ego": fused_ego,
            "bf16_warp": bf16,
            "ranks": ranks,
            "build_id": _native.build_id(),
        }
        print(json.dumps(rec), flush=True)
    finish(world)


if __name__ == "__main__":
    main()
