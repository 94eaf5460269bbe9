#!/usr/bin/env python3
"""Headline benchmark: frames/sec of ResNet50-TCAM CAM+bbox extraction at
224x224 on synthetic YTOv2.2-shaped clips (BASELINE.json metric/configs[1]).

One step = one 32-frame clip per GPU, resident in HBM: batched forward
(encoder + WGAP + U-Net decoder + seg head) -> softmax channel-1 CAM -> uint8
-> best box at every one of the 1000 taus (cam_curve_interval=.001) -> IoU vs
GT -> BoxEvaluator counters, all on the device.  N GPUs = N independent clips
(frame-sharded data parallelism, weak scaling); the only collective is the
final all-reduce of the BoxEvaluator counters.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402
from tcam_wsol_video_amd.utils.seeding import synthetic_boxes, synthetic_clip  # noqa: E402

METRIC = "frames/sec CAM+bbox, ResNet50-TCAM 224×224, 1/2/4/8 MI355X"
GFLOP_PER_FRAME = 55.29          # BASELINE.md §3 / SURVEY.md §8d (2 x MAC, hooks)
PEAK_FP32_MFMA_TFLOPS = 157.3    # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_FP32_MFMA_TFLOPS   # "1/16 of BF16 MFMA" (~2.5 PF dense)
# x6 path: every fp32 MAC costs 6 bf16 MACs (csrc/conv_x6.hip), so its
# fp32-equivalent ceiling is the bf16 dense peak / 6.
PEAK_X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
# f16x3 path: fp16 MFMA runs at the bf16 rate and every fp32 MAC costs 3 fp16 MACs
PEAK_F16X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 3
NUMERICS = {
    "x6": "fp32 operands split exactly into 3 bf16 parts, 6 cross products accumulated in "
          "fp32 on the bf16 MFMA (error ~ fp32 FMA chain)",
    "f16x3": "fp32 operands split into 2 fp16 parts (22 significand bits; per-channel "
             "power-of-two weight scales), 3 cross products accumulated in fp32 on the fp16 "
             "MFMA; activations checked against the fp16 range (|x| <= 65504), error vs "
             "fp64 within the fp32-FMA-chain bound (tests/test_gpu_f16.py, "
             "profiles/round3_f16x3_layer_error.txt); covered range: BN-normalised channels "
             "with |beta| + 3|gamma| in [2^-16, 8188] (small-range channels carry power-of-two "
             "exponents folded into the weights: models.act_exponents, verified at 2^-4 ... "
             "2^-12 per channel with no absolute slack)",
    "fp32": "native fp32 MFMA",
}
CONV_SOURCES = ("tcam_wsol_video_amd/csrc/conv_x6.hip", "tcam_wsol_video_amd/csrc/s3_util.h",
                "tcam_wsol_video_amd/csrc/common.h", "tcam_wsol_video_amd/csrc/stem.hip")


def conv_sources_sha() -> str:
    """sha256 over the conv kernel sources: stamps perfdata/pmc_traffic.json, whose
    PMC-measured traffic is reported only while the sources it was measured on are HEAD's."""
    import hashlib
    h = hashlib.sha256()
    for f in CONV_SOURCES:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
IMNET_MEAN = (0.485, .456, .406)
IMNET_STD = (.229, .224, .225)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_clip(frames: int, seed: int, size: int = 224, classes: int = 10):
    """Synthetic YTOv2.2-shaped clip: 360x480 uint8 frames,
    eval transform resize->224, ToTensor, ImageNet normalise; one GT box per
    frame in YTOv1 localization format resized with int() truncation."""
    clip = synthetic_clip(frames, seed=seed)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    x = F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False)
    x = (x - torch.tensor(IMNET_MEAN)[None, :, None, None]) / torch.tensor(IMNET_STD)[None, :, None, None]
    gt = torch.from_numpy(synthetic_boxes(clip, size)).int()[:, None, :]
    rng = np.random.default_rng(seed)
    targets = torch.from_numpy(rng.integers(0, classes, frames))
    return x.contiguous(), targets, gt


def cpu_baseline(model, x, targets, gt, taus, budget_s: float):
    """The oracle (CPU restatement of the reference path, batch-1 per frame as
    inference_wsol.py:332-337, faithful 1000-threshold findContours sweep)
    timed on this host's cores.  Test infrastructure, never the product."""
    from oracle import bbox_ref as BR
    from oracle import model_ref as R
    affinity = len(os.sched_getaffinity(0))
    # every core this process may run on, unless the host caps its share (the GPU box sets
    # OMP_NUM_THREADS to the per-GPU share of a shared machine)
    n_thr = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity)
    torch.set_num_threads(n_thr)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ev = BR.BoxEvaluatorRef(taus)
    t0 = time.perf_counter()
    n = 0
    while n < x.shape[0]:
        lo, fc, _ = R.tcam_forward(sd, x[n:n + 1])
        sm = R.cam_to_scoremap(R.segmentation_cam(fc), x.shape[2:])[0]
        _, order = torch.sort(lo[0], descending=True, stable=True)
        ev.accumulate(sm, gt[n].numpy(), int(targets[n]), order.numpy())
        n += 1
        if time.perf_counter() - t0 > budget_s and n >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": n_thr, "affinity_cores": affinity,
            "kind": "port",
            "sample": f"{n} frames of the same synthetic clip, batch-1 torch-CPU fp32 forward "
                      f"({n_thr} threads) + {len(taus)}-threshold findContours sweep "
                      f"(oracle/contours.c, 1 thread) + IoU/counters"}


def isolated_conv_pass(comp, x, targets, gt, steps: int = 2) -> dict:
    """The same launches on ONE forward stream (no clip overlap): per-launch
    durations without the concurrency of the headline run.  Reported beside the
    roofline, never as it."""
    timer = []
    ops.set_launch_timer(timer)
    saved = comp.fwds
    comp.fwds = comp.fwds[:1]
    try:
        for _ in range(steps):
            comp.evaluate_batch(x, targets, gt)
        comp.synchronize()
        torch.cuda.synchronize()
    finally:
        ops.set_launch_timer(None)
        comp.fwds = saved
    flops = sum(t[1] for t in timer)
    ms = sum(t[2].elapsed_time(t[3]) for t in timer)
    return {"streams": 1, "achieved": round(flops / (ms * 1e-3) / 1e12, 2),
            "avg_launch_ms": round(ms / len(timer), 4),
            "conv_ms_per_step": round(ms / steps, 3)}


def roofline_from_timer(timer, base, steps: int, precision: str, step_ms: float,
                        with_traffic: bool = True, clips=None):
    """Roofline of the dominant kernel family (the convolutions) from the HIP
    events recorded around every conv launch of the TIMED region, on the stream
    each launch ran on.  Algorithmic FLOPs = 2*Cout*K*N per launch over the
    logical input channels (fp32 MACs of the reference conv; neither the 6 bf16
    products of the x6 split nor the stem's 3->8 channel padding are counted).
    ``achieved`` = those FLOPs / the family's busy time (union of its launch intervals
    across the forward streams); ``per_launch_achieved`` = FLOPs / the sum of the
    launches' own durations, which double-counts the time two launches overlap."""
    if os.environ.get("TCAM_DUMP_LAUNCHES"):
        per = len(timer) // steps
        for t in timer[-per:]:
            ms_ = t[2].elapsed_time(t[3])
            log(f"launch {t[4]:40s} {ms_:8.3f} ms {t[1] / ms_ / 1e9:8.1f} TF")
    flops = sum(t[1] for t in timer)
    ms = sum(t[2].elapsed_time(t[3]) for t in timer)
    n_launch = len(timer)
    # launches of consecutive clips overlap on the forward streams: the family's busy
    # time is the UNION of its launch intervals (all events share the base event's clock)
    iv = [(base.elapsed_time(t[2]), base.elapsed_time(t[3]), t[1]) for t in timer]
    lo, hi = -1e30, 1e30
    if clips is not None and len(clips) >= 4:
        # a window of timed clips inside a longer pipelined run: keep the span in which only
        # timed clips run — from the start of the window's second clip (its stream's previous,
        # untimed clip has just finished) to the end of its second-to-last clip (the stream
        # the next, untimed clip starts on is busy until then) — and each launch's FLOPs in
        # proportion to its time inside that span
        a1, b1 = clips[1]
        a2, b2 = clips[-2]
        lo = min(iv[i][0] for i in range(a1, b1))
        hi = max(iv[i][1] for i in range(a2, b2))
    cl = []
    cflops = 0.0
    for a, b, f in iv:
        ca, cb = max(a, lo), min(b, hi)
        if cb > ca:
            cl.append((ca, cb))
            cflops += f * (cb - ca) / (b - a)
    cl.sort()
    busy, cur0, cur1 = 0.0, cl[0][0], cl[0][1]
    for a, b in cl[1:]:
        if a > cur1:
            busy += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    busy += cur1 - cur0
    achieved = cflops / (busy * 1e-3) / 1e12
    busy_per_step = busy / (cflops / (flops / steps))
    per_launch = flops / (ms * 1e-3) / 1e12
    if precision == "x6":
        peak, kern = PEAK_X6_TFLOPS, ("conv_x6_kernel + conv3x3_thin_kernel (all conv launches "
                                      "of the forward)")
        extra = {"peak_basis": "bf16 dense MFMA peak 2516.8 TF / 6 bf16 products per fp32 MAC",
                 "bf16_mfma_tflops": round(6 * achieved, 1)}
    elif precision == "f16x3":
        peak, kern = PEAK_F16X3_TFLOPS, ("conv_x6_kernel<FmtF16> + conv3x3_thin_kernel<FmtF16> + "
                                         "stem_f16x3_kernel + bottleneck_f16x3_kernel (all conv "
                                         "launches of the forward; layer 1's blocks fused)")
        extra = {"peak_basis": "fp16 dense MFMA peak 2516.8 TF (= bf16) / 3 fp16 products per "
                               "fp32 MAC",
                 "fp16_mfma_tflops": round(3 * achieved, 1)}
    else:
        peak, kern = PEAK_FP32_MFMA_TFLOPS, "conv_mfma_kernel (all conv launches of the forward)"
        extra = {"peak_basis": "fp32 MFMA peak (v_mfma_f32_32x32x2_f32)"}
    traffic, tnote = None, None
    pmc = os.path.join(ROOT, "tcam_wsol_video_amd", "perfdata", "pmc_traffic.json")
    if with_traffic and os.path.exists(pmc):   # measured on this workload
        with open(pmc) as fh:
            t = json.load(fh)
        stamp_ok = (t.get("conv_sources_sha") == conv_sources_sha() and
                    t.get("precision", "x6") == precision)
        if stamp_ok:
            traffic = round(t["hbm_bytes_per_launch"] / 1e9, 4)
            tnote = ("GB per conv launch (avg), L2 memory-side bytes from rocprofv3 PMC "
                     "FETCH_SIZE(x2, gfx950) + WRITE_SIZE, scripts/gpu.sh traffic + "
                     "scripts/pmc_traffic.py on conv sources " + t["conv_sources_sha"] +
                     " (" + t.get("commit", "?") + "); includes Infinity-Cache hits")
        else:
            tnote = ("omitted: perfdata/pmc_traffic.json was measured on other conv sources "
                     "or another precision than this run's")
    gflop_step = flops / steps / 1e9
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_note": tnote, "kernel": kern, **extra,
            "timed_in": "the timed region itself (all forward streams, HIP events on the "
                        "launch stream)",
            "launches_per_step": n_launch // steps,
            "algorithmic_gflop_per_step": round(gflop_step, 2),
            "conv_busy_ms_per_step": round(busy_per_step, 3),
            "avg_launch_ms": round(ms / n_launch, 4),
            "per_launch_achieved": round(per_launch, 2),
            # conv FLOPs of a step over the step's wall time (both streams together)
            "wall_achieved": round(gflop_step / step_ms, 2),
            "wall_frac": round(gflop_step / step_ms / peak, 4)}


def breakdown_pass(model, comp, x, targets, gt):
    """Device time of forward vs bbox+eval per step (HIP events, same stream)."""
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    with torch.no_grad():
        e[0].record()
        logits, _, _ = model(x, want_fcams=False)
        e[1].record()
        top1, top5 = ops.topk_flags(logits, targets)
        ngt = torch.full((gt.shape[0],), gt.shape[1], dtype=torch.int32, device=gt.device)
        comp.evaluator.accumulate_batch(model.cam_u8, gt, ngt, top1, top5)
        e[2].record()
    torch.cuda.synchronize()
    return {"forward_ms": round(e[0].elapsed_time(e[1]), 3),
            "cam_bbox_eval_ms": round(e[1].elapsed_time(e[2]), 3)}


def rate_pass(fn, steps: int, frames: int) -> dict:
    """frames/s of ``fn`` (one clip per call) over ``steps`` calls after 2 warm calls."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": round(frames * steps / dt, 2), "unit": "frames/s", "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 3)}


def side_rates(model, comp, xd, td, gd, frames: int, steps: int, fwd_streams: int) -> dict:
    """SURVEY.md §8d / BASELINE.md §4's two other rates of the same workload, short runs
    beside the headline: the validation mode (VALID_FAST_CAM_CURVE_INTERVAL = .004: 250
    taus, train_wsol.py:1473-1480) and the forward alone (encoder + WGAP + decoder + seg
    head + CAM/uint8, no bbox sweep), pipelined over the same forward streams."""
    comp250 = CAMComputer(model, cam_curve_interval=0.004, device=xd.device,
                          fwd_streams=fwd_streams)

    def valid():   # pipelined like the headline (rate_pass synchronises at the end)
        comp250.evaluate_batch(xd, td, gd)

    streams = [torch.cuda.Stream(device=xd.device, priority=-1) for _ in range(fwd_streams)]
    k = [0]

    def fwd_only():
        st = streams[k[0] % len(streams)]
        k[0] += 1
        st.wait_stream(torch.cuda.current_stream())
        # the f16x3 range check deferred to the end of the pass, as the batched evaluation
        # does (a direct forward would synchronise the host on it every clip)
        model.__dict__["_defer_f16_check"] = True
        try:
            with torch.cuda.stream(st), torch.no_grad():
                model(xd, want_fcams=False)
        finally:
            model.__dict__["_defer_f16_check"] = False

    v = rate_pass(valid, steps, frames)
    v["taus"] = len(comp250.cam_threshold_list)
    f = rate_pass(fwd_only, steps, frames)
    f["fwd_streams"] = fwd_streams
    ops.check_f16_overflow(xd.device)
    return {"valid_250tau": v, "forward_only": f}


def launch_ranks(n: int) -> int:
    """One rank per GPU via torch.distributed.run (rendezvous on 127.0.0.1), run as a
    child process; returns its exit status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~1 s timed region at N = 1
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=32, help="frames per clip per GPU")
    ap.add_argument("--interval", type=float, default=0.001, help="cam_curve_interval")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default=os.environ.get("TCAM_CONV_PRECISION", "f16x3"),
                    choices=("f16x3", "x6", "fp32"),
                    help="f16x3: fp16-split MFMA convs on S2 (default); x6: exact bf16-split "
                         "MFMA convs on S3; fp32: native fp32 MFMA convs")
    ap.add_argument("--fwd-streams", type=int, default=int(os.environ.get("TCAM_FWD_STREAMS", 2)),
                    help="forward streams pipelining consecutive clips (CAMComputer)")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the short side measurement of the other conv precision")
    ap.add_argument("--timer-window", type=int, default=5,
                    help="clips of the timed region whose conv launches carry the roofline's "
                         "HIP events (the middle ones; 0 = all)")
    ap.add_argument("--no-roofline-timer", action="store_true",
                    help="time the headline run without per-launch HIP events")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: start the N ranks here (one process per GPU) as
        # children, before this process touches the GPU, and exit with their status
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report "
            f"a {world}-rank measurement as {args.gpus} GPUs")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; more ranks than GPUs only for rehearsals on a smaller box
    # (TCAM_DIST_BACKEND=gloo: RCCL refuses two ranks on one device)
    dev_index = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        dist.init_process_group(os.environ.get("TCAM_DIST_BACKEND", "nccl"), rank=rank,
                                world_size=world)
    dev = torch.device("cuda", dev_index)

    model = build_r50_tcam(seed=0).to(dev)
    model.conv_precision = args.precision
    x, targets, gt = make_clip(args.frames, seed=1000 + rank)
    xd, td, gd = x.to(dev), targets.to(dev), gt.to(dev)
    comp = CAMComputer(model, cam_curve_interval=args.interval, device=dev,
                       fwd_streams=args.fwd_streams)

    for _ in range(args.warmup):
        comp.evaluate_batch(xd, td, gd)
    # the warm-up's held-back bbox sweep (CAMComputer runs each clip's sweep when the next
    # clip is queued) drains here, outside the timed region: the region then holds exactly
    # the K timed clips' sweeps (the last one flushed by the comp.synchronize() inside it)
    comp.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = None if args.no_roofline_timer else []
    # the roofline's per-launch HIP events cover a window of consecutive clips in the middle
    # of the timed region (all their conv launches, on both forward streams): binding events
    # to every dispatch of the region cost the measured rate 2.3 % at 20 steps
    # (profiles/round5_ab_launch_timer.txt); --timer-window 0 times every clip
    win = args.steps if args.timer_window <= 0 else min(args.steps, args.timer_window)
    w0 = (args.steps - win) // 2
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    if timer is not None:
        ops.set_launch_timer(timer, reserve=win * 64)   # events created outside the region
        ops.set_launch_timer(None)
    t0 = time.perf_counter()
    clips = []   # each timed clip's launches: timer[a:b]
    for i in range(args.steps):
        if timer is not None and i == w0:
            ops.set_launch_timer(timer)
        n0 = len(timer) if timer is not None else 0
        comp.evaluate_batch(xd, td, gd)
        if timer is not None and w0 <= i < w0 + win:
            clips.append((n0, len(timer)))
        if timer is not None and i == w0 + win - 1:
            ops.set_launch_timer(None)
    comp.synchronize()
    if world > 1:
        comp.evaluator._synch_across_gpus()  # the one exchange step: all-reduce counters
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ops.set_launch_timer(None)
    # raises (on every rank together) if an activation left the f16x3 range
    ops.check_f16_overflow(dev, all_ranks=True)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames_total = args.frames * args.steps * world
    value = frames_total / elapsed
    step_ms = elapsed / args.steps * 1e3
    roof = None
    if timer:
        roof = roofline_from_timer(timer, base, win, args.precision, step_ms,
                                   clips=clips if win < args.steps else None)
        roof["timed_in"] = (f"clips {w0}..{w0 + win - 1} of the timed region's {args.steps} "
                            f"(every conv launch of those clips, both forward streams, HIP "
                            f"events bound to the dispatches; busy time and FLOPs taken over "
                            f"the span in which only those clips run)")
        roof["isolated_one_stream"] = isolated_conv_pass(comp, xd, td, gd)
    brk = breakdown_pass(model, comp, xd, td, gd)

    alt = None
    if world == 1 and not args.no_alt:
        # the other conv precision, same workload, short run (reported beside)
        other = "x6" if args.precision != "x6" else "f16x3"
        model.conv_precision = other
        for _ in range(2):
            comp.evaluate_batch(xd, td, gd)
        comp.synchronize()
        torch.cuda.synchronize()
        n_alt = max(3, args.steps // 4)
        t1 = time.perf_counter()
        for _ in range(n_alt):
            comp.evaluate_batch(xd, td, gd)
        comp.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        alt = {"precision": other, "value": round(args.frames * n_alt / dt, 2),
               "unit": "frames/s", "steps": n_alt,
               "ms_per_step": round(dt / n_alt * 1e3, 3)}
        model.conv_precision = args.precision

    # the side rates over the headline's own step count, so that they compare with it
    rates = side_rates(model, comp, xd, td, gd, args.frames, args.steps, args.fwd_streams)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model, x, targets, gt, comp.cam_threshold_list, args.cpu_budget)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32",
            "numerics": NUMERICS[args.precision],
            "conv_precision": args.precision,
            "data": "synthetic (seeded YTOv2.2-shaped clip, random-init weights)",
            "config": {"workload": "ResNet50-TCAM CAM+bbox inference, 224x224",
                       "frames_per_step_per_gpu": args.frames,
                       "taus": len(comp.cam_threshold_list),
                       "iou_thresholds": [30, 50, 70],
                       "parallelism": f"dp{world} (frame-sharded clips)"},
            "roofline": roof, "cpu_baseline": cpu, "breakdown_ms_per_step": brk,
            "other_precision": alt,
            # the same clip's validation-mode (250 tau) and forward-only rates, per GPU
            **rates,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
