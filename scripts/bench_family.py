"""Throughput of the other BASELINE configs (configs[3], configs[4]): CAM+bbox frames/s
with the HIP-event conv roofline of the timed region (bench.roofline_from_timer).

  vgg16:           configs[3] — VGG16-TCAM, 32-frame 224x224 clip, CAM+bbox + the CRF
                   bilateral filter of the clip's softmaxed fcams (TCAM sigmas 15/100)
  inceptionv3:     InceptionV3-TCAM, one 8-frame 299x299 shard, CAM+bbox
  inceptionv3_tmp: configs[4] — a (8 x N)-frame 299x299 clip sharded 8 frames per rank;
                   per-frame CAMs all-gathered over the ranks (RCCL) into the temporal CAM
                   (CAM-TMP, sl_tc_knn 1 'before', README.md:312-314), boxes on it

    python scripts/bench_family.py [--workload all|vgg16|inceptionv3|inceptionv3_tmp]
    python scripts/bench_family.py --workload inceptionv3_tmp --gpus 8   (one rank per GPU)
Rank 0 prints one JSON line per workload; frames_per_s is the whole job (all ranks).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tcam_wsol_video_amd import crf, ops  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_inceptionv3_tcam, build_vgg16_tcam  # noqa: E402
from tcam_wsol_video_amd.parallel import TemporalCAM  # noqa: E402

GFLOP = {"vgg16": 124.22, "inceptionv3": 101.76}   # SURVEY.md §8d (2 x MAC)


def run(name, frames, size, steps, warmup, rank=0, world=1):
    dev = torch.device("cuda", torch.cuda.current_device())
    arch = "vgg16" if name == "vgg16" else "inceptionv3"
    model = (build_vgg16_tcam if arch == "vgg16" else build_inceptionv3_tcam)(seed=0).to(dev)
    temporal = name == "inceptionv3_tmp"
    if temporal:   # this rank's contiguous 8-frame shard of one (8 x world)-frame clip
        xa, ta, ga = bench.make_clip(frames * world, seed=1000, size=size)
        sl = slice(rank * frames, (rank + 1) * frames)
        x, targets, gt = xa[sl].contiguous(), ta[sl], ga[sl]
    else:
        x, targets, gt = bench.make_clip(frames, seed=1000 + rank, size=size)
    xd, td, gd = x.to(dev), targets.to(dev), gt.to(dev)
    raw = ((x * torch.tensor(bench.IMNET_STD)[None, :, None, None] +
            torch.tensor(bench.IMNET_MEAN)[None, :, None, None]) * 255).clamp(0, 255).to(dev)
    comp = CAMComputer(model, cam_curve_interval=0.001, device=dev,
                       keep_fcams=(name == "vgg16"),
                       fwd_streams=int(os.environ.get("TCAM_FAMILY_FWD_STREAMS", "2")),
                       temporal=TemporalCAM(1, "before", 0.0) if temporal else None)
    crf_loss = crf.DenseCRFLoss(weight=2e-9, sigma_rgb=15.0, sigma_xy=100.0, scale_factor=1.0)

    def step():
        comp.evaluate_batch(xd, td, gd)
        if name == "vgg16":   # the CRF on the stream that produced this clip's fcams
            with torch.cuda.stream(comp.fwds[(comp._k - 1) % len(comp.fwds)]):
                return crf_loss(raw, torch.softmax(model.cams, 1))
        return None

    for _ in range(warmup):
        step()
    comp.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer = []
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    ops.set_launch_timer(timer)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    comp.synchronize()
    if world > 1:
        comp.evaluator._synch_across_gpus()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ops.set_launch_timer(None)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # the PMC traffic file is the ResNet50 bench's: not reported for the other families
    from tcam_wsol_video_amd.models import _precision
    prec = _precision(model)
    roof = bench.roofline_from_timer(timer, base, steps, prec, dt / steps * 1e3,
                                     with_traffic=False)
    desc = {"vgg16": "VGG16-TCAM CAM+bbox + CRF filter, 224x224",
            "inceptionv3": "InceptionV3-TCAM CAM+bbox, 299x299 8-frame shard",
            "inceptionv3_tmp": f"InceptionV3-TCAM CAM-TMP+bbox, 299x299, {frames * world}-frame "
                               f"clip sharded {frames}/rank, CAM all-gather"}[name]
    return {"workload": desc, "n_gpus": world, "frames_per_step_per_gpu": frames,
            "frames_per_s": round(frames * world * steps / dt, 1),
            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
            "gflop_per_frame": GFLOP[arch], "precision": prec, "scaling": "weak",
            "roofline": roof}


WORKLOADS = {"vgg16": (32, 224), "inceptionv3": (8, 299), "inceptionv3_tmp": (8, 299)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="all", choices=["all"] + sorted(WORKLOADS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        return subprocess.call([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
                                f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    names = sorted(WORKLOADS) if a.workload == "all" else [a.workload]
    if world > 1:
        names = [n for n in names if n == "inceptionv3_tmp"] or names
    for n in names:
        frames, size = WORKLOADS[n]
        res = run(n, frames, size, a.steps, a.warmup, rank, world)
        if rank == 0:
            print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
