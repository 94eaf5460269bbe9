"""BASELINE.json configs[2]: ResNet50-TCAM training step, batch 8 clips x 32 frames per
GPU (reference batch_size is per process, wsol_loader.py:1020-1022), DDP over N GPUs
(one process per GPU, RCCL all-reduce of the flat decoder gradient).  Synthetic data:
seeded frames, random seeds (cams/tcam_seeding.py is a §8f 'next' row), raw images for
the CRF.  Prints one JSON line (rank 0): frames/s of the whole job.

    python scripts/bench_train.py [--steps K] [--warmup W] [--clips 8]
    torchrun --nproc-per-node N scripts/bench_train.py ...
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402
from tcam_wsol_video_amd.training import DecoderTrainer  # noqa: E402

PREFETCH = os.environ.get("TCAM_ENC_PREFETCH", "1") != "0"
GFLOP_TRAIN = 89.57   # 2 MAC_total + 4 MAC_dec+seg per frame


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clips", type=int, default=8)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--amp", action="store_true",
                    help="the reference's --amp True: autocast fp16 convolutions + GradScaler "
                         "(a side number: the fp32-accurate step is the parity path)")
    ap.add_argument("--no-crf", action="store_true",
                    help="diagnostic only: CRF term off (lambda 0), to size its share of the "
                         "step; not a TCAM step")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    n = args.clips * args.frames
    model = build_r50_tcam(seed=0).to(dev)
    x, _, _ = bench.make_clip(n, seed=2000 + rank)
    raw = ((x * torch.tensor(bench.IMNET_STD)[None, :, None, None] +
            torch.tensor(bench.IMNET_MEAN)[None, :, None, None]) * 255).clamp(0, 255)
    g = torch.Generator().manual_seed(rank)
    seeds = torch.randint(-1, 2, (n, 224, 224), generator=g, dtype=torch.int32)
    seeds[seeds < 0] = -255
    xd, rd, sd = x.to(dev), raw.to(dev), seeds.to(dev)
    tr = DecoderTrainer(model, amp=args.amp)
    if args.no_crf:
        tr.lam = (tr.lam[0], 0.0) + tuple(tr.lam[2:])
    for _ in range(args.warmup):
        tr.step(xd, rd, sd, next_images=xd if PREFETCH else None,
                next_raw=rd if PREFETCH else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        # the next batch (the same synthetic clip) is handed over, as a loader's prefetched
        # batch would be: its frozen-encoder forward overlaps this step's backward (one
        # encoder forward per step either way; the last one, for a step not taken, is
        # inside the timed region)
        losses = tr.step(xd, rd, sd, next_images=xd if PREFETCH else None,
                         next_raw=rd if PREFETCH else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    fps = n * args.steps * world / dt
    if rank == 0:
        print(json.dumps({
            "metric": "frames/sec TCAM training step, ResNet50-TCAM 224x224",
            "precision": "amp (fp16 operands, 1 fp16 MFMA product, fp32 accumulation, "
                         "GradScaler)" if args.amp else (
                "fp32-accurate f16x3 (decoder activations S2; weight and data gradients on "
                "per-channel scaled S2 copies of dy; frozen encoder f16x3)" if tr.f16 else
                "fp32-accurate x6 (decoder forward / data gradients x6, 3x3 weight gradients "
                "f16x3 with per-channel dy scales, frozen encoder f16x3)"),
            "train_prec": "amp" if args.amp else ("f16x3" if tr.f16 else "x6"),
            "applied_steps": tr.applied_steps,
            **({"diagnostic": "CRF term off (not a TCAM step)"} if args.no_crf else {}),
            "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
            "frames_per_step_per_gpu": n, "scaling": "weak",
            "achieved_tflops": round(fps * GFLOP_TRAIN / 1e3, 1),
            "losses_last": [round(float(v), 5) for v in losses.cpu()],
            "data": "synthetic frames/seeds, random-init weights",
            "parallelism": f"ddp{world} (RCCL all-reduce of 9.0M fp32 grads)"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
