"""Stage-1 (task STD_CL) training throughput: the README.md:239-266 run — ResNet50
STDClassifier (WSOL encoder + WGAP) trained end to end, batch 32 frames of 224x224 per GPU,
``--amp True`` in the README (``--amp`` here; the default is the fp32-accurate f16x3 step).
One step = train-mode forward, ClLoss, encoder backward, both SGD groups (and, with N > 1
ranks, the RCCL all-reduce of the 23.5M-parameter flat gradient).  Synthetic frames and
labels, seeded random-init weights.  Prints one JSON line (rank 0) with the step's
algorithmic FLOPs (conv forward + data gradient (no stem) + weight gradient, counted from
the model's geometry) against the MFMA ceiling of the precision.

    python scripts/bench_stdcl.py [--steps K] [--warmup W] [--batch 32] [--amp]
    torchrun --nproc-per-node N scripts/bench_stdcl.py ...
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
from tcam_wsol_video_amd.cl_training import ClassifierTrainer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_stdcl  # noqa: E402

PEAK_F16 = 2516.8          # TF/s dense fp16 MFMA (MI355X_MICROARCH)
PEAK = {"f16x3": PEAK_F16 / 3, "amp": PEAK_F16}


def step_gflop(model, H: int, W: int) -> dict:
    """Algorithmic GFLOP per frame of one training step: every encoder conv's forward
    (2 Cout Cin KH KW Ho Wo), its data gradient (all but the stem: the image needs none)
    and its weight gradient; output sizes from a CPU shape pass of the conv modules."""
    enc = model.encoder
    shapes = {}
    hooks = [m.register_forward_hook(lambda mod, i, o: shapes.__setitem__(mod, o.shape))
             for m in enc.modules() if isinstance(m, torch.nn.Conv2d)]
    with torch.no_grad():
        f = torch.nn.functional.max_pool2d(enc.conv1(torch.zeros(1, 3, H, W)), 3, 2, 1)
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
            for b in layer:
                o = b.conv3(b.conv2(b.conv1(f)))
                if b.downsample is not None:
                    b.downsample[0](f)
                f = o
    for hk in hooks:
        hk.remove()
    fwd = dgrad = 0.0
    for m, s in shapes.items():
        fl = 2.0 * m.out_channels * m.in_channels * m.kernel_size[0] * m.kernel_size[1] * \
            s[2] * s[3] / 1e9
        fwd += fl
        if m is not enc.conv1:
            dgrad += fl
    return {"fwd": fwd, "dgrad": dgrad, "wgrad": fwd, "total": fwd + dgrad + fwd}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--amp", action="store_true")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    model = build_r50_stdcl(seed=0)
    gf = step_gflop(model, 224, 224)
    model = model.to(dev)
    x, _, _ = bench.make_clip(args.batch, seed=3000 + rank)
    y = (torch.arange(args.batch) * 7 + rank) % 10
    xd, yd = x.to(dev), y.to(dev)
    tr = ClassifierTrainer(model, lr=0.001, amp=args.amp)
    for _ in range(args.warmup):
        tr.step(xd, yd)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step(xd, yd)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tr.check_overflow()
    fps = args.batch * args.steps * world / dt
    prec = "amp" if args.amp else "f16x3"
    ach = fps * gf["total"] / 1e3
    if rank == 0:
        print(json.dumps({
            "metric": "frames/sec stage-1 STD_CL training step, ResNet50 WSOL 224x224",
            "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
            "frames_per_step_per_gpu": args.batch, "scaling": "weak", "train_prec": prec,
            "precision": ("amp: autocast fp16 operands, one fp16 MFMA product, fp32 "
                          "accumulation, device GradScaler" if args.amp else
                          "fp32-accurate f16x3: activations S2, gradients S3 with per-channel "
                          "scaled S2 MFMA copies (three fp16 products per MAC)"),
            "gflop_per_frame": {k: round(v, 2) for k, v in gf.items()},
            "roofline": {"bound": "mfma", "achieved": round(ach, 1), "peak": round(PEAK[prec], 1),
                         "unit": "TFLOP/s", "frac": round(ach / PEAK[prec], 3),
                         "basis": "algorithmic conv FLOPs of the step / wall time"},
            "applied_steps": tr.applied_steps, "skipped_steps": tr.skipped_steps,
            "loss_last": round(float(loss), 5),
            "data": "synthetic frames/labels, random-init weights",
            "parallelism": f"ddp{world} (RCCL all-reduce of the 23.5M fp32 gradient)"}),
            flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
