"""End-to-end frames/s from JPEG files (SURVEY.md §8f row 3 feeding configs[1]): the
bench's ResNet50-TCAM CAM+bbox workload, but every 32-frame clip arrives as 32 JPEG files
(360x480 YTO-shaped frames, Pillow-encoded q90 4:2:0, held in host memory) and goes
bytes -> device decode (csrc/jpeg.hip) -> eval transform (Resize 224, ToTensor,
Normalize; csrc/frames.hip) -> forward -> CAM -> boxes at every tau -> counters.

Decode + transform of clip i+1 run on their own stream while the forward streams work on
clip i (one event orders each clip's forward after its frames).  Reports frames/s of the
whole pipeline beside the same run fed device-resident frames (the bench.py headline
path) and the per-core rate of the reference's host path (PIL decode + resize +
ToTensor/Normalize).  One JSON line.
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd import frames, jpeg  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402
from tcam_wsol_video_amd.utils.seeding import synthetic_boxes, synthetic_clip  # noqa: E402


def clip_files(n_clips: int, n_frames: int, q: int):
    out = []
    for c in range(n_clips):
        clip = synthetic_clip(n_frames, seed=500 + c)          # (T, 360, 480, 3) uint8
        datas = []
        for t in range(n_frames):
            b = io.BytesIO()
            Image.fromarray(clip[t]).save(b, "JPEG", quality=q, subsampling=2)
            datas.append(b.getvalue())
        gt = torch.from_numpy(np.asarray(synthetic_boxes(clip, 224), np.int32))[:, None, :]
        out.append((datas, gt))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=8, help="distinct clips (cycled)")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--interval", type=float, default=0.001)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = build_r50_tcam(seed=0).to(dev)
    comp = CAMComputer(model, cam_curve_interval=args.interval, device=dev, fwd_streams=2)
    files = clip_files(args.clips, args.frames, args.quality)
    targets = torch.zeros(args.frames, dtype=torch.int64, device=dev)
    gts = [g.to(dev) for _, g in files]
    dec = jpeg.JpegDecoder(dev)
    tf = frames.get_eval_tranforms(224)
    dstream = torch.cuda.Stream(dev)
    caller = torch.cuda.current_stream(dev)

    def step(k):
        datas, _ = files[k % len(files)]
        with torch.cuda.stream(dstream):
            clip = dec.decode_batch(datas)
            x, _ = tf(clip)
            ready = torch.cuda.Event()
            ready.record(dstream)
        caller.wait_event(ready)
        x.record_stream(caller)
        comp.evaluate_batch(x, targets, gts[k % len(files)])

    def run(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            fn(k)
        comp.synchronize()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for k in range(args.warmup):
        step(k)
    e2e = run(step, args.steps)

    # the same clips fed device-resident (decoded + transformed once up front)
    resident = []
    for datas, _ in files:
        x, _ = tf(dec.decode_batch(datas))
        resident.append(x.clone())

    def step_res(k):
        comp.evaluate_batch(resident[k % len(files)], targets, gts[k % len(files)])
    for k in range(args.warmup):
        step_res(k)
    res = run(step_res, args.steps)

    # decode + transform alone on the decode stream
    def step_dec(k):
        with torch.cuda.stream(dstream):
            tf(dec.decode_batch(files[k % len(files)][0]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step_dec(k)
    torch.cuda.synchronize()
    dec_only = time.perf_counter() - t0

    # reference host path per core: PIL decode + resize + ToTensor / Normalize
    mean = torch.tensor(frames.IMAGE_MEAN_VALUE)[:, None, None]
    std = torch.tensor(frames.IMAGE_STD_VALUE)[:, None, None]
    n, t0 = 0, time.perf_counter()
    datas = files[0][0]
    while time.perf_counter() - t0 < 5.0:
        with Image.open(io.BytesIO(datas[n % len(datas)])) as im:
            a = np.array(im.convert("RGB").resize((224, 224), Image.BILINEAR))
        torch.from_numpy(a).permute(2, 0, 1).float().div(255).sub_(mean).div_(std)
        n += 1
    host = n / (time.perf_counter() - t0)

    nf = args.frames * args.steps
    print(json.dumps({
        "metric": "frames/s CAM+bbox from JPEG files, ResNet50-TCAM 224, 1x MI355X",
        "value": round(nf / e2e, 2), "unit": "frames/s",
        "ms_per_clip": round(e2e / args.steps * 1e3, 3),
        "resident_frames_per_s": round(nf / res, 2),
        "decode_transform_only_frames_per_s": round(nf / dec_only, 2),
        "host_reference_path_frames_per_s_per_core": round(host, 1),
        "bytes_per_frame": int(np.mean([len(d) for f, _ in files for d in f])),
        "config": {"workload": "configs[1] fed from files", "frames_per_clip": args.frames,
                   "frame": "360x480 JPEG q%d 4:2:0 (synthetic YTO-shaped clips)" % args.quality,
                   "clips": args.clips, "steps": args.steps, "fwd_streams": 2},
        "data": "synthetic"}))


if __name__ == "__main__":
    main()
