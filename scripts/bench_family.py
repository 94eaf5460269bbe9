"""Per-config throughput of the other TCAM families on 1 MI355X (BASELINE.json configs[3],
configs[4] at one GPU): CAM+bbox frames/s with HIP-event conv roofline.

  vgg16:       VGG16-TCAM, 32-frame 224x224 clip, CAM+bbox + CRF bilateral filter of
               the clip's softmaxed fcams (DenseCRFLoss energy, TCAM sigmas 15/100)
  inceptionv3: InceptionV3-TCAM, 8-frame 299x299 shard (64-frame clip / 8 GPUs), CAM+bbox
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tcam_wsol_video_amd import crf, ops  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_inceptionv3_tcam, build_vgg16_tcam  # noqa: E402

GFLOP = {"vgg16": 124.22, "inceptionv3": 101.76}   # SURVEY.md §8d (2 x MAC)


def run(name, frames, size, steps=10, warmup=2):
    dev = torch.device("cuda:0")
    model = (build_vgg16_tcam if name == "vgg16" else build_inceptionv3_tcam)(seed=0).to(dev)
    x, targets, gt = bench.make_clip(frames, seed=1000, size=size)
    xd, td, gd = x.to(dev), targets.to(dev), gt.to(dev)
    raw = ((x * torch.tensor(bench.IMNET_STD)[None, :, None, None] +
            torch.tensor(bench.IMNET_MEAN)[None, :, None, None]) * 255).clamp(0, 255).to(dev)
    comp = CAMComputer(model, cam_curve_interval=0.001, device=dev,
                       keep_fcams=(name == "vgg16"), fwd_streams=2)
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
    timer = []
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    ops.set_launch_timer(timer)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    comp.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ops.set_launch_timer(None)
    # the PMC traffic file is the ResNet50 bench's: not reported for the other families
    roof = bench.roofline_from_timer(timer, base, steps, "x6", dt / steps * 1e3, with_traffic=False)
    return {"workload": f"{name}-TCAM CAM+bbox{' + CRF filter' if name == 'vgg16' else ''}, "
                        f"{size}x{size}", "frames_per_step": frames,
            "frames_per_s": round(frames * steps / dt, 1),
            "ms_per_step": round(dt / steps * 1e3, 3),
            "gflop_per_frame": GFLOP[name], "roofline": roof}


def main():
    out = [run("vgg16", 32, 224), run("inceptionv3", 8, 299)]
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
