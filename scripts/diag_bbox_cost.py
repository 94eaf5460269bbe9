"""Diagnostic: what the side-stream bbox stage costs the pipelined bench (same box, same
process): frames/s of bench.py's loop with and without BoxEvaluator.accumulate_batch."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402


def run(comp, x, t, g, steps=20):
    for _ in range(3):
        comp.evaluate_batch(x, t, g)
    comp.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        comp.evaluate_batch(x, t, g)
    comp.synchronize()
    torch.cuda.synchronize()
    return 32 * steps / (time.perf_counter() - t0)


def main():
    dev = torch.device("cuda")
    model = build_r50_tcam(seed=0).to(dev)
    x, t, g = (a.to(dev) for a in bench.make_clip(32, seed=1000))
    comp = CAMComputer(model, cam_curve_interval=0.001, device=dev, fwd_streams=2)
    real = comp.evaluator.accumulate_batch
    for rnd in range(2):
        comp.evaluator.accumulate_batch = real
        a = run(comp, x, t, g)
        comp.evaluator.accumulate_batch = lambda *args, **kw: None
        b = run(comp, x, t, g)
        print(f"round {rnd}: with bbox {a:.1f} frames/s, forward+CAM only {b:.1f} frames/s",
              flush=True)


if __name__ == "__main__":
    main()
