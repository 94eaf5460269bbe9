"""Diagnostic: where a short (20-step) headline run loses against a long one — host enqueue
time per clip, and the per-clip GPU completion times of the pipelined loop."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tcam_wsol_video_amd.inference import CAMComputer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402


def main():
    dev = torch.device("cuda")
    model = build_r50_tcam(seed=0).to(dev)
    x, t, g = (a.to(dev) for a in bench.make_clip(32, seed=1000))
    comp = CAMComputer(model, cam_curve_interval=0.001, device=dev, fwd_streams=2)
    for _ in range(5):
        comp.evaluate_batch(x, t, g)
    comp.synchronize()
    torch.cuda.synchronize()
    for steps in (20, 20, 100):
        evs = []
        t0 = time.perf_counter()
        host = []
        for _ in range(steps):
            h0 = time.perf_counter()
            comp.evaluate_batch(x, t, g)
            host.append(time.perf_counter() - h0)
            e = torch.cuda.Event(enable_timing=True)
            e.record(comp.fwds[(comp._k - 1) % len(comp.fwds)])
            evs.append(e)
        t_enq = time.perf_counter() - t0
        e_end = torch.cuda.Event(enable_timing=True)
        comp.synchronize()
        e_end.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gaps = [evs[0].elapsed_time(e) for e in evs] + [evs[0].elapsed_time(e_end)]
        print(f"steps {steps}: {32 * steps / dt:.1f} frames/s, wall {dt * 1e3:.2f} ms, host enqueue "
              f"{t_enq * 1e3:.2f} ms ({1e3 * sum(host) / steps:.2f} ms/clip, first "
              f"{1e3 * host[0]:.2f}), fwd done t(k)-t(0) ms: "
              f"{[round(v, 2) for v in gaps[:4]]} ... last fwd {gaps[-2]:.2f}, end {gaps[-1]:.2f}",
              flush=True)


if __name__ == "__main__":
    main()
