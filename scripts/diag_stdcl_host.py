"""Host-side time of the stage-1 step (is the step launch-bound?): the host time of K
steps without synchronising vs the wall time to the final synchronize."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tcam_wsol_video_amd.cl_training import ClassifierTrainer  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_stdcl  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for amp in (False, True):
        model = build_r50_stdcl(seed=0).to(dev)
        x, _, _ = bench.make_clip(32, seed=3000)
        xd, yd = x.to(dev), ((torch.arange(32) * 7) % 10).to(dev)
        tr = ClassifierTrainer(model, lr=0.001, amp=amp)
        for _ in range(3):
            tr.step(xd, yd)
        torch.cuda.synchronize()
        K = 10
        t0 = time.perf_counter()
        for _ in range(K):
            tr.step(xd, yd)
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        print(f"amp={amp}: host {th / K * 1e3:.2f} ms/step, wall {tw / K * 1e3:.2f} ms/step",
              flush=True)


if __name__ == "__main__":
    main()
