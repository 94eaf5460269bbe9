"""Time the HIP permutohedral filter (32-frame 224x224 clip, K=2, TCAM sigmas) against
the reference CPU filter (oracle/_ref, OpenMP over frames) on the same inputs."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd import crf  # noqa: E402


def main():
    n, k, h, w = int(os.environ.get("N", 32)), 2, 224, 224
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:h, 0:w]
    imgs = []
    for i in range(n):
        base = 128 + 100 * np.sin((xx + 2 * i) / 17.0) * np.cos(yy / 23.0)
        imgs.append(np.stack([base, 0.7 * base + 30, 255 - base], 0))
    img = (np.stack(imgs) + rng.normal(0, 6, (n, 3, h, w))).clip(0, 255).astype(np.float32)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    gi, gs = torch.from_numpy(img).to(dev), torch.from_numpy(seg).to(dev)
    for _ in range(3):
        out = crf.bilateral_filter(gi, gs, 15.0, 100.0)
    torch.cuda.synchronize()
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = crf.bilateral_filter(gi, gs, 15.0, 100.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res = {"kernel": "bilateral (permutohedral, d=5)", "frames": n, "K": k, "HxW": [h, w],
           "ms_per_call": round(ms, 4), "frames_per_s": round(n / ms * 1e3, 1),
           "algorithmic_bytes": 4 * h * w * (3 + 2 * k) * n,
           "achieved_GBps": round(4 * h * w * (3 + 2 * k) * n / ms / 1e6, 1)}
    try:
        from oracle import crf_ref as R
        if R.ref_available():
            cores = len(os.sched_getaffinity(0))
            ref = R.ref_bilateral(img[:2], seg[:2], 15.0, 100.0)
            t = time.perf_counter()
            ref = R.ref_bilateral(img, seg, 15.0, 100.0)
            dt = time.perf_counter() - t
            res["cpu_reference_ms"] = round(dt * 1e3, 2)
            res["cpu_threads"] = min(cores, n, int(os.environ.get("OMP_NUM_THREADS", cores)))
            res["bitexact_vs_reference"] = bool(np.array_equal(out.cpu().numpy(), ref))
    except Exception as ex:  # noqa: BLE001
        res["cpu_reference_error"] = str(ex)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
