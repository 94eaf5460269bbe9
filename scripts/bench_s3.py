"""Isolated timings of the S3 memory-bound kernels of the ResNet50-TCAM forward at the
bench shape (32 frames, 224^2): segmentation head, WGAP partial sums, stem max-pool,
decoder up2+resize.  GB/s = algorithmic bytes (one read of the input, one write of the
output) / kernel time (HIP events over REPS back-to-back calls).

    python scripts/bench_s3.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("B", "32"))
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    x = ops.s3_from_nchw(torch.randn(B, 16, 224, 224, device=dev, generator=g))
    w, b = torch.randn(2, 16, 3, 3, device=dev), torch.randn(2, device=dev)
    ms = timed(lambda: ops.seghead_cam_s3(x, w, b))
    byt = B * 224 * 224 * (16 * 6 + 2 * 4 + 4 + 1)
    res["seghead 16ch 224^2"] = (ms, byt)
    x = ops.s3_from_nchw(torch.randn(B, 2048, 28, 28, device=dev, generator=g))
    fw, fb = torch.randn(200, 2048, device=dev), torch.randn(200, device=dev)
    ms = timed(lambda: ops.wgap_s3(x, fw, fb))
    res["wgap 2048ch 28^2"] = (ms, B * 2048 * 784 * 6)
    x = ops.s3_from_nchw(torch.randn(B, 64, 112, 112, device=dev, generator=g))
    ms = timed(lambda: ops.maxpool3x3s2_s3(x))
    res["maxpool 64ch 112^2"] = (ms, B * 64 * (112 * 112 + 56 * 56) * 6)
    x = ops.s3_from_nchw(torch.randn(B, 2048, 28, 28, device=dev, generator=g))
    ms = timed(lambda: ops.up2_resize_s3(x, (28, 28)))
    res["up2_resize 2048ch 28^2"] = (ms, B * 2048 * 784 * 12)
    x = ops.s3_from_nchw(torch.randn(B, 256, 28, 28, device=dev, generator=g))
    ms = timed(lambda: ops.up2_resize_s3(x, (56, 56)))
    res["up2_resize 256ch 28->56"] = (ms, B * 256 * (784 + 3136) * 6)
    for k, (ms, byt) in res.items():
        print(json.dumps({"kernel": k, "us": round(ms * 1e3, 1),
                          "GB_per_s": round(byt / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
