"""Frame-preprocessing throughput: a 32-frame YTO-shaped clip
(360x480 uint8 RGB, decoded) -> the reference's eval transform (Resize((224, 224))
BILINEAR, ToTensor, Normalize) + raw_img, on the device (tcam_frames_preprocess) vs the
reference's per-frame CPU path (PIL resize + torchvision-style ToTensor / Normalize, one
process).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd import frames  # noqa: E402

MEAN = torch.tensor(frames.IMAGE_MEAN_VALUE)[:, None, None]
STD = torch.tensor(frames.IMAGE_STD_VALUE)[:, None, None]


def cpu_frame(img):
    r = Image.fromarray(img).resize((224, 224), Image.BILINEAR)
    a = np.array(r)
    t = torch.from_numpy(a).permute(2, 0, 1).contiguous().float().div(255)
    return t.sub_(MEAN).div_(STD), torch.from_numpy(a.astype(np.float32)).permute(2, 0, 1)


def main():
    B, steps = 32, 50
    rng = np.random.default_rng(0)
    clip = (rng.random((B, 360, 480, 3)) * 256).astype(np.uint8)
    dev = torch.device("cuda")
    x = torch.from_numpy(clip).to(dev)
    tr = frames.get_eval_tranforms(224)
    for _ in range(3):
        tr(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        tr(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 5.0:
        cpu_frame(clip[n % B])
        n += 1
    cpu = n / (time.perf_counter() - t0)
    nbytes = clip.nbytes + 2 * B * 3 * 224 * 224 * 4
    print(json.dumps({"metric": "frames/s eval transform (360x480 -> 224, norm + raw)",
                      "value": round(B / ms * 1e3, 1), "ms_per_clip": round(ms, 4),
                      "algorithmic_GBps": round(nbytes / ms / 1e6, 1),
                      "cpu_reference_frames_per_s": round(cpu, 1),
                      "cpu_sample": f"{n} frames, PIL resize + torch ToTensor/Normalize, "
                                    f"1 process ({torch.get_num_threads()} torch threads)"}))


if __name__ == "__main__":
    main()
