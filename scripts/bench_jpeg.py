"""Frame-decode throughput: YTO-shaped 360x480 JPEG frames (Pillow
encoder, quality 90, 4:2:0 -- synthetic, no dataset on the box) decoded on the device
(tcam_jpeg_pack on the host + tcam_jpeg_decode) vs the reference's per-frame
Image.open(...).convert('RGB') on one host core.  Batches of 32 (one clip) and 256 frames
(eight clips).  Per-kernel device times from rocprofv3 when run under it.  One JSON line."""
import io
import json
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import jpeg_cases as JC  # noqa: E402
from tcam_wsol_video_amd import jpeg  # noqa: E402


def smooth(h, w, seed):
    """Natural-looking frame: a few soft colour blobs + mild sensor noise."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w, 3))
    for _ in range(6):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(20, 120)
        m = np.exp(-((y - cy) ** 2 + (x - cx) ** 2) / (2 * r * r))[..., None]
        img = img * (1 - m) + rng.uniform(0, 255, 3) * m
    img += rng.normal(0, 3, img.shape)
    return Image.fromarray(np.clip(img, 0, 255).astype(np.uint8))


def frames(n, h=360, w=480, q=90, rst=0, kind="noisy"):
    kw = dict(quality=q, subsampling=2)
    if rst:
        kw["restart_marker_rows"] = rst
    make = (lambda k: JC.frame(h, w, seed=k)) if kind == "noisy" else (lambda k: smooth(h, w, k))
    return [JC.encode(make(k), **kw) for k in range(n)]


def time_device(dec, datas, steps):
    for _ in range(3):
        dec.decode(datas)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        dec.decode(datas)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    # host pack alone
    t1 = time.perf_counter()
    for _ in range(steps):
        jpeg.JpegDecoder.plan(datas)
    plan = (time.perf_counter() - t1) / steps
    return e0.elapsed_time(e1) / steps, wall * 1e3, plan * 1e3


def main():
    dev = torch.device("cuda")
    dec = jpeg.JpegDecoder(dev)
    res = {"metric": "frames/s JPEG decode (360x480, 4:2:0) -> RGB uint8 on the device",
           "data": "synthetic frames encoded by Pillow: 'noisy' = gradient + sigma-25 noise "
                   "(worst case, ~105 KB at q90), 'smooth' = colour blobs + sigma-3 noise"}
    for kind, q, n, rst in (("noisy", 90, 32, 0), ("noisy", 90, 256, 0), ("noisy", 90, 256, 1),
                            ("smooth", 90, 32, 0), ("smooth", 90, 256, 0),
                            ("smooth", 75, 256, 0)):
        datas = frames(n, q=q, rst=rst, kind=kind)
        ms_dev, ms_wall, ms_plan = time_device(dec, datas, 20)
        key = f"{kind}_q{q}_b{n}" + ("_rst" if rst else "")
        res[key] = {"frames_per_s": round(n / ms_wall * 1e3, 1),
                    "ms_per_batch_wall": round(ms_wall, 3),
                    "ms_per_batch_stream": round(ms_dev, 3),
                    "ms_host_plan": round(ms_plan, 3),
                    "bytes_per_frame": int(np.mean([len(d) for d in datas]))}
    datas = frames(32, kind="smooth")
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 5.0:
        with Image.open(io.BytesIO(datas[n % 32])) as im:
            np.asarray(im.convert("RGB"))
        n += 1
    res["cpu_baseline"] = {"value": round(n / (time.perf_counter() - t0), 1),
                           "unit": "frames/s", "cores": 1, "kind": "reference",
                           "sample": f"{n} smooth q90 frames, Image.open(BytesIO).convert('RGB') "
                                     "(Pillow 12.2 / libjpeg-turbo), one thread"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
