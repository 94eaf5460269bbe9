"""Diagnostics of the chunk-parallel Huffman decode: self-synchronisation rounds per
workgroup and per-kernel times for noisy vs smooth 360x480 frames (q75 / q90)."""
import io, json, os, sys
import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import jpeg_cases as JC  # noqa: E402
from tcam_wsol_video_amd import _lib, jpeg  # noqa: E402


def smooth(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w, 3))
    for _ in range(6):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(20, 120)
        col = rng.uniform(0, 255, 3)
        m = np.exp(-((y - cy) ** 2 + (x - cx) ** 2) / (2 * r * r))[..., None]
        img = img * (1 - m) + col * m
    img += rng.normal(0, 3, img.shape)
    return Image.fromarray(np.clip(img, 0, 255).astype(np.uint8))


def main():
    dev = torch.device("cuda")
    dec = jpeg.JpegDecoder(dev)
    lib = _lib.load()
    out = {}
    for kind in ("noisy", "smooth"):
        for q in (75, 90):
            im = (lambda k: JC.frame(360, 480, seed=k)) if kind == "noisy" else \
                (lambda k: smooth(360, 480, k))
            datas = [JC.encode(im(k), quality=q, subsampling=2) for k in range(32)]
            dec.decode(datas)
            torch.cuda.synchronize()
            rounds = torch.zeros(4096, dtype=torch.int32, device=dev)
            nwg = lib.tcam_jpeg_debug_rounds(dec._host[dec._k ^ 1].data_ptr(), rounds.data_ptr())
            dec.decode(datas)
            torch.cuda.synchronize()
            lib.tcam_jpeg_debug_rounds(None, None)
            r4 = rounds[:4 * nwg].view(nwg, 4).cpu().numpy()
            r = r4[:, 0]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                dec.decode(datas)
            e1.record()
            torch.cuda.synchronize()
            out[f"{kind}_q{q}"] = {"bytes_per_frame": int(np.mean([len(d) for d in datas])),
                                   "workgroups": int(nwg), "rounds_max": int(r.max()),
                                   "rounds_mean": round(float(r.mean()), 2),
                                   "fix_kcycles_mean": round(float(r4[:, 1].mean()) / 1e3, 1),
                                   "write_kcycles_lane0": round(float(r4[:, 2].mean()) / 1e3, 1),
                                   "write_blocks_lane0": round(float(r4[:, 3].mean()), 1),
                                   "ms_per_32": round(e0.elapsed_time(e1) / 10, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
