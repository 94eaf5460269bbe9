"""Phase stamps of the CRF lattice build (bilateral.hip): per merge block, the time to build the
part's LDS table (pass 1), place its vertices (global inserts), and walk the items in tile
order; per scatter block, the loads, the in-tile sort and the placement; on the bench clip
(32 frames 224^2, TCAM sigmas).

    python scripts/diag_crf_merge.py      (GPU)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd import _lib, crf  # noqa: E402


def main():
    n, k, h, w = int(os.environ.get("N", 32)), 2, 224, 224
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:h, 0:w]
    imgs = [np.stack([b, 0.7 * b + 30, 255 - b], 0) for b in
            (128 + 100 * np.sin((xx + 2 * i) / 17.0) * np.cos(yy / 23.0) for i in range(n))]
    img = (np.stack(imgs) + rng.normal(0, 6, (n, 3, h, w))).clip(0, 255).astype(np.float32)
    gi = torch.from_numpy(img).to(dev)
    gs = torch.rand(n, k, h, w, device=dev)
    lib = _lib.load()
    tiles = -(-((h * w + (1 if (h * w) % 4 else 0)) * 6) // 4096)
    dbg = torch.zeros(n * 8 * 4 + n * tiles * 4, dtype=torch.int64, device=dev)
    for _ in range(3):
        crf.bilateral_filter(gi, gs, 15.0, 100.0)
    lib.tcam_bilateral_set_debug(dbg.data_ptr())
    crf.bilateral_filter(gi, gs, 15.0, 100.0)
    torch.cuda.synchronize()
    lib.tcam_bilateral_set_debug(None)
    allst = dbg.view(-1, 4).cpu().numpy().astype(np.float64) / 100.0   # us (100 MHz)
    st, sc = allst[: n * 8], allst[n * 8:]
    t0 = st[:, 0].min()
    ph = np.diff(st, axis=1)
    out = {"blocks": int(st.shape[0]), "span_us": round(st[:, 3].max() - t0, 1),
           "start_spread_us": round(st[:, 0].max() - t0, 1)}
    for i, nm in enumerate(["table", "vertices", "walk"]):
        out[nm + "_us"] = {"median": round(float(np.median(ph[:, i])), 2),
                           "max": round(float(ph[:, i].max()), 2)}
    ph = np.diff(sc, axis=1)
    out["scatter_blocks"] = int(sc.shape[0])
    out["scatter_span_us"] = round(sc[:, 3].max() - sc[:, 0].min(), 1)
    for i, nm in enumerate(["load", "sort", "place"]):
        out["scatter_" + nm + "_us"] = {"median": round(float(np.median(ph[:, i])), 2),
                                         "max": round(float(ph[:, i].max()), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
