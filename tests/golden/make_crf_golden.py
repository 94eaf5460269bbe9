"""Generate tests/golden/crf_bilateral.npz: inputs and outputs of the REFERENCE
bilateral filters (oracle/_ref, compiled from /root/reference's own
crf/crfwrapper sources by oracle/Makefile).  Run here (the reference is absent
on the GPU box):  python tests/golden/make_crf_golden.py"""
import os
import sys
sys.dont_write_bytecode = True  # nothing may be written under /root/reference

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import crf_ref as R  # noqa: E402

CASES = [  # name, N, K, H, W, sigma_rgb, sigma_xy, kind (xy | colorD)
    ("a", 2, 2, 24, 20, 15.0, 100.0, "xy"),
    ("b", 1, 3, 13, 11, 5.0, 4.0, "xy"),       # P % 4 != 0: zero-feature padding vertices
    ("c", 1, 2, 16, 16, 15.0, 0, "color3"),
    ("d", 1, 1, 9, 7, 8.0, 0, "color1"),
]


def case_inputs(name, n, k, h, w):
    rng = np.random.default_rng(ord(name))
    yy, xx = np.mgrid[0:h, 0:w]
    base = 128 + 90 * np.sin(xx / 5.0) * np.cos(yy / 7.0)
    img = np.stack([base, 255 - base, base * 0.5], 0)[None].repeat(n, 0)
    img = (img + rng.normal(0, 8, img.shape)).clip(0, 255).astype(np.float32)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    return img, seg


def main():
    out = {}
    for name, n, k, h, w, sr, sx, kind in CASES:
        img, seg = case_inputs(name, n, k, h, w)
        if kind == "xy":
            res = R.ref_bilateral(img, seg, sr, sx)
        else:
            res = R.ref_colorbilateral(img, seg, sr, int(kind[-1]))
        out[f"{name}_img"], out[f"{name}_seg"], out[f"{name}_out"] = img, seg, res
        out[f"{name}_meta"] = np.array([n, k, h, w, sr, sx], np.float64)
        out[f"{name}_kind"] = np.array(kind)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                     "crf_bilateral.npz"), **out)


if __name__ == "__main__":
    main()
