"""CPU restatement of the reference's frame transforms (TEST INFRASTRUCTURE ONLY: the
checker of tcam_wsol_video_amd.frames, never the product path).

Reference: datasets/wsol_loader.py:903-908 (get_eval_tranforms: Resize((s, s)) ->
ToTensor -> Normalize(_IMAGE_MEAN_VALUE, _IMAGE_STD_VALUE), :46-47) and :960-970 (train:
Resize -> RandomCrop -> RandomHorizontalFlip -> ToTensor -> Normalize); raw_img
= np.array(resized, float32) (:603-606).  Resize is torchvision 0.12's TF.resize on a PIL
image, i.e. Pillow's Image.resize(size, BILINEAR) (third-party; the resample algorithm is
Pillow's src/libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc,
ImagingResampleHorizontal_8bpc / Vertical_8bpc), restated here in numpy integer
arithmetic.  Pinned against Pillow itself (importable in this image) in
tests/test_frames_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
MEAN = [0.485, 0.456, 0.406]   # wsol_loader.py:46
STD = [0.229, 0.224, 0.225]    # wsol_loader.py:47


def _bilinear(x: float) -> float:
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def resample_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs (BILINEAR, box [0, in_size)) + normalize_coeffs_8bpc.
    Returns (bounds (out, 2) int32 [xmin, n], kk (out, ksize) int32)."""
    in0, in1 = np.float32(0.0), np.float32(in_size)
    scale = float(in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = float(in0) + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for w in k:
            ww += w
        if ww != 0.0:
            k = [w / ww for w in k]
        bounds[xx] = (xmin, xmax)
        for x, w in enumerate(k):
            v = w * (1 << PRECISION_BITS)
            kk[xx, x] = int(-0.5 + v) if w < 0 else int(0.5 + v)
    return bounds, kk


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255)


def resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """(H, W, 3) uint8 -> (out_h, out_w, 3) uint8, Pillow's two-pass BILINEAR resample."""
    h, w, _ = img.shape
    bh, kh = resample_coeffs(w, out_w)
    bv, kv = resample_coeffs(h, out_h)
    src = img.astype(np.int64)
    half = 1 << (PRECISION_BITS - 1)
    tmp = np.empty((h, out_w, 3), np.int64)
    for xx in range(out_w):
        xmin, n = bh[xx]
        tmp[:, xx] = _clip8(half + (src[:, xmin:xmin + n] * kh[xx, :n, None]).sum(1))
    out = np.empty((out_h, out_w, 3), np.int64)
    for yy in range(out_h):
        ymin, n = bv[yy]
        out[yy] = _clip8(half + (tmp[ymin:ymin + n] * kv[yy, :n, None, None]).sum(0))
    return out.astype(np.uint8)


def to_tensor_normalize(u8: np.ndarray) -> np.ndarray:
    """(H, W, 3) uint8 -> (3, H, W) float32: ToTensor (x / 255) then Normalize, in fp32."""
    x = np.ascontiguousarray(u8.transpose(2, 0, 1)).astype(np.float32) / np.float32(255.0)
    m = np.asarray(MEAN, np.float32)[:, None, None]
    s = np.asarray(STD, np.float32)[:, None, None]
    return ((x - m) / s).astype(np.float32)


def transform(img: np.ndarray, resize: int, crop: int, top: int = 0, left: int = 0,
              flip: bool = False):
    """Resize((resize, resize)) -> crop (top, left, crop, crop) -> hflip -> (norm, raw)."""
    r = resize_bilinear(img, resize, resize)[top:top + crop, left:left + crop]
    if flip:
        r = r[:, ::-1]
    r = np.ascontiguousarray(r)
    return to_tensor_normalize(r), np.ascontiguousarray(r.transpose(2, 0, 1)).astype(np.float32)
