"""TEST INFRASTRUCTURE ONLY: numpy restatement of the TCAM pseudo-label seeder.

Restates (reference paths relative to sbelharbi/tcam-wsol-video):
  TCAMSeeder.forward / use_all_roi   dlib/cams/tcam_seeding.py:187-300
  GetRoiSingleCam.__call__/get_thresh dlib/cams/tcam_seeding.py:303-406
  _OneSample / _SFG / _SBG           dlib/cams/tcam_seeding.py:409-592
and the third-party algorithms they call (absent from this image, restated from
the versions pinned in dependencies/requirements.txt):
  skimage 0.17.2 ``filters.threshold_otsu`` over ``exposure.histogram`` (numpy
    1.21.5 ``np.histogram`` on a float32 image: float32 linspace edges, float32
    ``(a - first) * norm`` bin index with the +-1 edge corrections, float32 bin
    centres), ``measure.label(connectivity=1)`` (4-connected, labels numbered in
    raster order of each component's first pixel);
  kornia 0.6.4 ``morphology.erosion`` / ``dilation`` with an all-ones k x k
    structuring element (geodesic border: out-of-image pixels are ignored;
    origin (k//2, k//2));
  torch ``multinomial(p, k, replacement=False)``, which torch implements as
    ``topk(p / q, k)`` with q ~ Exp(1) (ATen/native/Distributions.cpp, the
    no-replacement fast path).  The q stream here is a counter-based Philox4x32-10
    keyed like the device kernel, so the sampled SETS are comparable bit for bit;
    the distribution is pinned to torch.multinomial by a statistical test.

Numerics follow numpy 1.21.5 value-based casting: a float32 array compared with
a float64 scalar is compared in float32 (the threshold is cast to float32).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
from scipy import ndimage

ROI_ALL = "roi_all"
ROI_H_DENSITY = "roi_high_density"
ROI_LARGEST = "largest"
SEED_UNIFORM = "seed_uniform"
SEED_WEIGHTED = "seed_weighted"

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al. 2011) over uint32 arrays -> 4 uint32 arrays."""
    c = [np.asarray(v, dtype=np.uint32).copy() for v in (c0, c1, c2, c3)]
    c = np.broadcast_arrays(*c)
    c = [v.astype(np.uint32) for v in c]
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = c[0].astype(np.uint64) * _M0
            p1 = c[2].astype(np.uint64) * _M1
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c


def exp_noise(frame: int, hw: int, seed: int, offset: int, lane: int) -> np.ndarray:
    """q ~ Exp(1) per pixel: u = (x + 0.5) 2^-32 from Philox lane ``lane``
    (0 = foreground draw, 1 = background draw), q = -log(u) in float64."""
    pix = np.arange(hw, dtype=np.uint32)
    out = philox4x32(pix, np.uint32(frame), np.uint32(offset & 0xFFFFFFFF),
                     np.uint32(offset >> 32), seed & 0xFFFFFFFF, seed >> 32)
    u = (out[lane].astype(np.float64) + 0.5) * (2.0 ** -32)
    return -np.log(u)


# ---------------------------------------------------------------------------
# Otsu threshold (GetRoiSingleCam.get_thresh, tcam_seeding.py:399-406)
# ---------------------------------------------------------------------------

def otsu_threshold(cam: np.ndarray) -> np.float32:
    """get_thresh: floor(cam * 255.) in float32, 0 if flat, else skimage 0.17.2
    threshold_otsu(nbins=256) over numpy 1.21.5's float32 histogram."""
    cam_ = np.floor(cam.astype(np.float32) * np.float32(255.0))
    if float(cam_.min()) == float(cam_.max()):
        return np.float32(0.0)
    return skimage_otsu(cam_)


def skimage_otsu(cam_: np.ndarray, nb: int = 256) -> np.float32:
    """skimage 0.17.2 threshold_otsu on a float32 image (numpy 1.21.5 histogram)."""
    cam_ = cam_.astype(np.float32)
    mn, mx = float(cam_.min()), float(cam_.max())
    # np.linspace(first, last, 257) in float64, cast to the bin dtype (float32)
    step = (mx - mn) / nb
    edges = (np.arange(nb + 1, dtype=np.float64) * step + mn)
    edges[-1] = mx
    edges = edges.astype(np.float32)
    norm = np.float32(nb / (mx - mn))
    a = cam_.ravel()
    f = (a - np.float32(mn)) * norm                      # float32
    idx = f.astype(np.intp)
    idx[idx == nb] -= 1
    idx[a < edges[idx]] -= 1
    inc = (a >= edges[idx + 1]) & (idx != nb - 1)
    idx[inc] += 1
    hist = np.bincount(idx, minlength=nb).astype(np.float64)
    centers = (edges[:-1] + edges[1:]) / np.float32(2.0)  # float32
    w1 = np.cumsum(hist)
    w2 = np.cumsum(hist[::-1])[::-1]
    hc = hist * centers.astype(np.float64)
    m1 = np.cumsum(hc) / w1
    m2 = (np.cumsum(hc[::-1]) / w2[::-1])[::-1]
    var12 = w1[:-1] * w2[1:] * (m1[:-1] - m2[1:]) ** 2
    return centers[:-1][int(np.argmax(var12))]


def label4(blobs: np.ndarray) -> Tuple[np.ndarray, int]:
    """skimage.measure.label(connectivity=1, background=0): raster-order labels."""
    lab, n = ndimage.label(blobs, structure=[[0, 1, 0], [1, 1, 1], [0, 1, 0]])
    return lab, n


def get_roi(cam: np.ndarray, roi_method: str, p_min_area_roi: float,
            thresh: Optional[float] = None):
    """GetRoiSingleCam.__call__ (tcam_seeding.py:312-396) ->
    (final_roi int64 (h,w), bbox_mask float32 (h,w), bbox int64 (1,4))."""
    cam = cam.astype(np.float32)
    h, w = cam.shape
    if thresh is None:
        th = otsu_threshold(cam)
    else:
        th = np.float32(thresh * 255.0)
    blobs = (cam * np.float32(255.0) >= th).astype(np.int64)
    bbox = np.array([0, 0, h - 1, w - 1]).reshape(1, 4)
    if roi_method == ROI_ALL:
        final = blobs
    else:
        lab, n = label4(blobs)
        nlab = n + (1 if (lab == 0).any() else 0)
        if nlab == 1:
            final = blobs
        else:
            min_area = (h * w) * p_min_area_roi
            dens, area = {}, {}
            cam64 = cam.astype(np.float64)
            for l in range(1, n + 1):
                s_roi = (lab == l).astype(float)
                s_cam = cam64 * s_roi
                a = s_roi.sum()
                dens[l] = s_cam.sum() / a
                area[l] = a
            if roi_method == ROI_H_DENSITY:
                l_roi = max(dens, key=dens.get)
                if area[l_roi] < min_area:
                    l_roi = max(area, key=area.get)
            elif roi_method == ROI_LARGEST:
                l_roi = max(area, key=area.get)
            else:
                raise NotImplementedError(roi_method)
            final = (lab == l_roi).astype(np.int64)
        # compute_bboxes_from_scoremaps_ext_contours(final, [0.5], multi=True)
        # on one (8-connected) component or an empty / full map: its extent.
        ys, xs = np.nonzero(final)
        if ys.size == 0:
            bbox = np.array([[0, 0, 0, 0]])
        else:
            bbox = np.array([[xs.min(), ys.min(), min(xs.max() + 1, w - 1),
                              min(ys.max() + 1, h - 1)]])
    mask = np.zeros((h, w), dtype=np.float32)
    x0, y0, x1, y1 = bbox.flatten()
    mask[y0:y1, x0:x1] = 1.0
    return final.astype(np.int64), mask, bbox.astype(np.int64)


def _morph(x: np.ndarray, k: int, op) -> np.ndarray:
    """kornia erosion/dilation, all-ones k x k kernel, geodesic border."""
    h, w = x.shape
    o = k // 2
    big = np.iinfo(np.int64).max if op is np.minimum else np.iinfo(np.int64).min
    pad = np.full((h + k - 1, w + k - 1), big, dtype=np.int64)
    pad[o:o + h, o:o + w] = x
    out = None
    for dy in range(k):
        for dx in range(k):
            v = pad[dy:dy + h, dx:dx + w]
            out = v.copy() if out is None else op(out, v)
    return out


def erode(x, k, iters):
    for _ in range(iters):
        x = _morph(x, k, np.minimum)
    return x


def dilate(x, k):
    return _morph(x, k, np.maximum) if k > 1 else x


def _select_top(vals: np.ndarray, n: int, descending: bool) -> np.ndarray:
    """torch.sort(stable=True) then the first n indices."""
    order = np.argsort(-vals if descending else vals, kind="stable")
    return order[:n]


def _sample(cand_raster: np.ndarray, probs: np.ndarray, k: int, q: np.ndarray) -> np.ndarray:
    """multinomial(probs, k, replacement=False) as topk(probs / q, k) -> pixels."""
    key = probs.astype(np.float64) / q[cand_raster]
    order = np.lexsort((cand_raster, -key))  # key desc, raster asc on ties
    return cand_raster[order[:k]]


def one_sample(cam: np.ndarray, cfg: dict, roi: Optional[np.ndarray], frame: int,
               seed: int, offset: int):
    """_OneSample.forward (tcam_seeding.py:436-467) -> (fg, bg) int64 (h, w)."""
    cam = cam.astype(np.float32)
    h, w = cam.shape
    fg = np.zeros((h, w), np.int64)
    bg = np.zeros((h, w), np.int64)
    if cam.min() == cam.max():
        return fg, bg
    _roi = None
    if cfg["use_roi"]:
        _roi = roi
        if _roi is None:
            _roi, _, _ = get_roi(cam, cfg["roi_method"], cfg["p_min_area_roi"])
        if cfg["fg_erode_iter"] > 0:
            _roi = erode(_roi.astype(np.int64), cfg["fg_erode_k"], cfg["fg_erode_iter"])
    # _SFG (tcam_seeding.py:470-521)
    if _roi is not None:
        n = int(np.float32(cfg["max_p"]) * np.float32(_roi.sum()))
        _cam = (cam * _roi.astype(np.float32)) + np.float32(1e-8)
    else:
        n = int(cfg["max_p"] * (h * w))
        _cam = cam + np.float32(1e-8)
    flat = _cam.reshape(-1)
    q_fg = exp_noise(frame, h * w, seed, offset, 0)
    q_bg = exp_noise(frame, h * w, seed, offset, 1)
    if n > 0 and cfg["max_"] > 0:
        cand = np.sort(_select_top(flat, n, True))           # torch.nonzero: raster order
        if cfg["seed_tech"] == SEED_UNIFORM:
            probs = np.ones(n, np.float32)
        else:
            probs = flat[cand]
        sel = _sample(cand, probs, min(cfg["max_"], n), q_fg)
        fg.reshape(-1)[sel] = 1
    # _SBG (tcam_seeding.py:524-563), always uniform
    n = int(cfg["min_p"] * h * w)
    flat = (cam + np.float32(1e-8)).reshape(-1)
    if n > 0 and cfg["min_"] > 0:
        cand = np.sort(_select_top(flat, n, False))
        probs = np.ones(n, np.float32)
        sel = _sample(cand, probs, min(cfg["min_"], n), q_bg)
        bg.reshape(-1)[sel] = 1
    return fg, bg


def seeder(x: np.ndarray, cfg: dict, roi: Optional[np.ndarray] = None, seed: int = 0,
           offset: int = 0) -> np.ndarray:
    """TCAMSeeder.forward (tcam_seeding.py:187-258): x (b,1,h,w) -> seeds (b,h,w) int64."""
    b, d, h, w = x.shape
    assert d == 1
    out = np.full((b, h, w), cfg["seg_ignore_idx"], np.int64)
    for i in range(b):
        r = None if roi is None else roi[i].reshape(h, w).astype(np.int64)
        fg, bg = one_sample(x[i, 0], cfg, r, i, seed, offset)
        fg = dilate(fg, cfg["ksz"])
        bg = dilate(bg, cfg["ksz"])
        both = (fg + bg) == 2
        fg[both] = 0
        bg[both] = 0
        out[i][fg == 1] = 1
        out[i][bg == 1] = 0
    return out


def use_all_roi(x: np.ndarray, roi: np.ndarray, ignore_idx: int) -> np.ndarray:
    """TCAMSeeder.use_all_roi (tcam_seeding.py:260-300)."""
    b, _, h, w = x.shape
    out = np.full((b, h, w), ignore_idx, np.int64)
    out[roi.reshape(b, h, w) == 1] = 1
    return out


def default_cfg(**kw) -> dict:
    """README.md:318-326 TCAM seeding settings (sl_tc_*)."""
    cfg = dict(seed_tech=SEED_WEIGHTED, min_=1, max_=1, max_p=0.6, min_p=0.1,
               fg_erode_k=11, fg_erode_iter=0, ksz=3, seg_ignore_idx=-255,
               roi_method=ROI_ALL, p_min_area_roi=0.05, use_roi=True)
    cfg.update(kw)
    return cfg


# ---------------------------------------------------------------------------
# Stage-1 CAM store ROI thresholds (learning/inference_wsol.py:1107-1124, 1144-1159)
# ---------------------------------------------------------------------------

def stotsu(x: np.ndarray) -> np.float32:
    """STOtsu.forward (cams/core_seeding.py:23-56) in float32 on integer-valued x:
    torch.histc(bins = max - min + 1) puts each integer in its own bin."""
    x = np.asarray(x, np.float32).ravel()
    mn, mx = np.float32(x.min()), np.float32(x.max())
    if mn == mx:
        return mn
    nb = int(mx - mn + 1)
    centers = (mn + np.arange(nb, dtype=np.float32)).astype(np.float32)
    hist = np.bincount((x - mn).astype(np.int64), minlength=nb).astype(np.float32)
    w1 = np.cumsum(hist, dtype=np.float32)
    w2 = np.cumsum(hist[::-1], dtype=np.float32)[::-1]
    hc = (hist * centers).astype(np.float32)
    m1 = (np.cumsum(hc, dtype=np.float32) / w1).astype(np.float32)
    m2 = (np.cumsum(hc[::-1], dtype=np.float32) / w2[::-1]).astype(np.float32)[::-1]
    d = (m1[:-1] - m2[1:]).astype(np.float32)
    var = ((w1[:-1] * w2[1:]).astype(np.float32) * (d * d)).astype(np.float32)
    return centers[:-1][int(np.argmax(var))]


def roi_threshold(cam: np.ndarray, size: int = 224) -> np.float32:
    """floor(F.interpolate(cam, (size, size), bilinear, align_corners=True) * 255)
    -> STOtsu, in [0, 255] (the file stores this / 255.)."""
    import torch
    import torch.nn.functional as F
    full = F.interpolate(torch.from_numpy(np.asarray(cam, np.float32))[None, None],
                         size=(size, size), mode="bilinear", align_corners=True)
    return stotsu(torch.floor(full * 255).numpy())
