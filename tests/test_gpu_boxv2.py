"""BoxAcc v2 (--box_v2_metric True -> multi_contour_eval, parseit.py:684-689) on the GPU:
every contour's box of every threshold (wsol_metrics.py:162-181), a tau scored by its best
IoU (wsol_metrics.py:342-368) — csrc/bbox_multi.hip against the oracle evaluator over the
border-following findContours restatement (oracle/contours.c): counters bit-exact on
random, smooth, KAT and full-size frames, and the compatibility lists of
compute_bboxes_from_scoremaps(multi_contour_eval=True) equal, order included."""
import numpy as np
import pytest
import torch
from scipy import ndimage

from oracle import bbox_ref as BR
from tcam_wsol_video_amd import metrics, ops
from tcam_wsol_video_amd.metrics import BoxEvaluator

pytestmark = pytest.mark.gpu


def _cams(kind, B, H, W, seed):
    rng = np.random.default_rng(seed)
    out = np.zeros((B, H, W), np.uint8)
    for b in range(B):
        if kind == "noise":
            v = rng.random((H, W))
        elif kind == "blobs":
            v = ndimage.gaussian_filter(rng.random((H, W)), max(1.0, min(H, W) / 12))
            v = (v - v.min()) / (np.ptp(v) + 1e-12)
        else:   # a few Gaussians + low noise (the bench's CAM statistics)
            yy, xx = np.mgrid[0:H, 0:W]
            v = np.zeros((H, W))
            for _ in range(int(rng.integers(2, 6))):
                cy, cx = rng.random() * H, rng.random() * W
                s = (0.05 + 0.2 * rng.random()) * max(H, W)
                v += rng.random() * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
            v = v / v.max() + 0.02 * rng.random((H, W))
            v = v / v.max()
        out[b] = np.clip(v * 255, 0, 255).astype(np.uint8)
    return out


def _gt(B, H, W, seed, G=3):
    rng = np.random.default_rng(seed)
    gt = np.zeros((B, G, 4), np.int32)
    ngt = rng.integers(1, G + 1, B).astype(np.int32)
    for b in range(B):
        for g in range(G):
            x0, x1 = sorted(rng.integers(0, W, 2))
            y0, y1 = sorted(rng.integers(0, H, 2))
            gt[b, g] = (x0, y0, x1, y1)
    return gt, ngt


def _check(u8, gt, ngt, taus, cuda):
    B = u8.shape[0]
    ev = BoxEvaluator(taus, device=cuda, multi_contour_eval=True)
    rng = np.random.default_rng(1)
    top1 = rng.integers(0, 2, B).astype(np.int32)
    top5 = np.maximum(top1, rng.integers(0, 2, B).astype(np.int32))
    best = torch.empty((B, len(taus)), dtype=torch.float64, device=cuda)
    ev.accumulate_batch(torch.from_numpy(u8).to(cuda), torch.from_numpy(gt).to(cuda),
                        torch.from_numpy(ngt).to(cuda), torch.from_numpy(top1).to(cuda),
                        torch.from_numpy(top5).to(cuda), best)
    ref = BR.BoxEvaluatorRef(taus, multi_contour_eval=True)
    for b in range(B):
        # a scoremap whose uint8 quantisation is exactly u8[b] (wsol_metrics.py:153)
        sm = np.minimum((u8[b].astype(np.float64) + 0.5) / 255.0, 1.0)
        preds = np.array([0, 1, 2, 3, 4, 5]) if top1[b] else (
            np.array([1, 2, 3, 4, 0, 5]) if top5[b] else np.array([1, 2, 3, 4, 5, 0]))
        ref.accumulate(sm, gt[b, :ngt[b]], 0, preds)
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(ev.num_correct[thr], ref.num_correct[thr])
        np.testing.assert_array_equal(ev.num_correct_top1[thr], ref.num_correct_top1[thr])
        np.testing.assert_array_equal(ev.num_correct_top5[thr], ref.num_correct_top5[thr])
    ev.cnt = ref.cnt
    assert ev.compute() == ref.compute() and ev.best_tau_list == ref.best_tau_list
    return ev, best


@pytest.mark.parametrize("kind,B,H,W", [("noise", 4, 17, 23), ("noise", 3, 64, 64),
                                        ("blobs", 6, 64, 80), ("smooth", 4, 224, 224),
                                        ("blobs", 3, 224, 224), ("smooth", 2, 299, 299),
                                        ("blobs", 2, 300, 257), ("smooth", 2, 320, 320)])
def test_multi_contour_counters_match_oracle(cuda, kind, B, H, W):
    u8 = _cams(kind, B, H, W, seed=H * 7 + W)
    gt, ngt = _gt(B, H, W, seed=H + W)
    taus = list(np.arange(0, 1, 0.001 if H == 224 else 0.01))
    _check(u8, gt, ngt, taus, cuda)


def test_multi_contour_kat_frames(cuda):
    """Multi-blob, ring (hole contour), ring with an island in its hole (nested), a frame-
    filling blob (clamp), an all-zero frame ([0,0,0,0]), a checkerboard (many contours),
    holes touching the frame (not contours)."""
    H = W = 40
    u8 = np.zeros((7, H, W), np.uint8)
    u8[0, 2:8, 3:12] = 200; u8[0, 20:35, 18:30] = 120; u8[0, 25:28, 5:9] = 250
    u8[1, 5:30, 5:30] = 180; u8[1, 12:20, 12:22] = 0
    u8[2] = u8[1]; u8[2, 15:17, 15:18] = 255
    u8[3] = 90
    u8[5, ::2, ::2] = 200; u8[5, 1::2, 1::2] = 140
    u8[6, :, :] = 170; u8[6, 0:10, 10:15] = 0; u8[6, 20:25, 20:26] = 30
    gt = np.array([[[3, 2, 11, 7], [18, 20, 29, 34], [12, 12, 21, 19]]] * 7, np.int32)
    ngt = np.array([3, 3, 3, 1, 2, 3, 3], np.int32)
    _check(u8, gt, ngt, list(np.arange(0, 1, 0.002)), cuda)


def test_compat_lists_match_oracle_in_order(cuda):
    """compute_bboxes_from_scoremaps(multi_contour_eval=True): the per-tau box lists (and
    counts) equal the oracle's, in OpenCV's list order."""
    for kind, H, W, seed in (("noise", 21, 19, 5), ("blobs", 48, 64, 6), ("smooth", 96, 96, 7)):
        u8 = _cams(kind, 1, H, W, seed)[0]
        sm = np.minimum((u8.astype(np.float64) + 0.5) / 255.0, 1.0)
        taus = list(np.arange(0, 1, 0.02))
        got, n_got = metrics.compute_bboxes_from_scoremaps(sm, taus, multi_contour_eval=True,
                                                           device=cuda)
        ref, n_ref = BR.compute_bboxes_from_scoremaps(sm, taus, multi_contour_eval=True)
        assert n_got == n_ref, kind
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)


def test_multi_contour_single_box_levels_agree_with_largest(cuda):
    """On frames whose every level is one simply connected blob, BoxAcc v2 equals the
    largest-contour BoxAcc (one contour per level)."""
    H = W = 64
    yy, xx = np.mgrid[0:H, 0:W]
    u8 = np.stack([np.clip(255 - 4 * np.hypot(yy - cy, xx - cx), 0, 255).astype(np.uint8)
                   for cy, cx in ((30, 30), (20, 40), (45, 15))])
    gt = np.array([[[20, 20, 40, 40]], [[30, 10, 50, 30]], [[5, 35, 25, 55]]], np.int32)
    ngt = np.ones(3, np.int32)
    taus = list(np.arange(0, 1, 0.01))
    cams = torch.from_numpy(u8).to(cuda)
    args = (torch.from_numpy(gt).to(cuda), torch.from_numpy(ngt).to(cuda),
            torch.ones(3, dtype=torch.int32, device=cuda),
            torch.ones(3, dtype=torch.int32, device=cuda))
    evs = []
    for multi in (False, True):
        ev = BoxEvaluator(taus, device=cuda, multi_contour_eval=multi)
        ev.accumulate_batch(cams, *args)
        evs.append(ev)
    assert torch.equal(evs[0].counters, evs[1].counters)
    assert int(evs[0].cls_correct) == 3
