"""CPU: the OpenCV findContours restatement (oracle/contours.c) on analytic
known-answer tests, and the GPU bbox characterisation (tests/bbox_emul.py,
implemented by csrc/bbox.hip) against that oracle on random images.

cv2 is absent from this image: these KATs are derived by hand from
OpenCV's documented semantics (wsol_metrics.py:127-197 calls), so the
OpenCV boundary itself is "parity unpinned" (DESIGN.md)."""
import numpy as np
import pytest
from scipy import ndimage

import bbox_emul as E
from oracle import bbox_ref as B


def _one(img):
    return B.find_contours(np.asarray(img, np.uint8), with_points=True)


def test_rectangle():
    z = np.zeros((6, 7), np.uint8)
    z[1:4, 2:6] = 1
    (c,) = _one(z)
    assert c["area"] == 6.0 and c["rect"] == (2, 1, 4, 3) and not c["is_hole"]
    # OpenCV outer contours start at the top-left pixel and go down first.
    assert c["points"].tolist() == [[2, 1], [2, 3], [5, 3], [5, 1]]


def test_ring_has_hole_contour():
    z = np.zeros((5, 5), np.uint8)
    z[1:4, 1:4] = 1
    z[2, 2] = 0
    cs = _one(z)
    assert [c["is_hole"] for c in cs] == [False, True]
    assert cs[0]["area"] == 4.0 and cs[1]["area"] == 2.0 and cs[1]["parent"] == 0


def test_line_and_point_have_zero_area():
    z = np.zeros((3, 6), np.uint8)
    z[1, 1:5] = 1
    (c,) = _one(z)
    assert c["area"] == 0.0 and c["rect"] == (1, 1, 4, 1)
    z = np.zeros((3, 3), np.uint8)
    z[1, 1] = 1
    (c,) = _one(z)
    assert c["area"] == 0.0 and c["rect"] == (1, 1, 1, 1)


def test_l_shape_half_area():
    z = np.zeros((4, 4), np.uint8)
    z[1, 1] = z[1, 2] = z[2, 2] = 1
    (c,) = _one(z)
    assert c["area"] == 0.5


def test_list_order_is_reverse_discovery():
    # two equal blobs: the later-discovered (right) one is listed first, so
    # max(contours, key=contourArea) picks it.
    z = np.zeros((6, 10), np.uint8)
    z[1:3, 1:3] = 1
    z[1:3, 6:8] = 1
    cs = _one(z)
    assert cs[0]["rect"][0] == 6 and cs[1]["rect"][0] == 1
    u8 = z * 200
    boxes, n = B.compute_bboxes_from_scoremaps(u8 / 255.0, [0.5])
    assert boxes[0].tolist() == [[6, 1, 8, 3]]


def test_empty_and_full():
    sm = np.zeros((8, 8))
    boxes, n = B.compute_bboxes_from_scoremaps(sm, [0.0, 0.5])
    assert [b.tolist() for b in boxes] == [[[0, 0, 0, 0]], [[0, 0, 0, 0]]] and n == [1, 1]
    sm = np.ones((8, 8))
    boxes, _ = B.compute_bboxes_from_scoremaps(sm, [0.0])
    # boundingRect w=8 -> x1 = 0 + 8 clamped to W-1 (wsol_metrics.py:175-178)
    assert boxes[0].tolist() == [[0, 0, 7, 7]]


def test_bigger_contour_area_not_pixel_count():
    # blob A: 3x3 square (area 4); blob B: 1x12 line (12 pixels, area 0)
    z = np.zeros((8, 16), np.uint8)
    z[1:4, 1:4] = 1
    z[6, 2:14] = 1
    boxes = B.boxes_for_levels(z * 255, np.array([0]))
    assert boxes[0].tolist() == [1, 1, 4, 4]


def test_tau_truncation():
    sm = np.zeros((10, 10))
    sm[2:5, 2:5] = 0.5  # u8 = 127
    sm[6:8, 6:8] = 1.0  # u8 = 255
    taus = list(np.arange(0, 1, 0.001))
    boxes, _ = B.compute_bboxes_from_scoremaps(sm, taus)
    u8 = (sm * 255).astype(np.uint8)
    for t, b in zip(taus, boxes):
        thr = int(t * np.max(u8))
        exp = [2, 2, 5, 5] if thr < 127 else [6, 6, 8, 8]
        assert b.tolist() == [exp], (t, thr)


@pytest.mark.parametrize("kind", ["noise", "smooth", "binary", "rings"])
def test_gpu_characterisation_matches_oracle(kind):
    rng = np.random.default_rng({"noise": 1, "smooth": 2, "binary": 3, "rings": 4}[kind])
    for _ in range(40):
        H, W = int(rng.integers(2, 36)), int(rng.integers(2, 36))
        if kind == "noise":
            u8 = rng.integers(0, 256, (H, W)).astype(np.uint8)
        elif kind == "smooth":
            f = ndimage.gaussian_filter(rng.random((H, W)), 1.5)
            u8 = (255 * f / (f.max() + 1e-12)).astype(np.uint8)
        elif kind == "binary":
            u8 = ((rng.random((H, W)) < 0.55) * 255).astype(np.uint8)
        else:
            yy, xx = np.mgrid[:H, :W]
            r = np.hypot(yy - H / 2, xx - W / 2)
            u8 = ((np.sin(r * rng.uniform(0.5, 2)) + 1) * 127).astype(np.uint8)
        levels = np.arange(256)
        np.testing.assert_array_equal(B.boxes_for_levels(u8, levels),
                                      E.boxes_for_levels(u8, levels))


def test_iou_matches_reference_formula():
    a = np.array([[0, 0, 9, 9], [5, 5, 5, 5], [3, 0, 2, 9]])
    b = np.array([[0, 0, 4, 4], [20, 20, 30, 30]])
    iou = B.calculate_multiple_iou(a, b)
    assert iou[0, 0] == 25 / 100 and iou[0, 1] == 0.0 and iou[1, 0] == 0.0
    assert B.calculate_multiple_iou(np.array([[2, 2, 4, 4]]), np.array([[3, 3, 6, 6]]))[0, 0] == 4 / (9 + 16 - 4)


# ---------------------------------------------------------------- BoxAcc v2 (multi-contour)
# compute_bboxes_from_scoremaps(multi_contour_eval=True), wsol_metrics.py:162-181 — the
# characterisation csrc/bbox_multi.hip computes, pinned against the border follower.

def _multi_char(img):
    """Every contour's (clamped) box as bbox_multi.hip derives it, plus its record
    (is_hole, key, parent key): 8-connected foreground components, and 4-connected
    background components not touching the frame grown by one pixel."""
    H, W = img.shape
    s8, s4 = np.ones((3, 3), int), ndimage.generate_binary_structure(2, 1)
    fl, _ = ndimage.label(img, structure=s8)
    bl, _ = ndimage.label(~img, structure=s4)
    flat = np.arange(H * W).reshape(H, W)
    recs, fkey, bkey, bhole = [], {}, {}, {}
    for k, sl in enumerate(ndimage.find_objects(fl), 1):
        key = int(flat[fl == k].min())
        fkey[k] = key
        y0, y1, x0, x1 = sl[0].start, sl[0].stop - 1, sl[1].start, sl[1].stop - 1
        recs.append([0, key, None, x0, y0, min(x1 + 1, W - 1), min(y1 + 1, H - 1)])
    for k, sl in enumerate(ndimage.find_objects(bl), 1):
        key = int(flat[bl == k].min())
        bkey[k] = key
        y0, y1, x0, x1 = sl[0].start, sl[0].stop - 1, sl[1].start, sl[1].stop - 1
        bhole[k] = not (y0 == 0 or x0 == 0 or y1 == H - 1 or x1 == W - 1)
        if bhole[k]:
            recs.append([1, key, None, x0 - 1, y0 - 1, min(x1 + 2, W - 1), min(y1 + 2, H - 1)])
    for r in recs:
        y, x = divmod(r[1], W)
        if r[0]:
            r[2] = fkey[fl[y, x - 1]]
        else:
            r[2] = -1 if x == 0 else (bkey[bl[y, x - 1]] if bhole[bl[y, x - 1]] else -1)
    return np.asarray(recs, dtype=np.int64).reshape(-1, 7)


def _random_masks(n, seed, max_hw=28):
    rng = np.random.default_rng(seed)
    for it in range(n):
        H, W = int(rng.integers(1, max_hw)), int(rng.integers(1, max_hw))
        if it % 3 == 0:
            yield ndimage.gaussian_filter(rng.random((H, W)), 1.0) > rng.random() * 0.6 + 0.2
        else:
            yield rng.random((H, W)) < rng.random()


def test_multi_contour_boxes_and_order_characterisation():
    """The box multiset of every findContours(RETR_TREE) contour = foreground components'
    boxes + holes' boxes grown by one; OpenCV's list order = the pre-order of the tree of
    first-pixel keys (siblings by decreasing key) — metrics.opencv_contour_order, the host
    half of the device's compatibility list."""
    from tcam_wsol_video_amd.metrics import opencv_contour_order
    for img in _random_masks(2500, seed=3):
        ref = B.contour_boxes(img)
        if not img.any():
            assert ref.tolist() == [[0, 0, 0, 0]]
            continue
        recs = _multi_char(img)
        rec8 = np.zeros((len(recs), 8), np.int64)
        rec8[:, :7] = recs
        np.testing.assert_array_equal(opencv_contour_order(rec8), ref)


def _kat(img):
    return B.contour_boxes(np.asarray(img, dtype=bool)).tolist()


def test_multi_contour_kats():
    # two blobs: both boxes, the later-discovered (lower) one first
    img = np.zeros((8, 10), bool)
    img[1:3, 1:4] = True
    img[5:7, 5:9] = True
    assert _kat(img) == [[5, 5, 9, 7], [1, 1, 4, 3]]
    # a ring: its outer box, then its hole's (the hole's border pixels 2..6, x + w = 7)
    ring = np.zeros((9, 9), bool)
    ring[1:8, 1:8] = True
    ring[3:6, 3:6] = False
    assert _kat(ring) == [[1, 1, 8, 8], [2, 2, 7, 7]]
    # nested: a blob inside the ring's hole follows the hole
    nest = ring.copy()
    nest[4, 4] = True
    assert _kat(nest) == [[1, 1, 8, 8], [2, 2, 7, 7], [4, 4, 5, 5]]
    # a frame-filling image: the clamp at W-1 / H-1
    assert _kat(np.ones((5, 6), bool)) == [[0, 0, 5, 4]]
    # nothing set: [0, 0, 0, 0], one box
    boxes, n = B.compute_bboxes_from_scoremaps(np.zeros((6, 6)), [0.0, 0.5], True)
    assert [b.tolist() for b in boxes] == [[[0, 0, 0, 0]]] * 2 and n == [1, 1]


def test_multi_contour_evaluator_takes_the_best_box():
    """BoxEvaluator.accumulate with multi_contour_eval (wsol_metrics.py:342-368): a tau is
    correct when ANY contour's box reaches the IoU threshold, where the largest-contour
    rule may pick another box."""
    sm = np.zeros((20, 20))
    sm[1:4, 1:4] = 0.9          # small bright blob: the GT
    sm[8:18, 8:18] = 0.5        # large dimmer blob: the largest contour at low tau
    gt = np.array([[1, 1, 3, 3]])
    taus = [0.0, 0.5, 0.6]
    one = B.BoxEvaluatorRef(taus)
    multi = B.BoxEvaluatorRef(taus, multi_contour_eval=True)
    for ev in (one, multi):
        ev.accumulate(sm, gt, 1, np.array([1, 0]))
    # tau 0 / 0.5: both blobs set; single picks the large one, multi finds the GT blob
    assert one.num_correct[50].tolist() == [0, 0, 1]
    assert multi.num_correct[50].tolist() == [1, 1, 1]
