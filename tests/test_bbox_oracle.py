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
