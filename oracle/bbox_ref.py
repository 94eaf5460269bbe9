"""TEST INFRASTRUCTURE ONLY: CPU restatement of the CAM->bbox->BoxEvaluator path.

Restates, over oracle/contours.c (OpenCV findContours restatement):
  compute_bboxes_from_scoremaps  dlib/metrics/wsol_metrics.py:127-197
  calculate_multiple_iou         dlib/metrics/wsol_metrics.py:77-124
  BoxEvaluator.accumulate/compute dlib/metrics/wsol_metrics.py:266-433
  check_scoremap_validity        dlib/utils/wsol.py:63-78
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Dict, List, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


class oc_contour(C.Structure):
    _fields_ = [("area2", C.c_int64), ("x0", C.c_int), ("y0", C.c_int), ("x1", C.c_int),
                ("y1", C.c_int), ("is_hole", C.c_int), ("parent", C.c_int), ("npts", C.c_int)]


def build() -> str:
    """Compile oracle/contours.c (gcc) into oracle/liboracle.so."""
    src = os.path.join(HERE, "contours.c")
    if (not os.path.exists(LIB)) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", LIB, src])
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        L.oc_find_contours.restype = C.c_int
        L.oc_find_contours.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                       C.c_void_p, C.c_int]
        L.oc_contour_points.restype = C.c_int
        L.oc_contour_points.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.oc_boxes_for_thresholds.restype = C.c_int
        L.oc_boxes_for_thresholds.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                              C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def find_contours(binary: np.ndarray, with_points: bool = False) -> List[dict]:
    """cv2.findContours(binary, RETR_TREE, CHAIN_APPROX_SIMPLE) summary, in
    OpenCV output order: dicts with area (=contourArea), rect (x, y, w, h),
    is_hole, parent (output index or -1) and optionally the points."""
    b = np.ascontiguousarray(binary != 0, dtype=np.uint8)
    H, W = b.shape
    cap = H * W + 8
    arr = (oc_contour * cap)()
    pcap = 8 * H * W + 64
    pts = np.zeros(2 * pcap, dtype=np.int32) if with_points else None
    n = lib().oc_find_contours(b.ctypes.data, H, W, arr, cap,
                               None if pts is None else pts.ctypes.data,
                               0 if pts is None else pcap)
    assert n >= 0
    out = []
    for i in range(n):
        c = arr[i]
        d = dict(area=c.area2 / 2.0, rect=(c.x0, c.y0, c.x1 - c.x0 + 1, c.y1 - c.y0 + 1),
                 is_hole=bool(c.is_hole), parent=c.parent, npts=c.npts)
        if with_points:
            dst = np.zeros(2 * c.npts, dtype=np.int32)
            lib().oc_contour_points(i, pts.ctypes.data, dst.ctypes.data, c.npts)
            d["points"] = dst.reshape(-1, 2)
        out.append(d)
    return out


def check_scoremap_validity(scoremap: np.ndarray) -> None:
    # utils/wsol.py:63-78
    if not isinstance(scoremap, np.ndarray):
        raise TypeError("Scoremap must be a numpy array")
    if scoremap.dtype != float:
        raise TypeError("Scoremap must be of np.float type")
    if len(scoremap.shape) != 2:
        raise ValueError("Scoremap must be a 2D array")
    if np.isnan(scoremap).any():
        raise ValueError("Scoremap must not contain nans.")
    if (scoremap > 1).any() or (scoremap < 0).any():
        raise ValueError("Scoremap must be in range [0, 1].")


def thresholds_to_levels(u8: np.ndarray, taus: Sequence[float]) -> np.ndarray:
    # thresh=int(threshold * np.max(scoremap_image)) (wsol_metrics.py:158)
    mx = np.max(u8)
    return np.array([int(t * mx) for t in taus], dtype=np.int32)


def contour_boxes(binary: np.ndarray) -> np.ndarray:
    """scoremap2bbox with multi_contour_eval=True (wsol_metrics.py:162-181): the clamped
    boundingRect of every contour of findContours(RETR_TREE), in OpenCV's list order;
    [[0, 0, 0, 0]] when there is none."""
    H, W = binary.shape
    cs = find_contours(binary)
    if not cs:
        return np.zeros((1, 4), dtype=np.int64)
    out = []
    for c in cs:
        x, y, w, h = c["rect"]
        out.append([x, y, min(x + w, W - 1), min(y + h, H - 1)])
    return np.asarray(out, dtype=np.int64)


def compute_bboxes_from_scoremaps(scoremap: np.ndarray, scoremap_threshold_list,
                                  multi_contour_eval: bool = False):
    """wsol_metrics.py:127-197."""
    if multi_contour_eval:
        check_scoremap_validity(scoremap)
        u8 = np.ascontiguousarray((scoremap * 255).astype(np.uint8))
        thr = thresholds_to_levels(u8, scoremap_threshold_list)
        cache, out = {}, []
        for t in thr.tolist():
            if t not in cache:
                cache[t] = contour_boxes(u8 > t)
            out.append(cache[t])
        return out, [len(b) for b in out]
    check_scoremap_validity(scoremap)
    H, W = scoremap.shape
    u8 = np.ascontiguousarray((scoremap * 255).astype(np.uint8))
    thr = thresholds_to_levels(u8, scoremap_threshold_list)
    boxes = np.zeros((len(thr), 4), dtype=np.int32)
    lib().oc_boxes_for_thresholds(u8.ctypes.data, H, W, thr.ctypes.data, len(thr),
                                  boxes.ctypes.data, None)
    return [b[None].astype(np.int64) for b in boxes], [1] * len(thr)


def boxes_for_levels(u8: np.ndarray, levels: np.ndarray) -> np.ndarray:
    u8 = np.ascontiguousarray(u8, dtype=np.uint8)
    H, W = u8.shape
    levels = np.ascontiguousarray(levels, dtype=np.int32)
    boxes = np.zeros((len(levels), 4), dtype=np.int32)
    lib().oc_boxes_for_thresholds(u8.ctypes.data, H, W, levels.ctypes.data, len(levels),
                                  boxes.ctypes.data, None)
    return boxes


def calculate_multiple_iou(box_a: np.ndarray, box_b: np.ndarray) -> np.ndarray:
    """wsol_metrics.py:77-124 (+1 inclusive-pixel convention)."""
    box_a = np.asarray(box_a)[:, None, :]
    box_b = np.asarray(box_b)[None, :, :]
    min_x = np.maximum(box_a[..., 0], box_b[..., 0])
    min_y = np.maximum(box_a[..., 1], box_b[..., 1])
    max_x = np.minimum(box_a[..., 2], box_b[..., 2])
    max_y = np.minimum(box_a[..., 3], box_b[..., 3])
    inter = np.maximum(0, max_x - min_x + 1) * np.maximum(0, max_y - min_y + 1)
    area_a = (box_a[..., 2] - box_a[..., 0] + 1) * (box_a[..., 3] - box_a[..., 1] + 1)
    area_b = (box_b[..., 2] - box_b[..., 0] + 1) * (box_b[..., 3] - box_b[..., 1] + 1)
    den = area_a + area_b - inter
    deg = np.where(den <= 0)
    den[deg] = 1
    ious = inter / den
    ious[deg] = 0
    return ious


class BoxEvaluatorRef:
    """BoxEvaluator (wsol_metrics.py:266-433) over in-memory GT boxes."""

    def __init__(self, cam_threshold_list, iou_threshold_list=(30, 50, 70),
                 multi_contour_eval: bool = False):
        self.cam_threshold_list = list(cam_threshold_list)
        self.iou_threshold_list = list(iou_threshold_list)
        self.multi_contour_eval = multi_contour_eval
        self.cls_correct = 0
        T = len(self.cam_threshold_list)
        self.cnt = 0
        self.num_correct = {t: np.zeros(T) for t in self.iou_threshold_list}
        self.num_correct_top1 = {t: np.zeros(T) for t in self.iou_threshold_list}
        self.num_correct_top5 = {t: np.zeros(T) for t in self.iou_threshold_list}

    def accumulate(self, scoremap, gt_boxes, target: int, preds_ordered) -> None:
        boxes, nbox = compute_bboxes_from_scoremaps(scoremap, self.cam_threshold_list,
                                                    self.multi_contour_eval)
        self.cls_correct += int(target == preds_ordered[0])
        boxes = np.concatenate(boxes, axis=0)
        miou = calculate_multiple_iou(boxes, np.asarray(gt_boxes))
        sliced, idx = [], 0
        for nr in nbox:
            sliced.append(max(miou.max(1)[idx:idx + nr]))
            idx += nr
        for thr in self.iou_threshold_list:
            ok = np.where(np.asarray(sliced) >= (thr / 100))[0]
            self.num_correct[thr][ok] += 1
            if target == preds_ordered[0]:
                self.num_correct_top1[thr][ok] += 1
            if target in preds_ordered[:5]:
                self.num_correct_top5[thr][ok] += 1
        self.cnt += 1

    def compute(self):
        """wsol_metrics.py:390-433: BoxAcc per IoU threshold; also best_tau_list and the
        top-1 / top-5 localisation accuracies."""
        out = []
        self.best_tau_list, self.top1, self.top5 = [], [], []
        for thr in self.iou_threshold_list:
            acc = self.num_correct[thr] * 100. / float(self.cnt)
            out.append(acc.max())
            self.best_tau_list.append(float(self.cam_threshold_list[np.argmax(acc)]))
            self.top1.append((self.num_correct_top1[thr] * 100. / float(self.cnt)).max())
            self.top5.append((self.num_correct_top5[thr] * 100. / float(self.cnt)).max())
        return out
