"""Device-resident BoxEvaluator (dlib/metrics/wsol_metrics.py:266-433).

The reference runs, per frame, a float64 D2H copy and up to 1000
``cv2.findContours`` calls on the CPU.  Here the whole sweep stays in HBM:
``bbox_levels`` computes the best box for every integer threshold level of
every frame at once, ``box_accumulate`` maps the tau list onto levels
(``int(tau * max(u8))``, wsol_metrics.py:158), scores IoU against GT and adds
to int32 counters on the device.  Counters are reduced across ranks with one
RCCL all-reduce in ``_synch_across_gpus`` (the reference all-gathers and sums,
wsol_metrics.py:372-388).
"""
from __future__ import annotations

import os
from copy import deepcopy
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch
import torch.distributed as dist

from . import ops

_RESIZE_LENGTH = 224  # constants.CROP_SIZE


def check_scoremap_validity(scoremap) -> None:
    """utils/wsol.py:63-78."""
    if not isinstance(scoremap, np.ndarray):
        raise TypeError(f"Scoremap must be a numpy array; it is {type(scoremap)}.")
    if scoremap.dtype != float:
        raise TypeError(f"Scoremap must be of np.float type; it is of {scoremap.dtype} type.")
    if len(scoremap.shape) != 2:
        raise ValueError(f"Scoremap must be a 2D array; it is {len(scoremap.shape)}D.")
    if np.isnan(scoremap).any():
        raise ValueError("Scoremap must not contain nans.")
    if (scoremap > 1).any() or (scoremap < 0).any():
        raise ValueError("Scoremap must be in range [0, 1]."
                         f"scoremap.min()={scoremap.min()}, scoremap.max()={scoremap.max()}.")


def check_box_convention(boxes, convention: str) -> None:
    """utils/wsol.py:28-60."""
    boxes = np.asarray(boxes)
    if (boxes < 0).any():
        raise RuntimeError("Box coordinates must be non-negative.")
    if len(boxes.shape) == 1:
        boxes = np.expand_dims(boxes, 0)
    elif len(boxes.shape) != 2:
        raise RuntimeError("Box array must have dimension (4) or (num_boxes, 4).")
    if boxes.shape[1] != 4:
        raise RuntimeError("Box array must have dimension (4) or (num_boxes, 4).")
    if convention == "x0y0x1y1":
        widths, heights = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    elif convention == "xywh":
        widths, heights = boxes[:, 2], boxes[:, 3]
    else:
        raise ValueError(f"Unknown convention {convention}.")
    if (widths < 0).any() or (heights < 0).any():
        raise RuntimeError(f"Boxes do not follow the {convention} convention.")


def resize_bbox(box, image_size, resize_size):
    """utils/tools.py:231-250 (int() truncation)."""
    check_box_convention(np.array(box), "x0y0x1y1")
    x0, y0, x1, y1 = map(float, box)
    iw, ih = map(float, image_size)
    nw, nh = map(float, resize_size)
    return int(x0 * nw / iw), int(y0 * nh / ih), int(x1 * nw / iw), int(y1 * nh / ih)


def calculate_multiple_iou(box_a, box_b) -> np.ndarray:
    """wsol_metrics.py:77-124 (host helper, +1 inclusive convention)."""
    box_a, box_b = np.asarray(box_a), np.asarray(box_b)
    check_box_convention(box_a, "x0y0x1y1")
    check_box_convention(box_b, "x0y0x1y1")
    a, b = box_a[:, None, :], box_b[None, :, :]
    ix = np.maximum(0, np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]) + 1)
    iy = np.maximum(0, np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]) + 1)
    inter = ix * iy
    area_a = (a[..., 2] - a[..., 0] + 1) * (a[..., 3] - a[..., 1] + 1)
    area_b = (b[..., 2] - b[..., 0] + 1) * (b[..., 3] - b[..., 1] + 1)
    den = area_a + area_b - inter
    deg = np.where(den <= 0)
    den[deg] = 1
    ious = inter / den
    ious[deg] = 0
    return ious


def _meta_path(metadata, key: str) -> str:
    if isinstance(metadata, str):
        return f"{metadata.rstrip('/')}/{key}.txt"
    if isinstance(metadata, dict):
        return metadata[key]
    return getattr(metadata, key)


def load_resized_boxes(metadata, resize_length: int = _RESIZE_LENGTH) -> Dict[str, list]:
    """BoxEvaluator._load_resized_boxes (wsol_metrics.py:285-293) over
    get_image_ids / get_bounding_boxes / get_image_sizes (wsol_loader.py:74-180)."""
    with open(_meta_path(metadata, "image_ids")) as f:
        ids = [ln.strip("\n") for ln in f.readlines()]
    boxes: Dict[str, list] = {}
    with open(_meta_path(metadata, "localization")) as f:
        for ln in f.readlines():
            i, a, b, c, d = ln.strip("\n").split(",")
            boxes.setdefault(i, []).append((float(a), float(b), float(c), float(d)))
    sizes = {}
    with open(_meta_path(metadata, "image_sizes")) as f:
        for ln in f.readlines():
            i, w, h = ln.strip("\n").split(",")
            sizes[i] = (int(w), int(h))
    return {i: [resize_bbox(b, sizes[i], (resize_length, resize_length)) for b in boxes[i]]
            for i in ids}


def _u8_from_scoremap(scoremap: np.ndarray, device) -> torch.Tensor:
    check_scoremap_validity(scoremap)
    u8 = (scoremap * 255).astype(np.uint8)  # wsol_metrics.py:153
    return torch.from_numpy(np.ascontiguousarray(u8))[None].to(device)


def opencv_contour_order(records: np.ndarray) -> np.ndarray:
    """The boxes of one level's contours (ops.bbox_contours records: is_hole, key, parent
    key, x0, y0, x1, y1) in cv2.findContours(RETR_TREE)'s list order: the pre-order of the
    contour tree with siblings in decreasing key order (cvInsertNodeIntoTree prepends each
    newly discovered contour — discovered in raster order of its component's first pixel —
    to its parent's children).  Pinned against the border-following oracle
    (tests/test_bbox_oracle.py)."""
    kids: Dict[int, list] = {}
    by_key = {}
    for r in records:
        by_key[int(r[1])] = r
        kids.setdefault(int(r[2]), []).append(int(r[1]))
    out = []
    stack = sorted(kids.get(-1, []))          # pop() takes the largest key first
    while stack:
        k = stack.pop()
        out.append(by_key[k][3:7])
        stack.extend(sorted(kids.get(k, [])))
    return np.asarray(out, dtype=np.int64).reshape(-1, 4)


def compute_bboxes_from_scoremaps(scoremap: Optional[np.ndarray], scoremap_threshold_list,
                                  multi_contour_eval: bool = False,
                                  bbox: Optional[list] = None, device="cuda"):
    """wsol_metrics.py:127-197, computed by the HIP bbox kernels.

    Returns (estimated_boxes_at_each_thr, number_of_box_list) like the reference.  With
    multi_contour_eval=True (box_v2_metric) every contour's box is returned, in OpenCV's
    list order (``ops.bbox_contours`` per distinct level + :func:`opencv_contour_order`).
    """
    taus = list(scoremap_threshold_list)
    if scoremap is None:
        assert bbox is not None
        return [np.array([bbox]) for _ in taus], [1] * len(taus)
    if multi_contour_eval:
        check_scoremap_validity(scoremap)
        u8h = np.ascontiguousarray((scoremap * 255).astype(np.uint8))
        u8 = torch.from_numpy(u8h).to(device)
        mx = int(u8h.max())
        present = np.zeros(257, bool)
        present[np.unique(u8h)] = True
        cache: Dict[int, np.ndarray] = {}
        out, counts = [], []
        for t in taus:
            thr = int(t * mx)
            if thr >= mx:
                out.append(np.zeros((1, 4), np.int64))
                counts.append(1)
                continue
            c = thr + 1
            while not present[c]:      # the image of thr is that of the next present value
                c += 1
            if c not in cache:
                cache[c] = opencv_contour_order(ops.bbox_contours(u8, c - 1))
            out.append(cache[c])
            counts.append(len(cache[c]))
        return out, counts
    u8 = _u8_from_scoremap(scoremap, device)
    boxes, vmax = ops.bbox_levels(u8)
    mx = int(vmax[0].item())
    table = boxes[0].cpu().numpy().astype(np.int64)
    out = []
    for t in taus:
        thr = int(t * mx)
        out.append(table[thr][None] if thr < mx else np.zeros((1, 4), np.int64))
    return out, [1] * len(taus)


# level ranges per frame of a drain sweep (BoxEvaluator.accumulate_batch(drain=True))
_DRAIN_CHUNKS = int(os.environ.get("TCAM_BBOX_DRAIN_CHUNKS", "4"))


class BoxEvaluator:
    """wsol_metrics.py:266-433 with device counters.

    ``gt_bboxes``: {image_id: [box, ...]} already resized to 224 (the
    reference builds it from metadata with resize_bbox); used by the
    reference-compatible :meth:`accumulate`.  :meth:`accumulate_batch` is the
    fast path used by :class:`~tcam_wsol_video_amd.inference.CAMComputer`.
    """

    def __init__(self, cam_threshold_list: Sequence[float],
                 iou_threshold_list: Sequence[int] = (30, 50, 70),
                 gt_bboxes: Optional[Dict[str, list]] = None, multi_contour_eval: bool = False,
                 device: Union[str, torch.device] = "cuda", metadata=None, **unused):
        """``metadata``: as the reference (wsol_metrics.py:266-293), the split's metadata —
        a folder with image_ids / image_sizes / localization.txt, or an object / dict
        with those file paths (wsol_loader.configure_metadata) — from which the GT boxes
        are read and resized to 224 with resize_bbox (``_load_resized_boxes``)."""
        self.cam_threshold_list = list(cam_threshold_list)
        self.iou_threshold_list = list(iou_threshold_list)
        self.multi_contour_eval = multi_contour_eval
        if gt_bboxes is None and metadata is not None:
            gt_bboxes = load_resized_boxes(metadata, _RESIZE_LENGTH)
        self.gt_bboxes = gt_bboxes or {}
        self.device = torch.device(device)
        T = len(self.cam_threshold_list)
        self.taus = torch.tensor(self.cam_threshold_list, dtype=torch.float64, device=self.device)
        # `>= (_THRESHOLD/100)` in Python float (wsol_metrics.py:357-358)
        self.iou_thr = torch.tensor([t / 100 for t in self.iou_threshold_list],
                                    dtype=torch.float64, device=self.device)
        self.counters = torch.zeros((3, len(self.iou_threshold_list), T), dtype=torch.int32,
                                    device=self.device)
        # frames whose argmax class is the target (Trainer._compute_accuracy,
        # train_wsol.py:1400-1435), on the device beside the counters
        self.cls_correct = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.cnt = 0
        self.best_tau_list: List[float] = []
        self.curve_s = None
        self.top1 = None
        self.top5 = None
        self.curve_top_1_5 = None
        self._flush = None   # CAMComputer: launches a clip it still holds back
        self._join = None    # CAMComputer: that, then the current stream waits for its streams

    # -- fast path ---------------------------------------------------------
    def accumulate_batch(self, cam_u8: torch.Tensor, gt: torch.Tensor, ngt: torch.Tensor,
                         top1: torch.Tensor, top5: torch.Tensor,
                         best_iou: Optional[torch.Tensor] = None, drain: bool = False,
                         gate: Optional[torch.Tensor] = None) -> None:
        """``drain``: nothing else will overlap this sweep (the last clip of a pass): run it
        on more level ranges per frame for a shorter latency (same boxes).  ``gate`` (a
        device int32, CAMComputer's per-clip f16x3 overflow flag): the clip's counts are
        added only when it is 0 — decided on the device, no host sync (``cnt`` still counts
        the frames: the caller takes them back when it re-evaluates the clip)."""
        if gate is not None:
            tot, cls = self.counters, self.cls_correct
            self.counters, self.cls_correct = torch.zeros_like(tot), torch.zeros_like(cls)
            try:
                self.accumulate_batch(cam_u8, gt, ngt, top1, top5, best_iou, drain)
            finally:
                keep = (gate == 0).to(torch.int32)
                tot.add_(self.counters * keep)
                cls.add_(self.cls_correct * keep)
                self.counters, self.cls_correct = tot, cls
            return
        if self.multi_contour_eval:
            # every contour's box; a tau scores its best IoU (wsol_metrics.py:342-368)
            iou, canon, vmax = ops.bbox_multi_iou(cam_u8, gt, ngt)
            ops.box_accumulate_multi(iou, canon, vmax, self.taus, gt, ngt, top1, top5,
                                     self.iou_thr, self.counters, best_iou)
        else:
            boxes, vmax = ops.bbox_levels(cam_u8, chunks=_DRAIN_CHUNKS if drain else 0)
            ops.box_accumulate(boxes, vmax, self.taus, gt, ngt, top1, top5, self.iou_thr,
                               self.counters, best_iou)
        # top1 = argmax(logits) == target (ties to the lower class, as torch.argmax)
        ops.flag_count(top1, self.cls_correct)
        self.cnt += int(cam_u8.shape[0])

    # -- reference-compatible path (wsol_metrics.py:295-370) ---------------
    def accumulate(self, scoremap, image_id: str, target: int, preds_ordered,
                   bbox=None, bbox_status=None) -> None:
        if scoremap is None:
            raise NotImplementedError("C_BOX boxes are outside the TCAM hot path")
        assert bbox is None and bbox_status is None
        gt = np.asarray(self.gt_bboxes[image_id], dtype=np.int32).reshape(-1, 4)
        u8 = _u8_from_scoremap(scoremap, self.device)
        preds = list(np.asarray(preds_ordered).tolist())
        top1 = torch.tensor([int(target == preds[0])], dtype=torch.int32, device=self.device)
        top5 = torch.tensor([int(target in preds[:5])], dtype=torch.int32, device=self.device)
        self.accumulate_batch(u8, torch.from_numpy(gt)[None].to(self.device),
                              torch.tensor([gt.shape[0]], dtype=torch.int32, device=self.device),
                              top1, top5)

    def _sync(self) -> None:
        # counters may be accumulated on a side stream (CAMComputer overlap), whose last clip
        # the computer may still hold back (its flush hook launches it)
        if self._flush is not None:
            self._flush()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    @property
    def num_correct(self) -> Dict[int, np.ndarray]:
        self._sync()
        c = self.counters[0].double().cpu().numpy()
        return {t: c[j] for j, t in enumerate(self.iou_threshold_list)}

    @property
    def num_correct_top1(self) -> Dict[int, np.ndarray]:
        self._sync()
        c = self.counters[1].double().cpu().numpy()
        return {t: c[j] for j, t in enumerate(self.iou_threshold_list)}

    @property
    def num_correct_top5(self) -> Dict[int, np.ndarray]:
        self._sync()
        c = self.counters[2].double().cpu().numpy()
        return {t: c[j] for j, t in enumerate(self.iou_threshold_list)}

    def _synch_across_gpus(self) -> None:
        """One all-reduce(sum) of the counters + cnt (RCCL when backend nccl)."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        if self._join is not None:
            # CAMComputer: launch the held-back clip and make the current stream (the one the
            # all-reduce is ordered on) wait for the side stream that accumulates the counters
            self._join()
        elif self._flush is not None:
            self._flush()
        dist.all_reduce(self.counters)
        dist.all_reduce(self.cls_correct)
        cnt = torch.tensor([self.cnt], dtype=torch.float64, device=self.counters.device)
        dist.all_reduce(cnt)
        self.cnt = int(cnt.item())

    def classification_accuracy(self) -> float:
        """Trainer._compute_accuracy (train_wsol.py:1400-1435): % of the evaluated frames
        (sampler padding included, as the reference counts them) whose argmax class is the
        target."""
        self._sync()
        return int(self.cls_correct.item()) / float(self.cnt) * 100

    def compute(self) -> List[float]:
        """wsol_metrics.py:390-433."""
        max_box_acc = []
        self.best_tau_list = []
        self.curve_s = {"x": self.cam_threshold_list}
        self.top1, self.top5 = [], []
        self.curve_top_1_5 = {"x": self.cam_threshold_list, "top1": dict(), "top5": dict()}
        nc, n1, n5 = self.num_correct, self.num_correct_top1, self.num_correct_top5
        for thr in self.iou_threshold_list:
            acc = nc[thr] * 100. / float(self.cnt)
            max_box_acc.append(acc.max())
            self.curve_s[thr] = acc
            self.best_tau_list.append(float(self.cam_threshold_list[np.argmax(acc)]))
            loc = n1[thr] * 100. / float(self.cnt)
            self.top1.append(loc.max())
            self.curve_top_1_5["top1"][thr] = deepcopy(loc)
            loc = n5[thr] * 100. / float(self.cnt)
            self.top5.append(loc.max())
            self.curve_top_1_5["top5"][thr] = deepcopy(loc)
        return max_box_acc
