"""Batched CAM computation + evaluation (learning/inference_wsol.py:105-457).

The reference ``CAMComputer.minibatch_accum`` loops over frames with batch 1:
forward, ``SegmentationCam`` softmax, bilinear resize, D2H float64, CPU bbox
sweep.  ``CAMComputer.evaluate_batch`` does the same work for a whole clip on
the device with no host round trip: one batched forward (eval-mode BN makes
this numerically the per-frame forward), the fused seg-head/softmax/uint8
kernel, the level-table bbox kernels and the device counters.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

import contextlib

from . import ops
from .metrics import BoxEvaluator
from .models import STD_CL, TCAM, UnetTCAM, STDClassifier, _precision, features_fc_weight


def _redirect(flag: Optional[torch.Tensor]):
    """The f16x3 launches inside write ``flag`` instead of the device's flag (or nothing
    changes when ``flag`` is None)."""
    return ops.f16_overflow_into(flag) if flag is not None else contextlib.nullcontext()


class SegmentationCam:
    """cams/builtincam.py:141-225 over a batched model.cams (B, 2, H, W)."""

    def __init__(self, model):
        self.model = model
        self.support_backgr = model.classification_head.support_background

    def __call__(self, class_idx=None, scores=None, normalized=True, reshape=None,
                 argmax: bool = False) -> torch.Tensor:
        cam = self.compute_cams(argmax=argmax)
        if reshape is not None:
            cam = torch.nn.functional.interpolate(cam[:, None], reshape, mode="bilinear",
                                                  align_corners=False)[:, 0]
        return cam[0] if cam.shape[0] == 1 else cam

    def compute_cams(self, argmax: bool = False) -> torch.Tensor:
        m = self.model
        if m.cams is None:
            raise AssertionError("forward the model first")
        if not argmax:
            return m.cam  # the fused kernel already produced softmax[:, 1]
        # argmax=True (fcam_argmax, off the default path): from the fcams.
        return torch.argmax(m.cams, dim=1).float()


def build_tcam_extractor(model, args=None) -> SegmentationCam:
    """cams/__init__.py:327-330."""
    model.eval()
    return SegmentationCam(model)


class CAM:
    """STD_CL CAM extractor (cams/cam.py:31-99): weights of ``fc_layer`` times
    the activations of ``target_layer`` (the last encoder stage)."""

    def __init__(self, model: STDClassifier, target_layer: str = "encoder.layer4.2.relu3",
                 fc_layer: str = "classification_head.fc"):
        from .models import TRG_LAYERS
        if target_layer not in TRG_LAYERS.values():
            raise NotImplementedError(f"CAM hook {target_layer!r}: the encoders' last stages "
                                      f"are {sorted(TRG_LAYERS.values())}")
        self.model = model
        self.target_layer = target_layer
        self._fc = dict(model.named_modules())[fc_layer]

    def __call__(self, class_idx, scores=None, normalized: bool = True, reshape=None):
        A = self.model.features
        if A is None:
            raise AssertionError("Inputs need to be forwarded in the model for the conv "
                                 "features to be hooked")
        if not normalized:
            raise NotImplementedError
        cls = torch.as_tensor(class_idx, dtype=torch.int32).reshape(-1)
        if cls.numel() == 1 and A.shape[0] > 1:
            cls = cls.expand(A.shape[0]).contiguous()
        size = reshape if reshape is not None else (
            A.shape[1:3] if ops.is_act(A) else A.shape[2:])
        w = self._fc.weight.detach().contiguous()
        if self._fc is self.model.classification_head.fc:
            w = features_fc_weight(self.model)   # the f16x3 features' channel exponents
        low, cam, _ = ops.std_cam(A, w, cls, tuple(size),
                                  want_u8=False)
        out = cam if reshape is not None else low
        return out[0] if out.shape[0] == 1 else out


class CAMComputer:
    """Batched evaluation of one split (inference_wsol.py:105-457).

    ``overlap=True`` runs the bbox sweep + counters of clip k on a side HIP
    stream, so they execute concurrently with the forward of clip k+1; the
    forward itself runs on a high-priority stream so that the convolutions'
    workgroups are dispatched ahead of the bbox kernels' whenever both wait
    for a CU.  The counters are complete once :meth:`synchronize` (or
    :meth:`compute_and_evaluate`) has run.
    """

    def __init__(self, model, cam_curve_interval: float = .001,
                 iou_threshold_list: Sequence[int] = (30, 50, 70), device="cuda",
                 overlap: bool = True, keep_fcams: bool = False, fwd_streams: int = 1,
                 temporal=None, multi_contour_eval: bool = False):
        """fwd_streams > 1 pipelines consecutive clips: clip k+1's forward may run while
        clip k's is still in flight (their small layers fill each other's idle CUs); the
        CAMs a call returns are then complete only after :meth:`synchronize`.

        ``temporal`` (a :class:`~tcam_wsol_video_amd.parallel.TemporalCAM`): the boxes
        are taken on the temporal CAM (CAM-TMP) of each frame instead of its own CAM;
        under torch.distributed each call's frames are this rank's contiguous shard of
        one clip, and the per-frame CAMs are all-gathered over the ranks first
        (BASELINE configs[4]).

        ``multi_contour_eval`` (``--box_v2_metric True``, parseit.py:684-689): every
        contour's box counts, a tau scores its best IoU (wsol_metrics.py:170-181, 342-368)."""
        self.model = model.eval()
        self.temporal = temporal
        self.keep_fcams = keep_fcams   # also materialise model.cams (fcams) per clip
        self.device = torch.device(device)
        self.cam_threshold_list = list(np.arange(0, 1, cam_curve_interval))
        self.evaluator = BoxEvaluator(self.cam_threshold_list, iou_threshold_list,
                                      device=self.device, multi_contour_eval=multi_contour_eval)
        self.side = (torch.cuda.Stream(device=self.device,
                                       priority=int(os.environ.get("TCAM_SIDE_PRIO", "0")))
                     if overlap else None)
        n = max(1, int(fwd_streams)) if overlap else 0
        self.fwds = [torch.cuda.Stream(device=self.device,
                                       priority=int(os.environ.get("TCAM_FWD_PRIO", "-1")))
                     for _ in range(n)]
        self.fwd = self.fwds[0] if self.fwds else None
        # f16x3 overflow recovery (TCAM_F16_RECOVER=0: off — the pass then raises at the
        # end): each clip's convolutions set their own flag, the clip's counts are gated on
        # it on the device, the flag travels to the host asynchronously, and a flagged clip
        # is re-evaluated on the exact x6 path in compute_and_evaluate (CAM-TMP excluded:
        # its per-clip all-gather is a collective a one-rank redo cannot join)
        self.recover = os.environ.get("TCAM_F16_RECOVER", "1") != "0" and temporal is None
        self._watch = []     # (event, pinned host flag, frames, clip inputs)
        self._redo = []      # clip inputs to re-evaluate in x6
        self.recovered_clips = 0
        self._k = 0
        self._pending = None
        if self.side is not None:
            self.evaluator._flush = lambda: self._flush(drain=True)
            self.evaluator._join = self.synchronize

    def _flush(self, drain: bool = False) -> None:
        """Launch the clip whose bbox sweep is held back (see evaluate_batch) on the side
        stream; ``drain``: no further clip follows, so it runs on more level ranges."""
        pend, self._pending = self._pending, None
        if pend is None:
            return
        ev, args, gate = pend
        self.side.wait_event(ev)
        for t in args + (gate,):
            if t is not None:
                t.record_stream(self.side)  # keep alive until the side stream is done
        with torch.cuda.stream(self.side):
            self.evaluator.accumulate_batch(*args, drain=drain, gate=gate)

    def synchronize(self) -> None:
        if self.side is not None:
            self._flush(drain=True)
        cur = torch.cuda.current_stream(self.device)
        for f in self.fwds:
            cur.wait_stream(f)
        if self.side is not None:
            cur.wait_stream(self.side)

    @torch.no_grad()
    def evaluate_batch(self, images: torch.Tensor, targets: torch.Tensor, gt: torch.Tensor,
                       ngt: Optional[torch.Tensor] = None,
                       best_iou: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One clip: forward -> CAM (uint8) -> boxes at every tau -> counters.

        images (B,3,H,W) fp32 on the device; targets (B,); gt (B,G,4) int32.
        Returns the uint8 CAMs (B,H,W).
        """
        self._poll()
        gate = None
        if self.recover and _precision(self.model) == "f16x3":
            gate = torch.zeros(1, dtype=torch.int32, device=self.device)
        if self.side is None:
            with _redirect(gate):
                cam_u8, top1, top5, ngt_ = self._forward(images, targets, gt, ngt)
            self.evaluator.accumulate_batch(cam_u8, gt, ngt_, top1, top5, best_iou, gate=gate)
            self._watch_clip(gate, images, targets, gt, ngt, best_iou,
                             torch.cuda.current_stream(self.device))
            return cam_u8
        caller = torch.cuda.current_stream(self.device)
        fwd = self.fwds[self._k % len(self.fwds)]
        self._k += 1
        fwd.wait_stream(caller)
        for t in (images, targets, gt, ngt, gate):
            if t is not None:
                t.record_stream(fwd)
        with torch.cuda.stream(fwd), _redirect(gate):
            cam_u8, top1, top5, ngt_ = self._forward(images, targets, gt, ngt)
        self._watch_clip(gate, images, targets, gt, ngt, best_iou, fwd)
        if len(self.fwds) == 1:
            caller.wait_stream(fwd)
        cam_u8.record_stream(caller)
        # the sweep of the previous clip goes out now; this clip's is held back until the
        # next call (or synchronize / a counter read, which know it is the last and give it
        # more level ranges per frame: nothing else overlaps that drain)
        self._flush()
        ev = torch.cuda.Event()
        ev.record(fwd)
        self._pending = (ev, (cam_u8, gt, ngt_, top1, top5, best_iou), gate)
        return cam_u8

    def _watch_clip(self, gate, images, targets, gt, ngt, best_iou, stream) -> None:
        """Send the clip's overflow flag to the host behind its forward (no sync); the
        inputs stay referenced until the flag has arrived (a few clips)."""
        if gate is None:
            return
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(stream):
            host.copy_(gate, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._watch.append((ev, host, int(images.shape[0]),
                            (images, targets, gt, ngt, best_iou)))

    def _poll(self, wait: bool = False) -> None:
        """Flags that have arrived: a clean clip is forgotten, an overflowed one is queued
        for the x6 re-evaluation and its frames are taken out of the count."""
        keep = []
        for ev, host, n, clip in self._watch:
            if wait:
                ev.synchronize()
            elif not ev.query():
                keep.append((ev, host, n, clip))
                continue
            if int(host.item()):
                self._redo.append(clip)
                self.evaluator.cnt -= n
        self._watch = keep

    def _forward(self, images, targets, gt, ngt):
        m = self.model
        # the f16x3 range check runs once, in compute_and_evaluate (no per-clip host sync);
        # the deferral holds for this forward only
        prev = m.__dict__.get("_defer_f16_check", False)
        m.__dict__["_defer_f16_check"] = True
        try:
            if isinstance(m, UnetTCAM):
                logits, _, _ = m(images, want_fcams=self.keep_fcams)
                cam, cam_u8 = m.cam, m.cam_u8
            elif isinstance(m, STDClassifier):
                logits = m(images)
                _, cam, cam_u8 = ops.std_cam(m.features, features_fc_weight(m), targets,
                                             tuple(images.shape[2:]))
            else:
                raise TypeError(type(m))
        finally:
            m.__dict__["_defer_f16_check"] = prev
        if self.temporal is not None:
            self.last_tmp_cam, cam_u8 = self.temporal(cam, want_cam=self.keep_fcams)
        self.last_logits, self.last_cam = logits, cam
        top1, top5 = ops.topk_flags(logits, targets)
        if ngt is None:
            ngt = torch.full((gt.shape[0],), gt.shape[1], dtype=torch.int32, device=gt.device)
        return cam_u8, top1, top5, ngt

    def recover_overflowed(self) -> int:
        """Re-evaluate on the exact x6 path every clip whose f16x3 activations left the S2
        range (their counts were gated off on the device); returns how many."""
        self.synchronize()
        self._poll(wait=True)
        redo, self._redo = self._redo, []
        if not redo:
            return 0
        m = self.model
        prev, rec = m.__dict__.get("conv_precision"), self.recover
        m.conv_precision, self.recover = "x6", False
        try:
            for images, targets, gt, ngt, best_iou in redo:
                self.evaluate_batch(images, targets, gt, ngt, best_iou)
            self.synchronize()
        finally:
            self.recover = rec
            if prev is None:
                m.__dict__.pop("conv_precision", None)
            else:
                m.conv_precision = prev
        self.recovered_clips += len(redo)
        return len(redo)

    def compute_and_evaluate(self):
        self.synchronize()
        self.recover_overflowed()
        # f16x3 plans: every activation of the pass stayed within the S2 range — on every
        # rank (a MAX all-reduce of the flag first: all ranks raise together or none does);
        # with recovery on, only an activation outside the per-clip flags can still raise
        ops.check_f16_overflow(self.device, all_ranks=True)
        if dist.is_available() and dist.is_initialized():
            self.evaluator._synch_across_gpus()
        return self.evaluator.compute()
