"""The TCAM training losses behind the reference's loss API (dlib/losses), on the device.

Same classes, constructor arguments and call convention as the reference, so its trainer
builds them unchanged (process/instantiators.py:143-245 for task TCAM):

  MasterLoss            losses/master.py:18-67   ``loss = masterloss(epoch=..., fcams=...,
                                                 raw_img=..., seeds=...)``, ``l_holder``
  SelfLearningTcams     losses/tcam.py:48-77     CE(fcams, seeds, ignore seg_ignore_idx)
  ConRanFieldTcams      losses/tcam.py:80-115    DenseCRFLoss(softmax(fcams)), scale 1
  MaxSizePositiveTcams  losses/tcam.py:235-278   ELB(-sum S[:, c]) over c in {0, 1}, / 2
  RgbJointConRanFieldTcams losses/tcam.py:158-232 ColorDenseCRFLoss over each knn_tc
                                                 group's width mosaic, mean over groups
  ELB                   losses/elb.py:15-137     extended log-barrier, t schedule

``MasterLoss.forward`` evaluates the active TCAM terms in ONE fused pass
(``training.tcam_losses``: softmax, the bilateral filter, ``tcam_tcam_losses``) and is one
autograd node whose backward is the fused d loss / d fcams — including
DenseCRFLossFunction's custom -2 lambda AS / N gradient (crf/dense_crf_loss.py:70-75).
Terms other than these three are outside the TCAM hot path and raise.
"""
from __future__ import annotations

import re
from typing import List, Optional

import torch
import torch.nn as nn

__all__ = ["ELB", "ElementaryLoss", "SelfLearningTcams", "ConRanFieldTcams",
           "MaxSizePositiveTcams", "RgbJointConRanFieldTcams", "MasterLoss",
           "group_ordered_frames", "loss_is_on"]


def loss_is_on(start, end, epoch: int) -> bool:
    """ElementaryLoss.is_on (losses/core.py:64-82) for the window [start, end]; an end of
    -1 means no end (core.py:48-49)."""
    if end == -1:
        end = None
    if start is None and end is None:
        return True
    if isinstance(start, int) and isinstance(end, int):
        return start <= epoch <= end
    if start is None and isinstance(end, int):
        return epoch <= end
    if isinstance(start, int) and end is None:
        return epoch >= start
    return False


def group_ordered_frames(seq_iter, frm_iter) -> List[List[int]]:
    """losses/tcam.py:32-45: the batch positions of each sequence (ascending sequence id),
    ordered by frame index (a stable sort: equal frame ids keep batch order)."""
    seq = [float(v) for v in torch.as_tensor(seq_iter).detach().cpu().reshape(-1).tolist()]
    frm = [float(v) for v in torch.as_tensor(frm_iter).detach().cpu().reshape(-1).tolist()]
    assert len(seq) == len(frm), (len(seq), len(frm))
    out = []
    for sv in sorted(set(seq)):
        idx = [i for i, v in enumerate(seq) if v == sv]
        out.append(sorted(idx, key=lambda i: frm[i]))
    return out


class ELB(nn.Module):
    """losses/elb.py:15-137: the barrier parameter ``t`` and its schedule.  The loss
    itself is evaluated inside the fused kernel (MaxSizePositiveTcams)."""

    def __init__(self, init_t: float = 1., max_t: float = 10., mulcoef: float = 1.01):
        super().__init__()
        assert isinstance(mulcoef, float) and mulcoef > 0.
        assert isinstance(init_t, float) and init_t > 0.
        assert isinstance(max_t, float) and max_t > init_t
        self.init_t = init_t
        self.mulcoef = float(mulcoef)
        self.max_t = float(max_t)
        self.t = float(init_t)

    def set_t(self, val):
        if isinstance(val, torch.Tensor):
            assert val.ndim == 1 and val.dtype == torch.float
            val = float(val.item())
        assert isinstance(val, float) and val > 0.
        self.t = val

    def get_t(self) -> torch.Tensor:
        return torch.tensor([self.t], dtype=torch.float)

    def update_t(self):
        # torch.min(t_lb * mulcoef, max_t) on fp32 buffers (elb.py:106-111)
        t = torch.tensor([self.t], dtype=torch.float) * torch.tensor([self.mulcoef],
                                                                       dtype=torch.float)
        self.t = float(torch.minimum(t, torch.tensor([self.max_t], dtype=torch.float)).item())

    def __str__(self):
        return f"{self.__class__.__name__}(): ELB method."


class ElementaryLoss(nn.Module):
    """losses/core.py:20-147 (epoch window, lambda, name)."""

    def __init__(self, cuda_id=None, name=None, lambda_=1., elb=nn.Identity(),
                 support_background=False, multi_label_flag=False, sigma_rgb=15.,
                 sigma_xy=100., scale_factor=0.5, start_epoch=None, end_epoch=None,
                 seg_ignore_idx=-255):
        super().__init__()
        self._name = name
        self.lambda_ = float(lambda_)
        self.elb = elb
        self.support_background = support_background
        assert not multi_label_flag
        self.multi_label_flag = multi_label_flag
        self.sigma_rgb = float(sigma_rgb)
        self.sigma_xy = float(sigma_xy)
        self.scale_factor = scale_factor
        if end_epoch == -1:
            end_epoch = None
        self.start_epoch = start_epoch
        self.end_epoch = end_epoch
        self.c_epoch = 0
        self.seg_ignore_idx = seg_ignore_idx

    def is_on(self, _epoch=None) -> bool:
        return loss_is_on(self.start_epoch, self.end_epoch,
                          self.c_epoch if _epoch is None else _epoch)

    def update_t(self):
        if isinstance(self.elb, ELB):
            self.elb.update_t()

    def set_t(self, v):
        if isinstance(self.elb, ELB):
            self.elb.set_t(v)

    def get_t(self):
        if isinstance(self.elb, ELB):
            return self.elb.get_t()
        return torch.tensor([0.0])

    @property
    def __name__(self):
        if self._name is not None:
            return self._name
        s1 = re.sub('(.)([A-Z][a-z]+)', r'\1_\2', self.__class__.__name__)
        return re.sub('([a-z0-9])([A-Z])', r'\1_\2', s1).lower()

    def forward(self, epoch=0, **kwargs):
        """A term on its own: the fused pass restricted to this term."""
        self.c_epoch = epoch
        m = MasterLoss()
        m.add(self)
        return m(epoch=epoch, **kwargs)


class SelfLearningTcams(ElementaryLoss):
    pass


class ConRanFieldTcams(ElementaryLoss):
    """losses/tcam.py:80-115; scale_factor != 1 filters resized copies (training._scaled_crf)."""


class MaxSizePositiveTcams(ElementaryLoss):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        assert isinstance(self.elb, ELB)


class RgbJointConRanFieldTcams(ElementaryLoss):
    """losses/tcam.py:158-232: the frames of each sequence of a knn_tc batch
    (``seq_iter`` / ``frm_iter``, group_ordered_frames) concatenated along the width
    (pair_samples) through ColorDenseCRFLoss(weight=lambda_, sigma_rgb, scale_factor):
    colour-only permutohedral filter (DIM 3) on the device; mean over the groups of >= 2
    frames (nan when there is none, as the reference's 0 / 0).  scale_factor != 1 resizes
    each mosaic (training.rgb_joint_crf)."""

    @staticmethod
    def pair_samples(o_idx, imgs: torch.Tensor, prob_cams: torch.Tensor):
        """losses/tcam.py:207-232 (the same width mosaic, for API parity; the loss builds
        its mosaics with tcam_mosaic_gather)."""
        assert imgs.ndim == 4 and imgs.shape[1] == 3 and prob_cams.ndim == 4
        assert len(o_idx) > 1, len(o_idx)
        idx = torch.as_tensor([int(i) for i in o_idx], device=imgs.device)
        return (torch.cat(list(imgs.index_select(0, idx)), dim=2)[None],
                torch.cat(list(prob_cams.index_select(0, idx.to(prob_cams.device))),
                          dim=2)[None])


class _FusedTcamLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fcams, raw, seeds, lam_sl, lam_crf, lam_size, t, s_rgb, s_xy, rgb,
                crf_scale):
        from .training import tcam_losses
        losses, dF = tcam_losses(fcams.detach().contiguous().float(), raw, seeds,
                                 (lam_sl, lam_crf, lam_size), t, (s_rgb, s_xy), rgb=rgb,
                                 crf_scale=crf_scale)
        ctx.save_for_backward(dF)
        terms = losses[1:]
        ctx.mark_non_differentiable(terms)
        return losses[:1], terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        (dF,) = ctx.saved_tensors
        return (dF * g_total.reshape(1, 1, 1, 1),) + (None,) * 10


class MasterLoss(nn.Module):
    """losses/master.py:18-67."""

    def __init__(self, cuda_id=None, name=None):
        super().__init__()
        self._name = name
        self.losses: List[ElementaryLoss] = []
        self.l_holder: List[torch.Tensor] = []
        self.n_holder = [self.__name__]

    @property
    def __name__(self):
        if self._name is not None:
            return self._name
        s1 = re.sub('(.)([A-Z][a-z]+)', r'\1_\2', self.__class__.__name__)
        return re.sub('([a-z0-9])([A-Z])', r'\1_\2', s1).lower()

    def add(self, loss_: ElementaryLoss):
        if not isinstance(loss_, (SelfLearningTcams, ConRanFieldTcams, MaxSizePositiveTcams,
                                  RgbJointConRanFieldTcams)):
            raise NotImplementedError(f"{type(loss_).__name__}: only the TCAM terms of the "
                                      f"README run are on the device path")
        self.losses.append(loss_)
        self.n_holder.append(loss_.__name__)

    def update_t(self):
        for loss in self.losses:
            loss.update_t()

    def get_t(self) -> list:
        return [[loss.__name__, loss.get_t().item()] for loss in self.losses]

    def set_t(self, l: list):
        for i, loss in enumerate(self.losses):
            name, t = l[i]
            if loss.__name__ == name:
                loss.set_t(t)

    def forward(self, epoch: int = 0, fcams: Optional[torch.Tensor] = None,
                raw_img: Optional[torch.Tensor] = None, seeds: Optional[torch.Tensor] = None,
                seq_iter=None, frm_iter=None, **unused) -> torch.Tensor:
        assert self.losses != []
        if fcams is None or fcams.dim() != 4 or fcams.shape[1] != 2:
            raise ValueError("TCAM losses take fcams (B, 2, H, W)")
        lam = {SelfLearningTcams: 0.0, ConRanFieldTcams: 0.0, MaxSizePositiveTcams: 0.0,
               RgbJointConRanFieldTcams: 0.0}
        t, sig, crf_scale = 1.0, (15.0, 100.0), 1.0
        rgb = None
        for loss in self.losses:
            loss.c_epoch = epoch
            if not loss.is_on():
                continue
            if isinstance(loss, RgbJointConRanFieldTcams):
                if rgb is not None:
                    raise NotImplementedError("two RgbJointConRanFieldTcams terms")
                if seq_iter is None or frm_iter is None:
                    raise ValueError("RgbJointConRanFieldTcams needs seq_iter / frm_iter")
                rgb = (loss.lambda_, loss.sigma_rgb, group_ordered_frames(seq_iter, frm_iter),
                       float(loss.scale_factor))
                continue
            lam[type(loss)] += loss.lambda_
            if isinstance(loss, MaxSizePositiveTcams):
                t = loss.elb.t
            if isinstance(loss, ConRanFieldTcams):
                sig = (loss.sigma_rgb, loss.sigma_xy)
                crf_scale = float(loss.scale_factor)
            if isinstance(loss, SelfLearningTcams) and loss.seg_ignore_idx != -255:
                raise NotImplementedError("seg_ignore_idx != -255")
        dev = fcams.device
        raw = None
        if lam[ConRanFieldTcams] or rgb is not None:
            if raw_img is None:
                raise ValueError("the CRF terms need raw_img (values in [0, 255])")
            raw = raw_img.to(device=dev, dtype=torch.float32).contiguous()
        if lam[SelfLearningTcams] and seeds is None:
            raise ValueError("SelfLearningTcams needs seeds")
        total, terms = _FusedTcamLoss.apply(
            fcams, raw, seeds if lam[SelfLearningTcams] else None, lam[SelfLearningTcams],
            lam[ConRanFieldTcams], lam[MaxSizePositiveTcams], float(t), sig[0], sig[1], rgb,
            crf_scale)
        by_type = {SelfLearningTcams: terms[0], ConRanFieldTcams: terms[1],
                   MaxSizePositiveTcams: terms[2]}
        if rgb is not None:
            by_type[RgbJointConRanFieldTcams] = terms[3]
        zero = torch.zeros((), device=dev)
        self.l_holder = [total] + [by_type[type(l)] if l.is_on() else zero
                                   for l in self.losses]
        return total
