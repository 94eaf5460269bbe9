"""The TCAM training losses behind the reference's loss API (dlib/losses), on the device.

Same classes, constructor arguments and call convention as the reference, so its trainer
builds them unchanged (process/instantiators.py:143-245 for task TCAM):

  MasterLoss            losses/master.py:18-67   ``loss = masterloss(epoch=..., fcams=...,
                                                 raw_img=..., seeds=...)``, ``l_holder``
  SelfLearningTcams     losses/tcam.py:48-77     CE(fcams, seeds, ignore seg_ignore_idx)
  ConRanFieldTcams      losses/tcam.py:80-115    DenseCRFLoss(softmax(fcams)), scale 1
  MaxSizePositiveTcams  losses/tcam.py:235-278   ELB(-sum S[:, c]) over c in {0, 1}, / 2
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
           "MaxSizePositiveTcams", "MasterLoss"]


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
        c = self.c_epoch if _epoch is None else _epoch
        s, e = self.start_epoch, self.end_epoch
        if s is None and e is None:
            return True
        if isinstance(s, int) and isinstance(e, int):
            return s <= c <= e
        if s is None and isinstance(e, int):
            return c <= e
        if isinstance(s, int) and e is None:
            return c >= s
        return False

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
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        if self.scale_factor != 1.:
            raise NotImplementedError("ConRanFieldTcams: crf_tc_scale != 1 (README runs 1.0) "
                                      "is not on the TCAM hot path")


class MaxSizePositiveTcams(ElementaryLoss):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        assert isinstance(self.elb, ELB)


class _FusedTcamLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fcams, raw, seeds, lam_sl, lam_crf, lam_size, t, s_rgb, s_xy):
        from .training import tcam_losses
        losses, dF = tcam_losses(fcams.detach().contiguous().float(), raw, seeds,
                                 (lam_sl, lam_crf, lam_size), t, (s_rgb, s_xy))
        ctx.save_for_backward(dF)
        terms = losses[1:]
        ctx.mark_non_differentiable(terms)
        return losses[:1], terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        (dF,) = ctx.saved_tensors
        return (dF * g_total.reshape(1, 1, 1, 1),) + (None,) * 8


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
        if not isinstance(loss_, (SelfLearningTcams, ConRanFieldTcams, MaxSizePositiveTcams)):
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
                **unused) -> torch.Tensor:
        assert self.losses != []
        if fcams is None or fcams.dim() != 4 or fcams.shape[1] != 2:
            raise ValueError("TCAM losses take fcams (B, 2, H, W)")
        lam = {SelfLearningTcams: 0.0, ConRanFieldTcams: 0.0, MaxSizePositiveTcams: 0.0}
        t, sig = 1.0, (15.0, 100.0)
        for loss in self.losses:
            loss.c_epoch = epoch
            if not loss.is_on():
                continue
            lam[type(loss)] += loss.lambda_
            if isinstance(loss, MaxSizePositiveTcams):
                t = loss.elb.t
            if isinstance(loss, ConRanFieldTcams):
                sig = (loss.sigma_rgb, loss.sigma_xy)
            if isinstance(loss, SelfLearningTcams) and loss.seg_ignore_idx != -255:
                raise NotImplementedError("seg_ignore_idx != -255")
        dev = fcams.device
        raw = None
        if lam[ConRanFieldTcams]:
            if raw_img is None:
                raise ValueError("ConRanFieldTcams needs raw_img (values in [0, 255])")
            raw = raw_img.to(device=dev, dtype=torch.float32).contiguous()
        if lam[SelfLearningTcams] and seeds is None:
            raise ValueError("SelfLearningTcams needs seeds")
        total, terms = _FusedTcamLoss.apply(
            fcams, raw, seeds if lam[SelfLearningTcams] else None, lam[SelfLearningTcams],
            lam[ConRanFieldTcams], lam[MaxSizePositiveTcams], float(t), sig[0], sig[1])
        by_type = {SelfLearningTcams: terms[0], ConRanFieldTcams: terms[1],
                   MaxSizePositiveTcams: terms[2]}
        zero = torch.zeros((), device=dev)
        self.l_holder = [total] + [by_type[type(l)] if l.is_on() else zero
                                   for l in self.losses]
        return total
