"""TCAM training step on the gfx950 kernels (BASELINE
configs[2]): the reference's ``Trainer._wsol_training`` for task TCAM
(learning/train_wsol.py:685-884) with ``freeze_cl=True`` (base/model.py:141-142,
164-215): the encoder and the WGAP head are frozen and in eval mode; the U-Net decoder
and the segmentation head train with batch-statistics BatchNorm under

  SelfLearningTcams (CE on the seeds, ignore -255)          losses/tcam.py:48-77
  ConRanFieldTcams (dense CRF, permutohedral filter)        losses/tcam.py:80-115
  MaxSizePositiveTcams (ELB log-barrier on the sizes)       losses/tcam.py:235-278

and torch.optim.SGD(momentum 0.9, dampening 0, weight_decay 1e-4, nesterov)
(process/instantiators.py:818-841, configure/config.py:181-185).  Multi-GPU: one
process per GPU; the flat gradient buffer is all-reduced (RCCL) and averaged, and rank
0's BatchNorm running statistics are broadcast — what DDP does (parallel/my_ddp.py).

Every tensor operation of the step is a kernel of libtcam_hip.so: x6 convolutions
(forward and data gradient), fp32-MFMA weight gradients, BatchNorm statistics / apply /
backward, up-sampling adjoints, the fused seg head, softmax, the bilateral filter, the
loss reductions and the SGD update.  Trainable parameters live in one flat fp32 buffer
that the module's ``nn.Parameter``s view, so ``state_dict()`` always shows the trained
weights.  Seeds come from the caller (TCAMSeeder, cams/tcam_seeding.py, is a §8f "next"
row).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F
import torch.distributed as dist
import torch.nn as nn

from . import _lib, crf, ops
from ._lib import check, tcam_conv_src
from .losses import ELB  # noqa: F401  (re-exported: training.ELB)
from .models import CenterBlock, UnetTCAM
from .ops import ConvSrc
from .seeding import prepare_std_cams

# UnetTCAM's eval plans that fold decoder weights / BN
DECODER_PLANS = ("dec_x6", "dec_f16x3", "dec_amp", "dec")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream



def rgb_joint_crf(raw_imgs: torch.Tensor, S: torch.Tensor, groups: Sequence[Sequence[int]],
                  lam: float, sigma_rgb: float, scale: float = 1.0):
    """RgbJointConRanFieldTcams.forward (losses/tcam.py:186-205) on the device, given the
    batch's softmaxed fcams ``S`` (B, 2, H, W) and ``groups`` = group_ordered_frames(...):
    each group of >= 2 frames is one width mosaic of its frames (pair_samples, :207-232)
    through ColorDenseCRFLoss (colour-only filter, DIM 3, scale 1;
    color_dense_crf_loss.py:33-78, 112-127); the loss is the mean over those groups.
    Returns (value (1,), d value / d S (B, 2, H, W)); with no such group the value is
    0 / 0 = nan, as the reference's (the trainer then skips the step).

    Groups of one length share one batched filter call (the filter is per image, so
    batching changes nothing); the gradient of frame b sums its occurrences in fixed
    order (a frame repeated by _fill_minibatch appears more than once).

    ``scale`` != 1 (--rgb_jcrf_tc_scale; color_dense_crf_loss.py:112-127): each mosaic is
    nearest-resized (image) / bilinear-resized (S) before the filter, as the reference
    resizes the concatenated pair, and -2 lam AS / c goes back through the bilinear
    resize's adjoint before the scatter to the frames."""
    lib = _lib.load()
    dev = S.device
    B, K, H, W = S.shape
    gx = torch.zeros_like(S)
    groups = [list(g) for g in groups if len(g) >= 2]
    if not groups:
        return torch.full((1,), float("nan"), device=dev), gx
    c = float(len(groups))
    raw = raw_imgs.to(device=dev, dtype=torch.float32).contiguous()
    if tuple(raw.shape) != (B, 3, H, W):
        raise ValueError(f"raw images {tuple(raw.shape)} vs fcams {tuple(S.shape)}")
    energy = torch.zeros(1, device=dev, dtype=torch.float32)
    ews = crf._energy_ws(dev)
    for L in sorted({len(g) for g in groups}):
        cls = [g for g in groups if len(g) == L]
        G = len(cls)
        idx_h = torch.tensor(cls, dtype=torch.int32)
        occ = [[] for _ in range(B)]
        for gi, g in enumerate(cls):
            for p, b in enumerate(g):
                occ[b].append(gi * L + p)
        start = [0]
        for o in occ:
            start.append(start[-1] + len(o))
        occ_h = torch.tensor([v for o in occ for v in o], dtype=torch.int32)
        tabs = torch.cat([idx_h.reshape(-1), torch.tensor(start, dtype=torch.int32), occ_h])
        tabs = tabs.to(dev)
        idx_d = tabs[:G * L]
        start_d = tabs[G * L:G * L + B + 1]
        occ_d = tabs[G * L + B + 1:]
        img_m = torch.empty((G, 3, H, L * W), device=dev, dtype=torch.float32)
        s_m = torch.empty((G, K, H, L * W), device=dev, dtype=torch.float32)
        check(lib.tcam_mosaic_gather(raw.data_ptr(), idx_d.data_ptr(), G, L, 3, H, W,
                                     img_m.data_ptr(), _stream()), "tcam_mosaic_gather")
        check(lib.tcam_mosaic_gather(S.data_ptr(), idx_d.data_ptr(), G, L, K, H, W,
                                     s_m.data_ptr(), _stream()), "tcam_mosaic_gather")
        coef = -2.0 * lam / c
        if scale != 1.0:
            img_m = F.interpolate(img_m, scale_factor=scale, mode="nearest",
                                  recompute_scale_factor=False).contiguous()
            s_req = s_m.requires_grad_(True)
            with torch.enable_grad():
                s_s = F.interpolate(s_req, scale_factor=scale, mode="bilinear",
                                    recompute_scale_factor=False, align_corners=False)
            s_f = s_s.detach().contiguous()
        else:
            s_f = s_m
        AS = crf.color_bilateral_filter(img_m, s_f, sigma_rgb, dim=3)
        e = torch.empty(1, device=dev, dtype=torch.float32)
        # each mosaic is its own N = 1 batch: sum_g -(S_g . AS_g)
        check(lib.tcam_crf_energy(s_f.data_ptr(), AS.data_ptr(), s_f.numel(), 1, e.data_ptr(),
                                  ews.data_ptr(), _stream()), "tcam_crf_energy")
        energy += e
        # d (lam / c sum_g E_g) / d S_g = -2 lam / c AS_g (ColorDenseCRFLossFunction.backward)
        if scale != 1.0:
            (gm,) = torch.autograd.grad(s_s, s_req, AS * coef)
            AS, coef = gm.float().contiguous(), 1.0
        check(lib.tcam_mosaic_scatter(AS.data_ptr(), start_d.data_ptr(), occ_d.data_ptr(), B, L,
                                      K, H, W, coef, 1, gx.data_ptr(), _stream()),
              "tcam_mosaic_scatter")
    return energy * (lam / c), gx


def _scaled_crf(raw_imgs: torch.Tensor, S: torch.Tensor, lam: float, sigma, scale: float):
    """ConRanFieldTcams at crf_tc_scale != 1 (losses/tcam.py:80-115 through
    crf/dense_crf_loss.py:95-123): the image nearest-resized and S bilinear-resized by
    ``scale``, the filter at sigma_xy * scale, value lam * -sum(S' AS') / N; d value / d S is
    -2 lam AS' / N taken back through the bilinear resize's adjoint (torch autograd of the
    resize, as the reference's own autograd does)."""
    Sv = S.detach().requires_grad_(True)
    with torch.enable_grad():
        val = crf.DenseCRFLoss(weight=lam, sigma_rgb=sigma[0], sigma_xy=sigma[1],
                               scale_factor=scale)(raw_imgs, Sv)
        (gS,) = torch.autograd.grad(val, Sv)
    return val.detach().reshape(1).float(), gS.float().contiguous()


def tcam_losses(fcams: torch.Tensor, raw_imgs: Optional[torch.Tensor],
                seeds: Optional[torch.Tensor], lam=(1.0, 2e-9, 0.01), elb_t: float = 1.0,
                sigma=(15.0, 100.0), rgb: Optional[tuple] = None, crf_scale: float = 1.0,
                lattice: Optional["crf.PreparedLattice"] = None):
    """The TCAM MasterLoss of one batch in two kernels + the CRF filter: returns the
    device tensor (total, self-learning, CRF, size) and d total / d fcams.

      SelfLearningTcams  CE(fcams, seeds, ignore -255) * lam[0]       losses/tcam.py:48-77
      ConRanFieldTcams   lam[1] * -sum(S * AS) / N, S = softmax(fcams),  :80-115
                         AS = bilateral(raw, S) (scale_factor 1)       dense_crf_loss.py:32-123
      MaxSizePositive    lam[2] / 2 * sum_c ELB_t(-sum_hw S[:, c])       :235-278, elb.py:119-137

    A zero lambda (or a missing seeds / raw_imgs) drops the term.  dF includes the CRF
    term's custom gradient -2 lam[1] AS / N (DenseCRFLossFunction.backward).  ``crf_scale``
    != 1 (--crf_tc_scale) filters resized copies (:func:`_scaled_crf`); its value and
    d / d S then enter the fused kernel as an extra term.  ``lattice``: a
    :class:`crf.PreparedLattice` of ``raw_imgs`` built ahead (same sigmas), applied here.
    ``rgb`` = (lam, sigma_rgb, groups): RgbJointConRanFieldTcams (:158-232,
    :func:`rgb_joint_crf`) as a fifth term; the loss tensor then has 5 entries (its value
    last)."""
    lib = _lib.load()
    dev = fcams.device
    B, _, H, W = fcams.shape
    HW = H * W
    S = torch.empty_like(fcams)
    check(lib.tcam_softmax2(fcams.data_ptr(), S.data_ptr(), B, HW, _stream()), "tcam_softmax2")
    lam_sl = lam[0] if seeds is not None else 0.0
    lam_crf = lam[1] if raw_imgs is not None else 0.0
    AS = None
    crf_val = None
    if lam_crf and crf_scale != 1.0:
        crf_val, crf_g = _scaled_crf(raw_imgs, S, lam_crf, sigma, crf_scale)
        lam_crf = 0.0
    elif lam_crf and lattice is not None:   # the image half ran ahead (DecoderTrainer.step)
        AS = lattice.apply(S)
    elif lam_crf:
        AS = crf.bilateral_filter(raw_imgs, S, sigma[0], sigma[1])
    if lattice is not None and AS is None:
        raise ValueError("tcam_losses: a prepared lattice must be applied (CRF term on, "
                         "scale 1)")
    if seeds is not None:
        seeds = seeds.to(device=dev, dtype=torch.int32).contiguous()
    gx = extra = None
    if rgb is not None:
        if raw_imgs is None:
            raise ValueError("RgbJointConRanFieldTcams needs raw_img (values in [0, 255])")
        extra, gx = rgb_joint_crf(raw_imgs, S, rgb[2], rgb[0], rgb[1],
                                  scale=rgb[3] if len(rgb) > 3 else 1.0)
    rgb_val = extra
    if crf_val is not None:   # the scaled CRF rides the extra-term slot
        extra = crf_val if extra is None else extra + crf_val
        gx = crf_g if gx is None else gx + crf_g
    losses = torch.empty(4 if extra is None else 5, device=dev, dtype=torch.float32)
    dF = torch.empty_like(fcams)
    ws = torch.empty(int(lib.tcam_tcam_loss_ws_bytes(B, HW)), dtype=torch.uint8, device=dev)
    check(lib.tcam_tcam_losses_ex(fcams.data_ptr(), S.data_ptr(),
                                  seeds.data_ptr() if (seeds is not None and lam_sl) else None,
                                  AS.data_ptr() if AS is not None else None,
                                  gx.data_ptr() if gx is not None else None,
                                  extra.data_ptr() if extra is not None else None, B, HW,
                                  lam_sl, lam_crf, lam[2], float(elb_t), losses.data_ptr(),
                                  dF.data_ptr(), ws.data_ptr(), _stream()), "tcam_tcam_losses")
    if crf_val is not None:   # report the two extra terms in their own slots
        losses[2:3].copy_(crf_val)
        if rgb_val is not None:
            losses[4:5].copy_(rgb_val)
        else:
            losses = losses[:4]
    return losses, dF


def fill_minibatch(x: Optional[torch.Tensor], mbatchsz: int) -> Optional[torch.Tensor]:
    """Trainer._fill_minibatch (learning/train_wsol.py:1006-1023): a short batch is
    repeated (whole copies, then cut) up to ``mbatchsz`` frames — so the last batch of an
    epoch has the full batch's BatchNorm statistics and loss normalisation."""
    if x is None:
        return None
    assert isinstance(mbatchsz, int) and mbatchsz > 0
    assert x.shape[0] <= mbatchsz, (x.shape[0], mbatchsz)
    if x.shape[0] == mbatchsz:
        return x
    t = -(-mbatchsz // x.shape[0])
    return torch.cat(t * [x])[:mbatchsz]


class _Conv:
    """One trainable conv (no bias) + BatchNorm + ReLU of the decoder (Conv2dReLU)."""

    def __init__(self, seq: nn.Sequential):
        self.conv: nn.Conv2d = seq[0]
        self.bn: nn.BatchNorm2d = seq[1]
        self.cout = self.conv.out_channels
        self.ctot = self.conv.in_channels
        self.wx6: Optional[torch.Tensor] = None      # forward operand
        self.wsc: Optional[torch.Tensor] = None      # its f16x3 per-column scales
        self.wdg: Optional[torch.Tensor] = None      # data-gradient operand
        self.dsc: Optional[torch.Tensor] = None      # its f16x3 scales
        self.dg_cout = 0                             # channels the dgrad produces


class DecoderTrainer:
    """Trains ``model.decoder`` + ``model.segmentation_head`` of a ResNet50 / VGG16 /
    InceptionV3 ``UnetTCAM`` (x6 path: fp32-accurate; the parity path).

    ``amp=True`` is the reference's ``--amp True`` (train_wsol.py:1077, 1155-1184:
    ``autocast`` + ``GradScaler``): the frozen encoder and the decoder run autocast's fp16
    convolutions (S1 activations, one fp16 MFMA product per MAC, fp32 accumulation, fp16
    outputs; BatchNorm statistics / affine, the losses and the update in fp32), the loss is
    scaled by a device-resident GradScaler scale (init 2^16, x2 every 2000 clean steps, x0.5
    on a non-finite gradient), the gradients are unscaled with a device-side non-finite
    check, and the step is skipped on the device when any rank found one."""

    def __init__(self, model: UnetTCAM, lr: float = 0.01, momentum: float = 0.9,
                 dampening: float = 0.0, weight_decay: float = 1e-4, nesterov: bool = True,
                 sl_lambda: float = 1.0, crf_lambda: float = 2e-9, size_lambda: float = 0.01,
                 crf_sigma_rgb: float = 15.0, crf_sigma_xy: float = 100.0,
                 crf_scale: float = 1.0, elb: Optional[ELB] = None, use_sl: bool = True, use_crf: bool = True,
                 use_size: bool = True, seeder=None, amp: bool = False,
                 init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000,
                 use_rgb: bool = False, rgb_lambda: float = 2e-9, rgb_sigma_rgb: float = 15.0,
                 rgb_scale: float = 1.0,
                 windows: Optional[Dict[str, tuple]] = None, prec: Optional[str] = None):
        if not model.freeze_cl:
            raise NotImplementedError("TCAM trains with freeze_cl=True (README.md:297)")
        self.model = model
        self.dev = next(model.parameters()).device
        if self.dev.type != "cuda":
            raise RuntimeError("training runs on the MI355X HIP path only")
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.lam_cfg = (sl_lambda if use_sl else 0.0, crf_lambda if use_crf else 0.0,
                        size_lambda if use_size else 0.0)
        self.use_cfg = (use_sl, use_crf, use_size)
        # RgbJointConRanFieldTcams (losses/tcam.py:158-232, --rgb_jcrf_tc): needs the
        # batch's (seq_iter, frm_iter) from the knn_tc loader
        self.rgb_cfg = ((float(rgb_lambda), float(rgb_sigma_rgb), float(rgb_scale)) if use_rgb
                        else None)
        # per-term epoch windows (*_tc_start_ep, *_tc_end_ep; ElementaryLoss.is_on,
        # losses/core.py:64-82): {"sl" | "crf" | "size" | "rgb": (start, end)}
        self.windows = dict(windows or {})
        self.epoch = 0
        self.set_epoch(0)
        self.sigma = (crf_sigma_rgb, crf_sigma_xy)
        self.crf_scale = float(crf_scale)   # --crf_tc_scale (dense_crf_loss.py:95-123)
        # the CRF lattice depends on the raw images only: built on a side stream while the
        # forward runs (crf.PreparedLattice), applied in the loss; TCAM_CRF_AHEAD=0 = inline
        self.crf_ahead = os.environ.get("TCAM_CRF_AHEAD", "1") != "0"
        self._crf_stream = None
        self._crf_pre = None    # the next step's lattice, built during this step's backward
        self.wgrad_side = os.environ.get("TCAM_WGRAD_SIDE", "1") != "0"
        # the fused BN-ReLU backward of the f16x3 step (TCAM_FUSED_BN_BWD=0: three passes)
        self.fused_bn_bwd = os.environ.get("TCAM_FUSED_BN_BWD", "1") != "0"
        self._wg_stream = None
        self._enc_stream = None
        self._enc_pre = None    # (images, version, plan, feats, event) of prefetch_encoder
        self.elb = elb or ELB()
        self.seeder = seeder
        self.steps = 0
        self.amp = bool(amp)
        # the fp32-accurate step's decoder: "f16x3" (default; TCAM_TRAIN_PREC=x6 restores x6):
        # activations (conv outputs, BN-ReLU outputs) in S2 on the f16x3 convolutions; the
        # gradients stay S3 and reach the f16x3 MFMA as per-channel scaled S2 copies (the
        # weight gradient divides the scales out in its reduction, the data gradient in its
        # per-step packed weights; tcam_dy_scaled_s2, tcam_pack_weight_f16x3)
        prec = prec or os.environ.get("TCAM_TRAIN_PREC", "f16x3")
        if prec not in ("f16x3", "x6"):
            raise ValueError(f"training precision {prec!r}: 'f16x3' or 'x6'")
        self.f16 = (not self.amp) and prec == "f16x3"
        self.fmt = "amp" if self.amp else ("f16x3" if self.f16 else "x6")  # decoder convs
        self.lay = ops.FMT_LAYOUT[self.fmt]           # and its activation layout
        self.glay = "s1" if self.amp else "s3"        # the gradients' layout
        # the 3x3 weight gradients of the fp32-accurate step: f16x3 (dy with per-channel
        # power-of-two scales, three fp16 MFMA products: half x6's work, the same fp64
        # error band) unless TCAM_WGRAD=x6
        self.wgrad_prec = "amp" if self.amp else \
            ("x6" if os.environ.get("TCAM_WGRAD", "f16x3") == "x6" else "f16x3")
        self.scaler_cfg = (float(growth_factor), float(backoff_factor), int(growth_interval))
        dec = model.decoder
        self.center = [_Conv(c) for c in dec.center] if isinstance(dec.center, CenterBlock) \
            else []
        self.blocks = [(_Conv(b.conv1), _Conv(b.conv2)) for b in dec.blocks]
        self.seg: nn.Conv2d = model.segmentation_head[0]
        # flat parameter / gradient / momentum buffers (parameter order = named_parameters)
        self.params: List[nn.Parameter] = [p for n, p in model.named_parameters()
                                           if n.startswith(("decoder.", "segmentation_head."))]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=self.dev, dtype=torch.float32)
        # gradient + one slot for the step's total loss: the DDP all-reduce carries the
        # loss with the gradient, and the SGD kernel skips the step on the device when the
        # summed loss is not finite (train_wsol.py:1181) — every rank sees the same sum
        # (AMP: one more slot, the GradScaler found_inf flag, summed over the ranks too)
        self._gbuf = torch.zeros(n + (2 if self.amp else 1), device=self.dev,
                                 dtype=torch.float32)
        self.grad = self._gbuf[:n]
        self.loss_gate = self._gbuf[n:n + 1]
        self.found_inf = self._gbuf[n + 1:n + 2] if self.amp else None
        # GradScaler state on the device (torch.cuda.amp.GradScaler: _scale, _growth_tracker)
        self.scale = torch.full((1,), float(init_scale), device=self.dev, dtype=torch.float32)
        self.growth_tracker = torch.zeros(1, device=self.dev, dtype=torch.int32)
        self.mom = torch.zeros(n, device=self.dev, dtype=torch.float32)
        # device counters: [applied steps, skipped (non-finite) steps]
        self.step_counts = torch.zeros(2, device=self.dev, dtype=torch.int32)
        self._finite = torch.zeros(1, device=self.dev, dtype=torch.float32)
        self.views: Dict[int, torch.Tensor] = {}
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view(p.shape)
            self.views[id(p)] = self.grad[off:off + k].view(p.shape)
            off += k
        # the BN modules' own running-statistics buffers are updated in place (never
        # re-bound: DDP and optimizers hold references to the module's tensors)
        self.bns = [c.bn for c in self._convs()]
        self.zero_bias: Dict[int, torch.Tensor] = {}
        self._bn_ws = None
        self._wg_ws = None
        self._chansum_ws = None
        self.repack()

    # ------------------------------------------------------------ helpers
    def set_epoch(self, epoch: int) -> None:
        """The Trainer's epoch (train_wsol.py:1046) as every loss term sees it: a term is
        active only inside its [start, end] window (losses/core.py:64-82)."""
        from .losses import loss_is_on
        self.epoch = int(epoch)
        on = {k: loss_is_on(*self.windows.get(k, (None, None)), self.epoch)
              for k in ("sl", "crf", "size", "rgb")}
        self.use = tuple(u and on[k] for u, k in zip(self.use_cfg, ("sl", "crf", "size")))
        self.lam = tuple(lm if on[k] else 0.0
                         for lm, k in zip(self.lam_cfg, ("sl", "crf", "size")))
        self.rgb = self.rgb_cfg if (self.rgb_cfg is not None and on["rgb"]) else None

    def _convs(self):
        out = list(self.center)
        for c1, c2 in self.blocks:
            out += [c1, c2]
        return out

    def g(self, p: torch.Tensor) -> torch.Tensor:
        return self.views[id(p)]

    def _zeros(self, n: int) -> torch.Tensor:
        z = self.zero_bias.get(n)
        if z is None:
            z = torch.zeros(n, device=self.dev, dtype=torch.float32)
            self.zero_bias[n] = z
        return z

    @staticmethod
    def _ws(cur: Optional[torch.Tensor], nbytes: int, dev) -> torch.Tensor:
        if cur is None or cur.numel() < nbytes:
            cur = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=dev)
        return cur

    def _pack_x6(self, w: torch.Tensor, mode: int, c0: int = 0, sel: int = 0,
                 cin_pad: int = 0) -> torch.Tensor:
        cout, ctot, kh, kw = w.shape
        K, M = (kh * kw * ctot, cout) if mode == 0 else (kh * kw * max(cout, cin_pad), sel)
        kp, mp = ops.conv_x6_weight_dims(K, M)
        out = torch.empty((kp // 32, 4, 3, mp, 8), device=self.dev, dtype=torch.bfloat16)
        check(_lib.load().tcam_pack_weight_x6(w.data_ptr(), out.data_ptr(), mode, cout, ctot, kh,
                                              kw, c0, sel, cin_pad, _stream()),
              "tcam_pack_weight_x6")
        return out

    def _pack(self, w: torch.Tensor, mode: int, c0: int = 0, sel: int = 0,
              cin_pad: int = 0) -> torch.Tensor:
        cout, ctot, kh, kw = w.shape
        if mode == 0:
            K, M = kh * kw * ctot, cout
        else:
            K, M = kh * kw * max(cout, cin_pad), sel
        kp, mp = ops.conv_x6_weight_dims(K, M)
        lib = _lib.load()
        if self.amp:   # autocast's fp16 weight
            out = torch.empty((kp // 32, 4, 1, mp, 8), device=self.dev, dtype=torch.float16)
            fn, name = lib.tcam_pack_weight_f16, "tcam_pack_weight_f16"
        else:
            out = torch.empty((kp // 32, 4, 3, mp, 8), device=self.dev, dtype=torch.bfloat16)
            fn, name = lib.tcam_pack_weight_x6, "tcam_pack_weight_x6"
        check(fn(w.data_ptr(), out.data_ptr(), mode, cout, ctot, kh, kw, c0, sel, cin_pad,
                 _stream()), name)
        return out

    @property
    def bn_flat(self) -> torch.Tensor:
        """A copy of every decoder BN running mean / var, concatenated."""
        return torch.cat([t.reshape(-1) for bn in self.bns
                          for t in (bn.running_mean, bn.running_var)])

    def set_bn_flat(self, flat: torch.Tensor) -> None:
        off = 0
        for bn in self.bns:
            for t in (bn.running_mean, bn.running_var):
                k = t.numel()
                t.copy_(flat[off:off + k].view_as(t))
                off += k

    def views_intact(self) -> bool:
        """True while every trainable Parameter still views this trainer's flat buffer
        (another trainer or a load that replaced ``.data`` breaks the aliasing)."""
        off = 0
        base = self.flat.data_ptr()
        for p in self.params:
            if p.data_ptr() != base + 4 * off:
                return False
            off += p.numel()
        return True

    def param_version(self) -> int:
        return sum(p._version for p in self.params)

    def _pack_f16(self, c: _Conv, w: torch.Tensor, mode: int, sel: int = 0,
                  kdiv: Optional[torch.Tensor] = None):
        """The f16x3 operand (+ per-column scales) of a trainable conv, packed on the device
        into the conv's own buffers; mode 1 = the data-gradient operand over the first
        ``sel`` input channels, divided by ``kdiv`` (dy's per-channel scales)."""
        cout, ctot, kh, kw = w.shape
        K, M = (kh * kw * ctot, cout) if mode == 0 else (kh * kw * cout, sel)
        kp, mp = ops.conv_x6_weight_dims(K, M)
        attr = ("wx6", "wsc") if mode == 0 else ("wdg", "dsc")
        wt, sc = getattr(c, attr[0]), getattr(c, attr[1])
        if wt is None or wt.dtype != torch.float16 or tuple(wt.shape) != (kp // 32, 4, 2, mp, 8):
            wt = torch.empty((kp // 32, 4, 2, mp, 8), device=self.dev, dtype=torch.float16)
            sc = torch.empty(mp, device=self.dev, dtype=torch.float32)
            setattr(c, attr[0], wt)
            setattr(c, attr[1], sc)
        check(_lib.load().tcam_pack_weight_f16x3(
            w.data_ptr(), wt.data_ptr(), sc.data_ptr(), mode, cout, ctot, kh, kw, 0,
            sel if mode else 0, 0, kdiv.data_ptr() if kdiv is not None else None, _stream()),
            "tcam_pack_weight_f16x3")
        return wt, sc

    def repack(self):
        """Split operands of every trainable conv from the flat fp32 weights."""
        self._packed_version = self.param_version()
        if self.f16:
            # the forward operands now; the data-gradient operands are packed in the
            # backward, once dy's scales are known
            for c in self._convs():
                self._pack_f16(c, c.conv.weight.data, 0)
            self.seg_dg = self._pack_x6(self.seg.weight.data, 1, 0, self.seg.in_channels,
                                        cin_pad=8)
            self.seg_w, self.seg_b = self.seg.weight.data, self.seg.bias.data
            return
        for c in self._convs():
            c.wx6 = self._pack(c.conv.weight.data, 0)
        for i, (c1, c2) in enumerate(self.blocks):
            c2.wdg = self._pack(c2.conv.weight.data, 1, 0, c2.ctot)
            c2.dg_cout = c2.ctot
            c1.wdg, c1.dg_cout = None, 0     # packed lazily (its slice depends on the input)
        for c in self.center:
            c.wdg = None
        # the seg head's data gradient reads dfcams padded to 8 channels
        self.seg_dg = self._pack(self.seg.weight.data, 1, 0, self.seg.in_channels, cin_pad=8)
        # the seg head's forward operands (AMP: autocast's fp16 weight and bias)
        if self.amp:
            self.seg_w = self.seg.weight.data.half().float()
            self.seg_b = self.seg.bias.data.half().float()
        else:
            self.seg_w, self.seg_b = self.seg.weight.data, self.seg.bias.data

    # --------------------------------------------------------------- ops
    def _bn_fwd(self, c: _Conv, y: torch.Tensor):
        lib = _lib.load()
        B, H, W, Cc = ops.s3_dims(y)
        P = B * H * W
        self._bn_ws = self._ws(self._bn_ws, int(lib.tcam_bn_ws_bytes(P, Cc)), self.dev)
        mean = torch.empty(Cc, device=self.dev)
        invstd = torch.empty(Cc, device=self.dev)
        bn = c.bn
        lay = self.lay
        check(getattr(lib, f"tcam_bn_stats_{lay}")(
            y.data_ptr(), P, Cc, bn.eps, bn.momentum, mean.data_ptr(), invstd.data_ptr(),
            bn.running_mean.data_ptr(), bn.running_var.data_ptr(), self._bn_ws.data_ptr(),
            _stream()), f"tcam_bn_stats_{lay}")
        out = torch.empty_like(y)
        check(getattr(lib, f"tcam_bn_relu_{lay}")(
            y.data_ptr(), mean.data_ptr(), invstd.data_ptr(), bn.weight.data_ptr(),
            bn.bias.data_ptr(), out.data_ptr(), P, Cc, _stream()), f"tcam_bn_relu_{lay}")
        return out, mean, invstd

    def _bn_bwd(self, c: _Conv, dout, out, y, mean, invstd):
        """dy of bn_relu (S3 / S1, the gradients' layout); the f16x3 step returns
        (dy2, scale): dy's per-channel scaled S2 copy for the f16x3 weight and data
        gradients (the max |dy| per channel comes out of the backward kernel itself)."""
        lib = _lib.load()
        B, H, W, Cc = ops.s3_dims(y)
        P = B * H * W
        self._bn_ws = self._ws(self._bn_ws, int(lib.tcam_bn_ws_bytes(P, Cc)), self.dev)
        if self.f16 and self.fused_bn_bwd:
            # one fused pass pair: the scaled S2 copy straight out of the backward (the
            # mask recomputed from y: every decoder BN is a BN-ReLU), DESIGN.md "Training"
            self._bn_ws = self._ws(self._bn_ws, int(lib.tcam_bn_bwd_scaled_ws_bytes(P, Cc)),
                                   self.dev)
            dy2 = ops.lay_empty("s2", B, H, W, Cc, self.dev)
            scale = torch.empty(Cc, device=self.dev, dtype=torch.float32)
            check(lib.tcam_bn_relu_bwd_scaled_s3s2(
                dout.data_ptr(), None, y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                c.bn.weight.data_ptr(), c.bn.bias.data_ptr(), None, dy2.data_ptr(),
                scale.data_ptr(), self.g(c.bn.weight).data_ptr(), self.g(c.bn.bias).data_ptr(),
                P, Cc, self._bn_ws.data_ptr(), _stream()), "tcam_bn_relu_bwd_scaled_s3s2")
            return dy2, scale
        if self.f16:
            dy = ops.lay_empty("s3", B, H, W, Cc, self.dev)
            amax = torch.empty(Cc, device=self.dev, dtype=torch.int32)
            check(lib.tcam_bn_relu_bwd_s3s2(dout.data_ptr(), out.data_ptr(), y.data_ptr(),
                                            mean.data_ptr(), invstd.data_ptr(),
                                            c.bn.weight.data_ptr(), dy.data_ptr(),
                                            self.g(c.bn.weight).data_ptr(),
                                            self.g(c.bn.bias).data_ptr(), P, Cc,
                                            self._bn_ws.data_ptr(), amax.data_ptr(), _stream()),
                  "tcam_bn_relu_bwd_s3s2")
            return self._dy_scaled(dy, amax)
        dy = torch.empty_like(y)
        if self.amp and self.fused_bn_bwd:   # two passes, the mask recomputed from y
            check(lib.tcam_bn_relu_bwd_fused_s1(
                dout.data_ptr(), None, y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                c.bn.weight.data_ptr(), c.bn.bias.data_ptr(), dy.data_ptr(),
                self.g(c.bn.weight).data_ptr(), self.g(c.bn.bias).data_ptr(), P, Cc,
                self._bn_ws.data_ptr(), _stream()), "tcam_bn_relu_bwd_fused_s1")
            return dy
        name = f"tcam_bn_relu_bwd_{self.lay}"
        check(getattr(lib, name)(dout.data_ptr(), out.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                 invstd.data_ptr(), c.bn.weight.data_ptr(), dy.data_ptr(),
                                 self.g(c.bn.weight).data_ptr(), self.g(c.bn.bias).data_ptr(),
                                 P, Cc, self._bn_ws.data_ptr(), _stream()), name)
        return dy

    def _dy_scaled(self, dy: torch.Tensor, amax: Optional[torch.Tensor] = None):
        """(dy2, scale): the per-channel power-of-two scaled S2 copy of an S3 gradient (max
        |dy_c| scale_c in [2^14, 2^15)); amax computed here when not given."""
        B, H, W, Cc = ops.s3_dims(dy)
        P = B * H * W
        compute = amax is None
        if compute:
            amax = torch.empty(Cc, device=self.dev, dtype=torch.int32)
        scale = torch.empty(Cc, device=self.dev, dtype=torch.float32)
        dy2 = ops.lay_empty("s2", B, H, W, Cc, self.dev)
        check(_lib.load().tcam_dy_scaled_s2(dy.data_ptr(), P, Cc, amax.data_ptr(),
                                            1 if compute else 0, scale.data_ptr(),
                                            dy2.data_ptr(), _stream()), "tcam_dy_scaled_s2")
        return dy2, scale

    def _wgrad_s2(self, srcs, dy2: torch.Tensor, dsc: torch.Tensor, dw: torch.Tensor,
                  cout_store: Optional[int] = None):
        """3x3 weight gradient of the f16x3 step: S2 sources, dy's scaled S2 copy."""
        lib = _lib.load()
        B, Ho, Wo, Cd = ops.s3_dims(dy2)
        arr = (tcam_conv_src * len(srcs))()
        for i, s in enumerate(srcs):
            _, H, W, Cc = ops.s3_dims(s.t)
            arr[i] = tcam_conv_src(s.t.data_ptr(), Cc, H, W, s.stride, 1 if s.up2 else 0)
        nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, len(srcs), B, Cd, Ho, Wo, 3, 3))
        self._wg_ws = self._ws(self._wg_ws, nb, self.dev)
        check(lib.tcam_conv_wgrad_s2_f16x3(arr, len(srcs), B, dy2.data_ptr(), dsc.data_ptr(), Cd,
                                           Ho, Wo, 3, 3, 1, 1, cout_store or Cd, dw.data_ptr(),
                                           self._wg_ws.data_ptr(), self._wg_ws.numel(),
                                           _stream()), "tcam_conv_wgrad_s2_f16x3")

    def _dgrad_f16(self, c: _Conv, dy2: torch.Tensor, dsc: torch.Tensor, sel: int, H: int,
                   W: int) -> torch.Tensor:
        """Data gradient of the f16x3 step w.r.t. the first ``sel`` input channels: the
        transposed / rotated weight packed this step over dy's scales, the f16x3 conv of
        dy2, an S3 output."""
        wt, sc = self._pack_f16(c, c.conv.weight.data, 1, sel, kdiv=dsc)
        return ops.conv2d_f16x3_s3out([ConvSrc(dy2)], wt, sc, self._zeros(sel), sel, H, W, 3, 1)

    def _wgrad(self, srcs, dy: torch.Tensor, cout: int, k, pad, dw: torch.Tensor,
               cout_store: Optional[int] = None):
        lib = _lib.load()
        B, Ho, Wo, Cd = ops.s3_dims(dy)
        kh, kw = (k, k) if isinstance(k, int) else k
        arr = (tcam_conv_src * len(srcs))()
        for i, s in enumerate(srcs):
            _, H, W, Cc = ops.s3_dims(s.t)
            arr[i] = tcam_conv_src(s.t.data_ptr(), Cc, H, W, s.stride, 1 if s.up2 else 0)
        nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, len(srcs), B, Cd, Ho, Wo, kh, kw))
        self._wg_ws = self._ws(self._wg_ws, nb, self.dev)
        args = (arr, len(srcs), B, dy.data_ptr(), Cd, Ho, Wo, kh, kw, pad, pad, cout_store or Cd,
                dw.data_ptr(), self._wg_ws.data_ptr(), self._wg_ws.numel())
        if self.wgrad_prec == "f16x3":
            # (an x beyond the fp16 range sets the f16x3 overflow flag: raised by the next
            # evaluation's check, ops.check_f16_overflow)
            name = "tcam_conv_wgrad_s3_f16x3"
            check(lib.tcam_conv_wgrad_s3_f16x3(*args, ops.f16_overflow_flag(self.dev).data_ptr(),
                                                _stream()), name)
        else:
            name = f"tcam_conv_wgrad_{self.lay}"
            check(getattr(lib, name)(*args, _stream()), name)

    # ------------------------------------------------------------ forward
    def forward(self, images: torch.Tensor):
        """Frozen encoder (eval, folded BN) + training decoder.  Returns (cl_logits, fcams,
        state) — the reference forward's outputs (base/model.py:124-162)."""
        m = self.model
        # the frozen encoder's folded plan: the model's own cache, re-folded whenever an
        # encoder parameter / buffer changes (load_state_dict, load_checkpoint, ...)
        # (the frozen encoder runs at the model's inference precision — f16x3 by default,
        # fp32-accurate at half x6's MFMA work — and its features enter the x6 decoder
        # re-laid out to S3, exactly)
        from .models import _encoder_plan_x6, _plan_exps, _precision, unscale_in
        prec = _precision(m)
        prec = prec if prec in ("x6", "f16x3") else "x6"
        if self.amp:
            prec = "amp"     # autocast covers the frozen encoder too (train_wsol.py:1162)
        enc = m._plan_get("enc_" + prec,
                          lambda: _encoder_plan_x6(m.encoder, images.device, prec), m.encoder)
        pre, self._enc_pre = self._enc_pre, None
        if pre is not None and pre[0] is images and pre[1] == images._version and pre[2] is enc:
            # the frozen encoder already ran on these images (prefetch_encoder); its own
            # overflow flag joins the device's flag now, in the step that uses the features
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(pre[4])
            feats = pre[3]
            for f in feats:
                f.record_stream(cur)
            pre[5].record_stream(cur)
            ops.merge_f16_overflow(pre[5])
        else:
            with torch.no_grad():
                feats = enc.forward(images.contiguous().float())
        head = m.classification_head
        # f16x3 plans store activation channels times 2^e (models.act_exponents): the
        # classifier absorbs them, the x6 decoder gets the features unscaled (exact on S3)
        exps = _plan_exps(enc, len(feats))
        cl_logits = ops.wgap_s3(feats[-1], unscale_in(head.fc.weight.detach().contiguous(),
                                                      exps[-1]),
                                head.fc.bias.detach().contiguous())
        if self.f16:
            # S2 features straight into the f16x3 decoder (a feature with channel exponents
            # is unscaled on an exact S3 copy and re-split)
            fs = [ops.relayout(f, "f16x3") if e is None else
                  ops.relayout(ops.scale_channels(ops.relayout(f, "x6"), e, negate=True),
                               "f16x3")
                  for f, e in zip(list(feats[1:])[::-1], list(exps[1:])[::-1])]
        else:
            fs = [ops.scale_channels(ops.relayout(f, self.fmt), e, negate=True)
                  for f, e in zip(list(feats[1:])[::-1], list(exps[1:])[::-1])]
        x, skips = fs[0], fs[1:]
        st = {"center": [], "blocks": []}
        for c in self.center:
            H, W = x.shape[1], x.shape[2]
            y = ops.conv2d_x6([ConvSrc(x)], c.wx6, self._zeros(c.cout), c.cout, H, W, 3, 1,
                              False, wscale=c.wsc if self.f16 else None)
            a, mean, inv = self._bn_fwd(c, y)
            st["center"].append((x, y, a, mean, inv))
            x = a
        for i, (c1, c2) in enumerate(self.blocks):
            skip = skips[i] if i < len(skips) else None
            h, w = x.shape[1], x.shape[2]
            resized = None
            if skip is None:
                srcs = [ConvSrc(x, up2=True)]
                Ho, Wo = 2 * h, 2 * w
            else:
                Ho, Wo = skip.shape[1], skip.shape[2]
                if (2 * h, 2 * w) == (Ho, Wo):
                    srcs = [ConvSrc(x, up2=True), ConvSrc(skip)]
                else:
                    resized = ops.up2_resize_s3(x, (Ho, Wo))
                    srcs = [ConvSrc(resized), ConvSrc(skip)]
            y1 = ops.conv2d_x6(srcs, c1.wx6, self._zeros(c1.cout), c1.cout, Ho, Wo, 3, 1, False,
                               wscale=c1.wsc if self.f16 else None)
            a1, m1, i1 = self._bn_fwd(c1, y1)
            y2 = ops.conv2d_x6([ConvSrc(a1)], c2.wx6, self._zeros(c2.cout), c2.cout, Ho, Wo, 3,
                               1, False, wscale=c2.wsc if self.f16 else None)
            a2, m2, i2 = self._bn_fwd(c2, y2)
            st["blocks"].append(dict(x=x, srcs=srcs, resized=resized, y1=y1, a1=a1, m1=m1,
                                     i1=i1, y2=y2, a2=a2, m2=m2, i2=i2, hw=(h, w)))
            x = a2
        fcams, _, _ = ops.seghead_cam_s3(x, self.seg_w, self.seg_b, want_fcams=True,
                                         want_u8=False)
        if self.amp:   # the seg head's fp16 autocast output
            fcams = fcams.half().float()
        st["seg_hw"] = None
        if tuple(fcams.shape[2:]) != tuple(images.shape[2:]):
            # base/model.py:148-154: fcams resized (bilinear, align_corners=True) to the
            # input size (InceptionV3: 300 -> 299); the backward takes its adjoint
            st["seg_hw"] = tuple(fcams.shape[2:])
            fcams, _, _ = ops.resize_cam(fcams, tuple(images.shape[2:]), want_fcams=True,
                                         want_u8=False)
        st["dec_out"] = x
        m.x_in = images
        m.cams = fcams.detach()
        return cl_logits, fcams, st

    # ----------------------------------------------------------- the step
    def step(self, images: torch.Tensor, raw_imgs: Optional[torch.Tensor],
             seeds: Optional[torch.Tensor] = None, std_cams: Optional[torch.Tensor] = None,
             roi: Optional[torch.Tensor] = None, seq_iter=None,
             frm_iter=None, next_images: Optional[torch.Tensor] = None,
             next_raw: Optional[torch.Tensor] = None) -> Dict[str, float]:
        """One optimisation step on a batch; returns the device loss tensor (4,):
        total, self-learning, CRF, size (5 with RgbJointConRanFieldTcams on: its value
        last).

        Seeds come from the caller, or — as train_wsol.py:846-859 — from the stage-1
        CAMs ``std_cams`` (b, 1, h', w') through ``prepare_std_cams_disq`` and
        ``self.seeder`` (a :class:`~tcam_wsol_video_amd.seeding.TCAMSeeder`).
        ``seq_iter`` / ``frm_iter``: the knn_tc loader's per-frame sequence / frame-order
        ids (wsol_loader.py:616-624), needed by the RgbJoint term.
        ``next_images``: the next step's batch, already enqueued by the caller: its frozen
        encoder forward runs on a side stream while this step's backward runs
        (:meth:`prefetch_encoder`; the next step uses it if it gets the same, unmodified
        tensor).  ``next_raw``: likewise the next batch's raw frames, whose CRF lattice is
        then built during this step's backward."""
        next_ready = None
        if next_images is not None or next_raw is not None:
            next_ready = torch.cuda.Event()
            next_ready.record(torch.cuda.current_stream(self.dev))
        if seeds is None and std_cams is not None and self.use[0]:
            if self.seeder is None:
                raise ValueError("std_cams given but DecoderTrainer.seeder is not set")
            cams_inter = prepare_std_cams(std_cams, tuple(images.shape[2:]))
            seeds = self.seeder.seeds_i32(cams_inter, roi)
        if (self.use[1] or self.rgb is not None) and raw_imgs is None:
            raise ValueError("the CRF loss needs the raw images (values in [0, 255])")
        rgb = None
        if self.rgb_cfg is not None:
            # the term stays in the loss vector (0 outside its epoch window)
            from .losses import group_ordered_frames
            if self.rgb is None:
                rgb = (0.0, self.rgb_cfg[1], [], self.rgb_cfg[2])
            else:
                if seq_iter is None or frm_iter is None:
                    raise ValueError("RgbJointConRanFieldTcams needs seq_iter / frm_iter "
                                     "(knn_tc batches)")
                rgb = (self.rgb[0], self.rgb[1], group_ordered_frames(seq_iter, frm_iter),
                       self.rgb[2])
        lattice, pre = None, self._crf_pre
        self._crf_pre = None
        crf_on = self.crf_ahead and self.use[1] and self.lam[1] and self.crf_scale == 1.0
        if pre is not None and crf_on and pre.matches(raw_imgs, *self.sigma):
            lattice = pre          # built during the previous step's backward
        elif pre is not None:
            pre.discard()
        if crf_on and lattice is None:
            if self._crf_stream is None:
                self._crf_stream = torch.cuda.Stream(device=self.dev)
            lattice = crf.PreparedLattice(raw_imgs.to(device=self.dev, dtype=torch.float32),
                                          2, self.sigma[0], self.sigma[1],
                                          stream=self._crf_stream)
        try:
            cl_logits, fcams, st = self.forward(images)
            use_raw = self.use[1] or (rgb is not None and rgb[2])
            losses, dF = tcam_losses(fcams, raw_imgs if use_raw else None,
                                     seeds if self.use[0] else None, self.lam, self.elb.t,
                                     self.sigma, rgb=rgb if (rgb and rgb[2]) else None,
                                     crf_scale=self.crf_scale, lattice=lattice)
        except BaseException:
            # a lattice prepared for this step that was never applied holds a pooled
            # workspace (and a filled hash table): release it
            if lattice is not None and lattice._slot is not None:
                lattice.discard()
            raise
        if rgb is not None and not rgb[2]:   # term off this epoch: a zero slot
            losses = torch.cat([losses, torch.zeros(1, device=losses.device)])
        self.loss_gate.copy_(losses[:1])
        if self.amp:   # scaler.scale(loss).backward(): d(S loss)/d fcams, an fp16 tensor
            dF = (dF * self.scale).half().float()
        self.backward(dF, st)
        if next_images is not None:
            self.prefetch_encoder(next_images, ready=next_ready)
        if next_raw is not None and crf_on and next_raw.is_cuda:
            self._crf_pre = crf.PreparedLattice(next_raw, 2, self.sigma[0], self.sigma[1],
                                                stream=self._crf_stream, ready=next_ready)
        if not self.amp:
            # an f16x3 operand beyond the fp16 range (the frozen encoder's convolutions or
            # the f16x3 weight gradient) made this step's gradient invalid: the loss slot
            # becomes NaN, so the gated SGD kernel skips the step on every rank (the flag
            # stays set until check_overflow() reports it)
            self.loss_gate.masked_fill_(ops.f16_overflow_flag(self.dev).bool(), float("nan"))
        if self.amp:   # scaler.unscale_: 1/scale, non-finite check (device)
            self.found_inf.zero_()
            check(_lib.load().tcam_amp_unscale(self.grad.data_ptr(), self.grad.numel(),
                                               self.scale.data_ptr(),
                                               self.found_inf.data_ptr(), _stream()),
                  "tcam_amp_unscale")
        self.all_reduce_and_step(gated=True)
        self.steps += 1
        return losses

    def prefetch_encoder(self, images: torch.Tensor,
                         ready: Optional["torch.cuda.Event"] = None) -> None:
        """The frozen encoder's forward of ``images`` on a side stream (after ``ready``, or
        after the work queued so far on the current stream); the next :meth:`forward` of the
        same, unmodified tensor takes these features instead of recomputing them.  The
        encoder is frozen (eval plan, no parameter it reads changes in a step), so the
        features are the ones the forward would compute."""
        from .models import _encoder_plan_x6, _precision
        m = self.model
        prec = _precision(m)
        prec = prec if prec in ("x6", "f16x3") else "x6"
        if self.amp:
            prec = "amp"
        enc = m._plan_get("enc_" + prec,
                          lambda: _encoder_plan_x6(m.encoder, images.device, prec), m.encoder)
        if self._enc_stream is None:
            self._enc_stream = torch.cuda.Stream(device=self.dev)
        side = self._enc_stream
        cur = torch.cuda.current_stream(self.dev)
        x = images.contiguous().float()
        if ready is not None and x is images:
            side.wait_event(ready)
        else:
            # (a conversion just enqueued on the current stream must land first)
            side.wait_stream(cur)
        x.record_stream(side)
        with torch.cuda.stream(side), torch.no_grad():
            # the prefetch's own overflow flag: the gate of THIS step (read on the current
            # stream, not ordered against the side stream) must not see the next batch's
            # overflow; forward() merges it when the features are used
            flag = torch.zeros(1, dtype=torch.int32, device=self.dev)
            with ops.f16_overflow_into(flag):
                feats = enc.forward(x)
            ev = torch.cuda.Event()
            ev.record(side)
        self._enc_pre = (images, images._version, enc, feats, ev, flag)

    def close(self) -> None:
        """Release what a step left for the next one: the next batch's prepared CRF lattice
        (its pooled workspace) and the prefetched encoder features (end of an epoch or of
        training, or after a failed step)."""
        pre, self._crf_pre = self._crf_pre, None
        if pre is not None:
            pre.discard()
        self._enc_pre = None

    def check_overflow(self) -> None:
        """Raise (a host sync) when an f16x3 operand left the fp16 range since the last
        check: those steps were skipped on the device, and the run must switch precision.
        Under torch.distributed a collective: the flag is MAX-reduced over the ranks first,
        so every rank raises together or none does (the gated SGD already skipped the step
        on every rank)."""
        try:
            ops.check_f16_overflow(self.dev, all_ranks=True)
        except FloatingPointError:
            raise FloatingPointError(
                "an f16x3 operand exceeded the fp16 range |x| <= 65504 during training: the "
                "affected steps were skipped.  Train the decoder's 3x3 weight gradients on "
                "x6 (TCAM_WGRAD=x6) and run the frozen encoder on x6 "
                "(model.conv_precision = 'x6')") from None

    @property
    def applied_steps(self) -> int:
        """SGD steps applied (steps whose all-reduced loss was finite); a host sync."""
        return int(self.step_counts[0].item())

    @property
    def skipped_steps(self) -> int:
        return int(self.step_counts[1].item())

    def backward(self, dF: torch.Tensor, st):
        """Decoder + seg-head backward.  The weight gradients only feed the optimizer, so
        they run on a side stream (``_wgrad_side``) beside the data-gradient chain, joined
        here before returning; TCAM_WGRAD_SIDE=0 keeps them inline."""
        try:
            self._backward_impl(dF, st)
        finally:
            if self._wg_stream is not None:
                torch.cuda.current_stream(self.dev).wait_stream(self._wg_stream)

    def _wgrad_side(self, fn, *tensors):
        """Runs ``fn`` (a weight-gradient launch) on the side stream after everything queued
        so far on the current stream; the tensors it reads are marked in use by that stream
        so the allocator does not hand their memory out before it is done."""
        if not self.wgrad_side:
            fn()
            return
        if self._wg_stream is None:
            self._wg_stream = torch.cuda.Stream(device=self.dev)
        side = self._wg_stream
        side.wait_stream(torch.cuda.current_stream(self.dev))
        for t in tensors:
            t.record_stream(side)
        with torch.cuda.stream(side):
            fn()

    def _backward_impl(self, dF: torch.Tensor, st):
        lib = _lib.load()
        if st.get("seg_hw") is not None:    # adjoint of the fcams resize
            Hs, Ws = st["seg_hw"]
            d = torch.empty((dF.shape[0], 2, Hs, Ws), device=dF.device, dtype=torch.float32)
            check(lib.tcam_resize_ac_bwd(dF.data_ptr(), d.data_ptr(), dF.shape[0] * 2, Hs, Ws,
                                         dF.shape[2], dF.shape[3], _stream()),
                  "tcam_resize_ac_bwd")
            dF = d
        B, _, H, W = dF.shape
        x16 = st["dec_out"]
        cin = ops.s3_dims(x16)[3]
        # seg head: bias grad, weight grad (dy = dfcams padded to 8 channels), data grad
        self._chansum_ws = self._ws(self._chansum_ws,
                                    int(lib.tcam_chansum_ws_bytes(B, 2, H * W)), self.dev)
        check(lib.tcam_chansum_nchw(dF.data_ptr(), B, 2, H * W, self.g(self.seg.bias).data_ptr(),
                                    self._chansum_ws.data_ptr(), _stream()), "tcam_chansum_nchw")
        if self.amp:   # the fp16 bias of the autocast seg-head conv: an fp16 gradient
            gb = self.g(self.seg.bias)
            gb.copy_(gb.half().float())
        if self.f16:
            return self._backward_f16(dF, st, x16, cin)
        dF8 = ops.s3_from_nchw(dF, 8, self.fmt)
        self._wgrad_side(lambda: self._wgrad([ConvSrc(x16)], dF8, 8, 3, 1,
                                             self.g(self.seg.weight), cout_store=2), x16, dF8)
        dx = ops.conv2d_x6([ConvSrc(dF8)], self.seg_dg, self._zeros(cin), cin, H, W, 3, 1, False)
        for bi in range(len(self.blocks) - 1, -1, -1):
            c1, c2 = self.blocks[bi]
            s = st["blocks"][bi]
            Ho, Wo = s["y1"].shape[1], s["y1"].shape[2]
            dy2 = self._bn_bwd(c2, dx, s["a2"], s["y2"], s["m2"], s["i2"])
            self._wgrad_side(lambda: self._wgrad([ConvSrc(s["a1"])], dy2, c2.cout, 3, 1,
                                                 self.g(c2.conv.weight)), s["a1"], dy2)
            da1 = ops.conv2d_x6([ConvSrc(dy2)], c2.wdg, self._zeros(c2.ctot), c2.ctot, Ho, Wo,
                                3, 1, False)
            dy1 = self._bn_bwd(c1, da1, s["a1"], s["y1"], s["m1"], s["i1"])
            self._wgrad_side(lambda: self._wgrad(s["srcs"], dy1, c1.cout, 3, 1,
                                                 self.g(c1.conv.weight)),
                             dy1, *[q.t for q in s["srcs"]])
            if bi == 0 and not self.center:
                break   # the encoder is frozen: no gradient below the first block
            # gradient w.r.t. the block input x (first source channels only)
            cx = ops.s3_dims(s["x"])[3]
            if c1.wdg is None or c1.dg_cout != cx:
                c1.wdg = self._pack(c1.conv.weight.data, 1, 0, cx)
                c1.dg_cout = cx
            dxu = ops.conv2d_x6([ConvSrc(dy1)], c1.wdg, self._zeros(cx), cx, Ho, Wo, 3, 1,
                                False)
            h, w = s["hw"]
            dx = ops.lay_empty(self.lay, B, h, w, cx, self.dev)
            if s["resized"] is not None:
                name = f"tcam_up2_resize_bwd_{self.lay}"
                check(getattr(lib, name)(dxu.data_ptr(), dx.data_ptr(), B, cx, h, w, Ho, Wo,
                                         _stream()), name)
            else:
                name = f"tcam_up2_bwd_{self.lay}"
                check(getattr(lib, name)(dxu.data_ptr(), dx.data_ptr(), B, cx, h, w, _stream()),
                      name)
        for ci in range(len(self.center) - 1, -1, -1):
            c = self.center[ci]
            xin, y, a, mean, inv = st["center"][ci]
            dyc = self._bn_bwd(c, dx, a, y, mean, inv)
            self._wgrad_side(lambda: self._wgrad([ConvSrc(xin)], dyc, c.cout, 3, 1,
                                                 self.g(c.conv.weight)), xin, dyc)
            if ci > 0:
                if c.wdg is None:
                    c.wdg = self._pack(c.conv.weight.data, 1, 0, c.ctot)
                Hc, Wc = y.shape[1], y.shape[2]
                dx = ops.conv2d_x6([ConvSrc(dyc)], c.wdg, self._zeros(c.ctot), c.ctot, Hc, Wc,
                                   3, 1, False)

    def _backward_f16(self, dF: torch.Tensor, st, x16: torch.Tensor, cin: int):
        """The f16x3 step's backward below the seg-head bias: gradients in S3, each
        reaching the f16x3 weight / data gradients as its per-channel scaled S2 copy."""
        lib = _lib.load()
        B, _, H, W = dF.shape
        dF8 = ops.s3_from_nchw(dF, 8, "x6")
        d2, dsc = self._dy_scaled(dF8)
        self._wgrad_side(lambda: self._wgrad_s2([ConvSrc(x16)], d2, dsc, self.g(self.seg.weight),
                                                cout_store=2), x16, d2, dsc)
        # the seg head's data gradient: x6 on dfcams (S3; 8 -> 16 channels, cheap)
        dx = ops.conv2d_x6([ConvSrc(dF8)], self.seg_dg, self._zeros(cin), cin, H, W, 3, 1, False)
        for bi in range(len(self.blocks) - 1, -1, -1):
            c1, c2 = self.blocks[bi]
            s = st["blocks"][bi]
            Ho, Wo = s["y1"].shape[1], s["y1"].shape[2]
            dy2, sc2 = self._bn_bwd(c2, dx, s["a2"], s["y2"], s["m2"], s["i2"])
            self._wgrad_side(lambda: self._wgrad_s2([ConvSrc(s["a1"])], dy2, sc2,
                                                    self.g(c2.conv.weight)), s["a1"], dy2, sc2)
            da1 = self._dgrad_f16(c2, dy2, sc2, c2.ctot, Ho, Wo)
            dy1, sc1 = self._bn_bwd(c1, da1, s["a1"], s["y1"], s["m1"], s["i1"])
            self._wgrad_side(lambda: self._wgrad_s2(s["srcs"], dy1, sc1, self.g(c1.conv.weight)),
                             dy1, sc1, *[q.t for q in s["srcs"]])
            if bi == 0 and not self.center:
                break   # the encoder is frozen: no gradient below the first block
            # gradient w.r.t. the block input x (first source channels only)
            cx = ops.s3_dims(s["x"])[3]
            dxu = self._dgrad_f16(c1, dy1, sc1, cx, Ho, Wo)
            h, w = s["hw"]
            dx = ops.lay_empty("s3", B, h, w, cx, self.dev)
            if s["resized"] is not None:
                check(lib.tcam_up2_resize_bwd_s3(dxu.data_ptr(), dx.data_ptr(), B, cx, h, w, Ho,
                                                 Wo, _stream()), "tcam_up2_resize_bwd_s3")
            else:
                check(lib.tcam_up2_bwd_s3(dxu.data_ptr(), dx.data_ptr(), B, cx, h, w, _stream()),
                      "tcam_up2_bwd_s3")
        for ci in range(len(self.center) - 1, -1, -1):
            c = self.center[ci]
            xin, y, a, mean, inv = st["center"][ci]
            dyc, scc = self._bn_bwd(c, dx, a, y, mean, inv)
            self._wgrad_side(lambda: self._wgrad_s2([ConvSrc(xin)], dyc, scc,
                                                    self.g(c.conv.weight)), xin, dyc, scc)
            if ci > 0:
                dx = self._dgrad_f16(c, dyc, scc, c.ctot, y.shape[1], y.shape[2])

    def all_reduce_and_step(self, gated: bool = False):
        """DDP gradient average (RCCL all-reduce of the flat buffer), BN buffer broadcast
        from rank 0, SGD update of the flat weights, repack of the conv operands.
        ``gated``: the step is skipped on the device when the all-reduced loss slot
        (``loss_gate``) is not finite (train_wsol.py:1181)."""
        scale = 1.0
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(self._gbuf if gated else self.grad, op=dist.ReduceOp.SUM)
            bn = self.bn_flat
            dist.broadcast(bn, src=0)       # DDP broadcast_buffers: rank 0's statistics
            self.set_bn_flat(bn)
            scale = 1.0 / dist.get_world_size()
        cnt = self.step_counts
        if self.amp:   # scaler.step(optimizer) + scaler.update(), on the device
            g, b, itv = self.scaler_cfg
            check(_lib.load().tcam_sgd_step_amp(
                self.flat.data_ptr(), self.grad.data_ptr(), self.mom.data_ptr(),
                self.flat.numel(), self.lr, self.momentum, self.dampening, self.weight_decay,
                1 if self.nesterov else 0, scale, self._gbuf[-2:].data_ptr(), cnt.data_ptr(),
                cnt.data_ptr() + 4, self.scale.data_ptr(), self.growth_tracker.data_ptr(),
                g, b, itv, _stream()), "tcam_sgd_step_amp")
            # one multi-tensor launch for every BN's counter
            torch._foreach_add_([bn.num_batches_tracked for bn in self.bns], 1)
            self.repack()
            self.model.invalidate_plans(DECODER_PLANS)
            return
        gate = self.loss_gate if gated else self._finite
        check(_lib.load().tcam_sgd_step_gated(self.flat.data_ptr(), self.grad.data_ptr(),
                                              self.mom.data_ptr(), self.flat.numel(), self.lr,
                                              self.momentum, self.dampening, self.weight_decay,
                                              1 if self.nesterov else 0, scale, gate.data_ptr(),
                                              cnt.data_ptr(), cnt.data_ptr() + 4, _stream()),
              "tcam_sgd_step_gated")
        # one multi-tensor launch for every BN's counter
        torch._foreach_add_([bn.num_batches_tracked for bn in self.bns], 1)
        self.repack()
        self.model.invalidate_plans(DECODER_PLANS)


class MyStepLR(torch.optim.lr_scheduler.StepLR):
    """learning/lr_scheduler.py:6-35: StepLR whose rate never drops below ``min_lr``
    (lr = max(base_lr * gamma ** (epoch // step_size), min_lr)); stepped once per epoch
    after the evaluation (main.py:93-114, train_wsol.py:1853-1854)."""

    def __init__(self, optimizer, step_size, gamma=0.1, last_epoch=-1, min_lr=1e-6):
        self.step_size, self.gamma, self.min_lr = step_size, gamma, min_lr
        torch.optim.lr_scheduler.LRScheduler.__init__(self, optimizer, last_epoch)

    def get_lr(self):
        k = self.last_epoch // self.step_size
        return [max(b * self.gamma ** k, self.min_lr) for b in self.base_lrs]


class _TrainerStepLR(MyStepLR):
    """MyStepLR over a host-side stand-in of the reference's TCAM optimizer (one group at
    the trainer's lr, instantiators.py:751-754): ``trainer.lr`` follows every ``step()``;
    ``state_dict()`` is what the reference checkpoints as 'lr_scheduler'."""

    def __init__(self, trainer, step_size, gamma, min_lr):
        self._trainer = trainer
        shadow = torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=trainer.lr)
        super().__init__(shadow, step_size=step_size, gamma=gamma, min_lr=min_lr)

    def step(self, epoch=None):
        self.optimizer.step()   # no gradients: a no-op that keeps the scheduler's order check
        super().step()
        self._trainer.lr = float(self.optimizer.param_groups[0]["lr"])

    def state_dict(self):
        sd = super().state_dict()
        sd.pop("_trainer", None)
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self.optimizer.param_groups[0]["lr"] = self.get_last_lr()[0]
        self._trainer.lr = float(self.get_last_lr()[0])


def lr_schedule(trainer: "DecoderTrainer", step_size: int, gamma: float,
                min_lr: float) -> MyStepLR:
    """The trainer's per-epoch learning-rate schedule (opt__lr_scheduler, 'mystep')."""
    return _TrainerStepLR(trainer, step_size, gamma, min_lr)


class _TrainForward(torch.autograd.Function):
    """UnetTCAM.forward in train mode as one autograd node over the device kernels:
    forward = DecoderTrainer.forward (frozen eval encoder, batch-statistics decoder BN),
    backward = DecoderTrainer.backward (seg head, BN, wgrad and dgrad kernels).  Gradients
    reach the decoder / seg-head Parameters through autograd, so a reference loop —
    ``loss = MasterLoss(...)(fcams=model(x)[1], ...); loss.backward(); opt.step()`` —
    and DDP's gradient hooks (parallel/my_ddp.py) work unchanged (train_wsol.py:1162-1184,
    base/model.py:124-162)."""

    @staticmethod
    def forward(ctx, engine, images, *params):
        cl_logits, fcams, st = engine.forward(images)
        ctx.engine, ctx.st = engine, st
        ctx.mark_non_differentiable(cl_logits)
        return cl_logits, fcams

    @staticmethod
    def backward(ctx, g_logits, g_fcams):
        eng, st = ctx.engine, ctx.st
        ctx.st = None
        if st is None:
            raise RuntimeError("UnetTCAM train-mode forward: backward called twice")
        eng.backward(g_fcams.contiguous().float(), st)
        return (None, None) + tuple(eng.g(p).clone() for p in eng.params)


def train_forward(model: UnetTCAM, images: torch.Tensor):
    """(cl_logits, fcams) of a UnetTCAM in train mode (decoder BN on batch statistics,
    running statistics updated), differentiable w.r.t. the decoder and seg head when grad
    mode is on.  Used by UnetTCAM.forward when ``model.training``."""
    eng = model.__dict__.get("_train_engine")
    if eng is None or not eng.views_intact():
        eng = DecoderTrainer(model)
        model.__dict__["_train_engine"] = eng
    elif eng.param_version() != eng._packed_version:
        eng.repack()    # an optimizer stepped the Parameters in place
    if torch.is_grad_enabled() and any(p.requires_grad for p in eng.params):
        cl_logits, fcams = _TrainForward.apply(eng, images, *eng.params)
    else:
        cl_logits, fcams, _ = eng.forward(images)
    # nn.BatchNorm2d.forward in train mode (one multi-tensor launch for every BN's counter)
    torch._foreach_add_([bn.num_batches_tracked for bn in eng.bns], 1)
    model.invalidate_plans(DECODER_PLANS)   # running statistics moved
    return cl_logits, fcams
