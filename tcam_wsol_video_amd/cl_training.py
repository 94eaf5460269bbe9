"""Stage-1 training on the gfx950 kernels: the STD_CL classifier (ResNet50 encoder + WGAP
head) trained end to end — the reference's ``Trainer._wsol_training`` for task STD_CL
(learning/train_wsol.py:700-714: ``cl_logits = model(images)``, ``loss = ClLoss``) with
``--freeze_encoder False`` (README.md:239-266), the run whose best weights every TCAM run
starts from (README.md:267-276).

Forward (train mode, encoders/resnet.py:140-232, poolings/core.py:109-115): every conv on
the MFMA conv kernels with batch-statistics BatchNorm (running statistics updated), the
Bottleneck tail ``relu(bn3(conv3) + shortcut)`` as one kernel, WGAP's pool + fc.
Loss: ``nn.CrossEntropyLoss`` (losses/std.py:19-53).  Backward: the head, then each
Bottleneck in reverse — BN backward (masks from the block output), the data gradients as
the forward conv of dy with the packed transposed weights (a stride-2 conv's through zero
insertion; conv1 and the projection shortcut in one K-concatenated launch), the weight
gradients (1x1: ``tcam_wgrad11_*``; 3x3 stride 1: the decoder's ``tcam_conv_wgrad_s2_f16x3``;
the 3x3/2 conv through zero insertion; the 7x7/2 stem as im2col + the 1x1 GEMM) on a side
stream beside the data-gradient chain — the max-pool adjoint, the stem BN.  Update:
torch.optim.SGD with the reference's two parameter groups (process/instantiators.py:736-807:
``encoder.layer4.*`` and ``classification_head.*`` at ``lr * lr_classifier_ratio``), momentum
0.9, nesterov, weight decay 1e-4 (configure/config.py:177-202), skipped on the device when the
loss is not finite (train_wsol.py:1181).

Precision: ``prec="f16x3"`` (default, fp32-accurate: activations S2, gradients S3, the
MFMA operands per-channel scaled S2 copies — the decoder step's scheme, DESIGN.md "The
f16x3 training step"), or ``amp=True`` — the README's ``--amp True``: autocast's fp16
convolutions on S1 tensors with a device-side GradScaler (train_wsol.py:1077, 1155-1184).

Multi-GPU: one process per GPU; the flat gradient buffer (with the loss slot) is
all-reduced and averaged, rank 0's BatchNorm running statistics are broadcast (DDP).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from . import _lib, ops
from ._lib import check, tcam_conv_src, tcam_pack_item
from .models import RESNET50, STDClassifier
from .ops import ConvSrc

# STDClassifier's eval plans fold encoder weights / BN statistics
ENCODER_PLANS = ("enc_x6", "enc_f16x3", "enc_amp", "enc")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class _EConv:
    """One trainable encoder conv (no bias) and the BatchNorm after it, with its packed
    operands: ``wt`` / ``wsc`` the forward's, ``dwt`` / ``dsc`` the data gradient's."""

    __slots__ = ("conv", "bn", "cout", "cin", "k", "stride", "pad", "wt", "wsc", "cin_pad", "dwt")

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d, cin_pad: int = 0):
        self.conv, self.bn = conv, bn
        self.cout, self.cin = conv.out_channels, conv.in_channels
        self.k = conv.kernel_size[0]
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.wt = self.wsc = None
        self.cin_pad = cin_pad
        self.dwt = None   # AMP: the data gradient's operand, packed with the forward's


class _Block:
    __slots__ = ("c1", "c2", "c3", "ds")

    def __init__(self, blk):
        self.c1 = _EConv(blk.conv1, blk.bn1)
        self.c2 = _EConv(blk.conv2, blk.bn2)
        self.c3 = _EConv(blk.conv3, blk.bn3)
        self.ds = _EConv(blk.downsample[0], blk.downsample[1]) if blk.downsample is not None \
            else None


class ClassifierTrainer:
    """Trains every parameter of a ResNet50 ``STDClassifier`` (encoder + WGAP head)."""

    def __init__(self, model: STDClassifier, lr: float = 0.001, momentum: float = 0.9,
                 dampening: float = 0.0, weight_decay: float = 1e-4, nesterov: bool = True,
                 lr_classifier_ratio: float = 10.0, cl_lambda: float = 1.0, amp: bool = False,
                 init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000,
                 prec: Optional[str] = None):
        if getattr(model, "encoder_name", None) != RESNET50:
            raise NotImplementedError("stage-1 training runs the ResNet50 encoder "
                                      "(README.md:239-266)")
        self.model = model
        self.dev = next(model.parameters()).device
        if self.dev.type != "cuda":
            raise RuntimeError("training runs on the MI355X HIP path only")
        self.momentum, self.dampening = momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.lr_ratio = float(lr_classifier_ratio)
        self.lrs = [float(lr), float(lr) * self.lr_ratio]   # the two parameter groups
        self.cl_lambda = float(cl_lambda)
        self.amp = bool(amp)
        prec = prec or os.environ.get("TCAM_TRAIN_PREC", "f16x3")
        if not self.amp and prec != "f16x3":
            raise ValueError(f"stage-1 training precision {prec!r}: 'f16x3' (or amp=True)")
        self.fmt = "amp" if self.amp else "f16x3"
        self.lay = ops.FMT_LAYOUT[self.fmt]      # activations: S1 / S2
        self.glay = "s1" if self.amp else "s3"   # gradients: S1 / S3
        self.scaler_cfg = (float(growth_factor), float(backoff_factor), int(growth_interval))
        enc = model.encoder
        self.stem = _EConv(enc.conv1, enc.bn1, cin_pad=8)
        self.layers: List[List[_Block]] = [[_Block(b) for b in layer]
                                           for layer in (enc.layer1, enc.layer2, enc.layer3,
                                                         enc.layer4)]
        self.fc: nn.Linear = model.classification_head.fc
        # flat parameter / gradient / momentum buffers (named_parameters order: the
        # encoder, whose layer4 is last, then the head — so the reference's second
        # parameter group, layer4 + head at lr * lr_classifier_ratio, is the tail)
        named = list(model.named_parameters())
        self.params: List[nn.Parameter] = [p for _, p in named]
        n = sum(p.numel() for p in self.params)
        self.split = 0
        for name, p in named:
            if name.startswith(("encoder.layer4.", "classification_head.")):
                break
            self.split += p.numel()
        self.flat = torch.empty(n, device=self.dev, dtype=torch.float32)
        # gradient + the step's loss (+ AMP's found_inf): all-reduced together
        self._gbuf = torch.zeros(n + (2 if self.amp else 1), device=self.dev,
                                 dtype=torch.float32)
        self.grad = self._gbuf[:n]
        self.loss_gate = self._gbuf[n:n + 1]
        self.found_inf = self._gbuf[n + 1:n + 2] if self.amp else None
        self.scale = torch.full((1,), float(init_scale), device=self.dev, dtype=torch.float32)
        self.growth_tracker = torch.zeros(1, device=self.dev, dtype=torch.int32)
        # the first group's scaler.update() writes a shadow (one update per step)
        self._scale_shadow = self.scale.clone()
        self._tracker_shadow = self.growth_tracker.clone()
        self.mom = torch.zeros(n, device=self.dev, dtype=torch.float32)
        # device counters per group: [applied steps, skipped steps]
        self.step_counts = torch.zeros(2, device=self.dev, dtype=torch.int32)
        self._counts_g1 = torch.zeros(2, device=self.dev, dtype=torch.int32)
        self.views: Dict[int, torch.Tensor] = {}
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view(p.shape)
            self.views[id(p)] = self.grad[off:off + k].view(p.shape)
            off += k
        self.bns = [m for m in model.modules() if isinstance(m, nn.BatchNorm2d)]
        self.zero_bias: Dict[int, torch.Tensor] = {}
        self.steps = 0
        self._ws: Dict[str, torch.Tensor] = {}
        self.wgrad_side = os.environ.get("TCAM_WGRAD_SIDE", "1") != "0"
        # the fused BN-ReLU backward with a bound-based MFMA scale (TCAM_FUSED_BN_BWD=0: the
        # three-pass path: backward + channel maxima, scale, re-split)
        self.fused_bn_bwd = os.environ.get("TCAM_FUSED_BN_BWD", "1") != "0"
        # the stem's weight gradient as im2col + the 1x1 MFMA GEMM (0: the fp32-MFMA general path)
        self.stem_im2col = os.environ.get("TCAM_STEM_IM2COL", "1") != "0"
        # the repack as one batched launch (two on f16x3) once the operand buffers exist
        self.batched_pack = os.environ.get("TCAM_BATCHED_PACK", "1") != "0"
        self._pack_items = None
        self._pack_table = None
        self._wg_stream = None
        self._stem_dw = None
        self.repack()

    # ------------------------------------------------------------ helpers
    @property
    def lr(self) -> float:
        return self.lrs[0]

    def trainable_names(self) -> List[str]:
        """The flat buffer's parameter names, in order (checkpoints)."""
        return [n for n, _ in self.model.named_parameters()]

    def loss_t(self) -> list:
        """MasterLoss([ClLoss]).get_t() (losses/master.py:37-41; no ELB: t = 0)."""
        return [["cl_loss", 0.0]]

    def close(self) -> None:
        """(the trainer keeps nothing for the next step)"""

    def g(self, p: torch.Tensor) -> torch.Tensor:
        return self.views[id(p)]

    def _zeros(self, n: int) -> torch.Tensor:
        z = self.zero_bias.get(n)
        if z is None:
            z = torch.zeros(n, device=self.dev, dtype=torch.float32)
            self.zero_bias[n] = z
        return z

    def _workspace(self, key: str, nbytes: int) -> torch.Tensor:
        cur = self._ws.get(key)
        if cur is None or cur.numel() < nbytes:
            if cur is not None and self._wg_stream is not None:
                cur.record_stream(self._wg_stream)
            cur = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.dev)
            self._ws[key] = cur
        return cur

    def _convs(self):
        yield self.stem
        for layer in self.layers:
            for b in layer:
                yield b.c1
                yield b.c2
                yield b.c3
                if b.ds is not None:
                    yield b.ds

    def views_intact(self) -> bool:
        off, base = 0, self.flat.data_ptr()
        for p in self.params:
            if p.data_ptr() != base + 4 * off:
                return False
            off += p.numel()
        return True

    def param_version(self) -> int:
        return sum(p._version for p in self.params)

    @property
    def bn_flat(self) -> torch.Tensor:
        return torch.cat([t.reshape(-1) for bn in self.bns
                          for t in (bn.running_mean, bn.running_var)])

    def set_bn_flat(self, flat: torch.Tensor) -> None:
        off = 0
        for bn in self.bns:
            for t in (bn.running_mean, bn.running_var):
                k = t.numel()
                t.copy_(flat[off:off + k].view_as(t))
                off += k

    def _pack(self, w: torch.Tensor, mode: int, sel: int = 0, cin_pad: int = 0,
              kdiv: Optional[torch.Tensor] = None, out=None):
        """The MFMA operand of conv weight ``w`` (Cout, Cin, KH, KW): mode 0 the forward's,
        mode 1 the data gradient's (transposed, rotated, over the first ``sel`` input
        channels, divided by ``kdiv`` = dy's per-channel scales on the f16x3 path).
        Returns (wt, wscale or None)."""
        cout, ctot, kh, kw = w.shape
        if mode == 0:
            K, M = kh * kw * max(ctot, cin_pad), cout
        else:
            K, M = kh * kw * cout, sel
        kp, mp = ops.conv_x6_weight_dims(K, M)
        lib = _lib.load()
        if self.amp:
            wt = out[0] if out is not None and out[0] is not None and \
                tuple(out[0].shape) == (kp // 32, 4, 1, mp, 8) else \
                torch.empty((kp // 32, 4, 1, mp, 8), device=self.dev, dtype=torch.float16)
            check(lib.tcam_pack_weight_f16(w.data_ptr(), wt.data_ptr(), mode, cout, ctot, kh, kw,
                                           0, sel if mode else 0, cin_pad, _stream()),
                  "tcam_pack_weight_f16")
            return wt, None
        if out is not None and out[0] is not None and \
                tuple(out[0].shape) == (kp // 32, 4, 2, mp, 8):
            wt, sc = out
        else:
            wt = torch.empty((kp // 32, 4, 2, mp, 8), device=self.dev, dtype=torch.float16)
            sc = torch.empty(mp, device=self.dev, dtype=torch.float32)
        check(lib.tcam_pack_weight_f16x3(w.data_ptr(), wt.data_ptr(), sc.data_ptr(), mode, cout,
                                         ctot, kh, kw, 0, sel if mode else 0, cin_pad,
                                         _p(kdiv), _stream()), "tcam_pack_weight_f16x3")
        return wt, sc

    def repack(self):
        """The forward operands of every conv from the flat fp32 weights: once the operand
        buffers exist, one batched launch for all of them (two on f16x3: the column scales,
        then the parts; ``tcam_pack_weights``) instead of one or two per conv
        (TCAM_BATCHED_PACK=0: per conv)."""
        self._packed_version = self.param_version()
        convs = list(self._convs())
        # AMP: the data-gradient operands that need no dy scale go into the same batch (every
        # c3 / c2, and c1 of the identity blocks; a projection block's c1 is packed in the
        # backward, K-concatenated with its shortcut)
        dconvs = [c for layer in self.layers for b in layer
                  for c in (b.c3, b.c2) + ((b.c1,) if b.ds is None else ())] \
            if self.amp and self.batched_pack else []
        if not self.batched_pack or any(c.wt is None for c in convs) or \
                any(c.dwt is None for c in dconvs):
            for c in convs:
                c.wt, c.wsc = self._pack(c.conv.weight.data, 0, cin_pad=c.cin_pad,
                                         out=(c.wt, c.wsc))
            for c in dconvs:
                c.dwt, _ = self._pack(c.conv.weight.data, 1, sel=c.cin, out=(c.dwt, None))
            return
        n = len(convs) + len(dconvs)
        if self._pack_items is None or len(self._pack_items) != n:
            self._pack_items = (tcam_pack_item * n)()
            lib = _lib.load()
            self._pack_table = torch.empty(int(lib.tcam_pack_table_bytes(n)), device=self.dev,
                                           dtype=torch.uint8)
        for it, (c, mode) in zip(self._pack_items, [(c, 0) for c in convs] +
                                 [(c, 1) for c in dconvs]):
            w = c.conv.weight.data
            cout, ctot, kh, kw = w.shape
            it.w, it.out = w.data_ptr(), (c.wt if mode == 0 else c.dwt).data_ptr()
            it.wscale = None if self.amp else c.wsc.data_ptr()
            it.kdiv = None
            it.mode, it.CoutW, it.CtotW, it.KH, it.KW = mode, cout, ctot, kh, kw
            it.c0, it.cout_sel = 0, (c.cin if mode else 0)
            it.cin_pad = c.cin_pad if mode == 0 else 0
        check(_lib.load().tcam_pack_weights(self._pack_items, n, 0 if self.amp else 1,
                                            self._pack_table.data_ptr(), _stream()),
              "tcam_pack_weights")

    # --------------------------------------------------------------- ops
    def _conv(self, srcs, c: _EConv, H: int, W: int) -> torch.Tensor:
        return ops.conv2d_x6(srcs, c.wt, self._zeros(c.cout), c.cout, H, W, c.k, c.pad, False,
                             wscale=c.wsc)

    def _bn_stats(self, c: _EConv, y: torch.Tensor):
        lib = _lib.load()
        B, H, W, Cc = ops.s3_dims(y)
        P = B * H * W
        ws = self._workspace("bn", int(lib.tcam_bn_ws_bytes(P, Cc)))
        mean = torch.empty(Cc, device=self.dev)
        invstd = torch.empty(Cc, device=self.dev)
        bn = c.bn
        check(getattr(lib, f"tcam_bn_stats_{self.lay}")(
            y.data_ptr(), P, Cc, bn.eps, bn.momentum, mean.data_ptr(), invstd.data_ptr(),
            bn.running_mean.data_ptr(), bn.running_var.data_ptr(), ws.data_ptr(), _stream()),
            f"tcam_bn_stats_{self.lay}")
        return mean, invstd

    def _bn_relu(self, c: _EConv, y: torch.Tensor):
        lib = _lib.load()
        mean, invstd = self._bn_stats(c, y)
        B, H, W, Cc = ops.s3_dims(y)
        out = torch.empty_like(y)
        check(getattr(lib, f"tcam_bn_relu_{self.lay}")(
            y.data_ptr(), mean.data_ptr(), invstd.data_ptr(), c.bn.weight.data_ptr(),
            c.bn.bias.data_ptr(), out.data_ptr(), B * H * W, Cc, _stream()),
            f"tcam_bn_relu_{self.lay}")
        return out, mean, invstd

    def _bn_bwd(self, c: _EConv, dout, out, y, mean, invstd, scaled: bool = True,
                masky: bool = False, need_s3: bool = False):
        """dy of a BatchNorm whose output went through the ReLU that produced ``out``
        (the mask): the f16x3 step returns (dy S3 or None, dy2, scale) — dy2 its
        per-channel scaled S2 copy for the MFMA, from the fused backward (``masky``: a
        BN-ReLU, the mask recomputed from y; ``need_s3``: dy itself too) — or (dy, None,
        None) with ``scaled`` False; AMP returns (dy S1, None, None)."""
        lib = _lib.load()
        B, H, W, Cc = ops.s3_dims(y)
        P = B * H * W
        gw, gb = self.g(c.bn.weight), self.g(c.bn.bias)
        if scaled and not self.amp and self.fused_bn_bwd:
            ws = self._workspace("bn", int(lib.tcam_bn_bwd_scaled_ws_bytes(P, Cc)))
            dy = ops.lay_empty("s3", B, H, W, Cc, self.dev) if need_s3 else None
            dy2 = ops.lay_empty("s2", B, H, W, Cc, self.dev)
            scale = torch.empty(Cc, device=self.dev, dtype=torch.float32)
            check(lib.tcam_bn_relu_bwd_scaled_s3s2(
                dout.data_ptr(), None if masky else out.data_ptr(), y.data_ptr(),
                mean.data_ptr(), invstd.data_ptr(), c.bn.weight.data_ptr(),
                c.bn.bias.data_ptr(), _p(dy), dy2.data_ptr(), scale.data_ptr(), gw.data_ptr(),
                gb.data_ptr(), P, Cc, ws.data_ptr(), _stream()), "tcam_bn_relu_bwd_scaled_s3s2")
            return dy, dy2, scale
        ws = self._workspace("bn", int(lib.tcam_bn_ws_bytes(P, Cc)))
        dy = ops.lay_empty(self.glay, B, H, W, Cc, self.dev)
        if self.amp and self.fused_bn_bwd:
            check(lib.tcam_bn_relu_bwd_fused_s1(
                dout.data_ptr(), None if masky else out.data_ptr(), y.data_ptr(),
                mean.data_ptr(), invstd.data_ptr(), c.bn.weight.data_ptr(),
                c.bn.bias.data_ptr(), dy.data_ptr(), gw.data_ptr(), gb.data_ptr(), P, Cc,
                ws.data_ptr(), _stream()), "tcam_bn_relu_bwd_fused_s1")
            return dy, None, None
        if self.amp:
            check(lib.tcam_bn_relu_bwd_s1(dout.data_ptr(), out.data_ptr(), y.data_ptr(),
                                          mean.data_ptr(), invstd.data_ptr(),
                                          c.bn.weight.data_ptr(), dy.data_ptr(), gw.data_ptr(),
                                          gb.data_ptr(), P, Cc, ws.data_ptr(), _stream()),
                  "tcam_bn_relu_bwd_s1")
            return dy, None, None
        amax = torch.empty(Cc, device=self.dev, dtype=torch.int32) if scaled else None
        check(lib.tcam_bn_relu_bwd_s3s2(dout.data_ptr(), out.data_ptr(), y.data_ptr(),
                                        mean.data_ptr(), invstd.data_ptr(),
                                        c.bn.weight.data_ptr(), dy.data_ptr(), gw.data_ptr(),
                                        gb.data_ptr(), P, Cc, ws.data_ptr(), _p(amax), _stream()),
              "tcam_bn_relu_bwd_s3s2")
        if not scaled:
            return dy, None, None
        scale = torch.empty(Cc, device=self.dev, dtype=torch.float32)
        dy2 = ops.lay_empty("s2", B, H, W, Cc, self.dev)
        check(lib.tcam_dy_scaled_s2(dy.data_ptr(), P, Cc, amax.data_ptr(), 0, scale.data_ptr(),
                                    dy2.data_ptr(), _stream()), "tcam_dy_scaled_s2")
        return dy, dy2, scale

    def _dgrad(self, srcs, w: torch.Tensor, kdiv: Optional[torch.Tensor], sel: int, H: int,
               W: int, k: int, pad: int, c: Optional[_EConv] = None) -> torch.Tensor:
        """Data gradient: the stride-1 conv of dy (``srcs``: its MFMA copies) with the
        transposed, rotated weight ``w`` -> the gradient of the first ``sel`` input channels
        at H x W (S3 on the f16x3 path, S1 on AMP).  ``c``: the conv whose operand the AMP
        repack already packed (``c.dwt``), if it did."""
        if self.amp and c is not None and c.dwt is not None and self.batched_pack:
            return ops.conv2d_x6(srcs, c.dwt, self._zeros(sel), sel, H, W, k, k - 1 - pad, False)
        wt, sc = self._pack(w, 1, sel=sel, kdiv=kdiv)
        if self.amp:
            return ops.conv2d_x6(srcs, wt, self._zeros(sel), sel, H, W, k, k - 1 - pad, False)
        return ops.conv2d_f16x3_s3out(srcs, wt, sc, self._zeros(sel), sel, H, W, k, k - 1 - pad)

    def _zero_up2(self, t: torch.Tensor, H: int, W: int) -> torch.Tensor:
        B, Hi, Wi, Cc = ops.s3_dims(t)
        out = ops.act_empty(t, B, H, W, Cc)
        gb = {"s1": 16, "s2": 32, "s3": 48}[ops._lay(t)]
        check(_lib.load().tcam_zero_up2(t.data_ptr(), out.data_ptr(), gb, B, Cc, H, W, Hi, Wi,
                                        _stream()), "tcam_zero_up2")
        return out

    # -------------------------------------------------------- weight gradients
    def _side(self, fn, *tensors):
        """Runs ``fn`` (a weight-gradient launch) on the side stream after everything queued
        so far on the current stream (TCAM_WGRAD_SIDE=0: inline)."""
        if not self.wgrad_side:
            fn()
            return
        if self._wg_stream is None:
            self._wg_stream = torch.cuda.Stream(device=self.dev)
        side = self._wg_stream
        side.wait_stream(torch.cuda.current_stream(self.dev))
        for t in tensors:
            if t is not None:
                t.record_stream(side)
        with torch.cuda.stream(side):
            fn()

    def _wgrad11(self, x: torch.Tensor, stride: int, dy: torch.Tensor,
                 dsc: Optional[torch.Tensor], dw: torch.Tensor) -> None:
        lib = _lib.load()
        B, Hin, Win, Cin = ops.s3_dims(x)
        _, Ho, Wo, Cout = ops.s3_dims(dy)
        nb = int(lib.tcam_wgrad11_ws_bytes(B, Cin, Hin, Win, stride, Cout, Ho, Wo))
        if nb == 0:
            raise ValueError("tcam_wgrad11: unsupported geometry")
        ws = self._workspace("wg", nb)
        if self.amp:
            check(lib.tcam_wgrad11_s1(x.data_ptr(), B, Cin, Hin, Win, stride, dy.data_ptr(), Cout,
                                      Ho, Wo, dw.data_ptr(), ws.data_ptr(), ws.numel(),
                                      _stream()), "tcam_wgrad11_s1")
        else:
            check(lib.tcam_wgrad11_s2_f16x3(x.data_ptr(), B, Cin, Hin, Win, stride, dy.data_ptr(),
                                            dsc.data_ptr(), Cout, Ho, Wo, dw.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _stream()),
                  "tcam_wgrad11_s2_f16x3")

    def _srcs(self, x: torch.Tensor, stride: int):
        _, H, W, Cc = ops.s3_dims(x)
        arr = (tcam_conv_src * 1)()
        arr[0] = tcam_conv_src(x.data_ptr(), Cc, H, W, stride, 0)
        return arr

    def _wgrad_conv(self, x: torch.Tensor, c: _EConv, dy: torch.Tensor,
                    dy2: Optional[torch.Tensor], dsc: Optional[torch.Tensor],
                    dw: torch.Tensor, cout_store: Optional[int] = None,
                    stride: Optional[int] = None) -> None:
        """KxK weight gradient of conv ``c`` on input ``x``: the 3x3 / stride-1 fast path
        (f16x3 on dy2 / dsc, or AMP's fp16 product) or the fp32-MFMA general path (dy).
        ``stride`` overrides the conv's (1 with dy zero-inserted onto the input grid)."""
        lib = _lib.load()
        B, Ho, Wo, Cd = ops.s3_dims(dy if dy is not None else dy2)
        stride = c.stride if stride is None else stride
        arr = self._srcs(x, stride)
        fast = c.k == 3 and stride == 1 and c.pad == 1
        if self.amp:
            nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, 1, B, Cd, Ho, Wo, c.k, c.k))
            ws = self._workspace("wg", nb)
            check(lib.tcam_conv_wgrad_s1(arr, 1, B, dy.data_ptr(), Cd, Ho, Wo, c.k, c.k, c.pad,
                                         c.pad, cout_store or Cd, dw.data_ptr(), ws.data_ptr(),
                                         ws.numel(), _stream()), "tcam_conv_wgrad_s1")
        elif fast:
            nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, 1, B, Cd, Ho, Wo, 3, 3))
            ws = self._workspace("wg", nb)
            check(lib.tcam_conv_wgrad_s2_f16x3(arr, 1, B, dy2.data_ptr(), dsc.data_ptr(), Cd, Ho,
                                               Wo, 3, 3, 1, 1, cout_store or Cd, dw.data_ptr(),
                                               ws.data_ptr(), ws.numel(), _stream()),
                  "tcam_conv_wgrad_s2_f16x3")
        else:
            nb = int(lib.tcam_conv_wgrad_generic_ws_bytes(arr, 1, B, Cd, Ho, Wo, c.k, c.k))
            ws = self._workspace("wg", nb)
            check(lib.tcam_conv_wgrad_s3s2(arr, 1, B, dy.data_ptr(), Cd, Ho, Wo, c.k, c.k, c.pad,
                                           c.pad, cout_store or Cd, dw.data_ptr(), ws.data_ptr(),
                                           ws.numel(), _stream()), "tcam_conv_wgrad_s3s2")

    # ------------------------------------------------------------ forward
    def forward(self, images: torch.Tensor):
        """Train-mode forward: (cl_logits (B, K) fp32, state for :meth:`backward`)."""
        lib = _lib.load()
        if images.dim() != 4 or images.shape[1] != 3 or not images.is_cuda:
            raise ValueError("expected a (B, 3, H, W) cuda tensor")
        if self.param_version() != self._packed_version:
            self.repack()
        x = images.contiguous().float()
        B, _, H, W = x.shape
        x0 = ops.s3_from_nchw(x, 8, self.fmt)
        s = self.stem
        H1, W1 = (H + 2 * s.pad - s.k) // s.stride + 1, (W + 2 * s.pad - s.k) // s.stride + 1
        y0 = self._conv([ConvSrc(x0, s.stride)], s, H1, W1)
        a0, m0, i0 = self._bn_relu(s, y0)
        f = ops.maxpool3x3s2_s3(a0)
        st = {"x0": x0, "stem": (y0, a0, m0, i0), "pool_in": a0, "pool_out": f, "blocks": []}
        for layer in self.layers:
            for b in layer:
                Bq, Hi, Wi, _ = ops.s3_dims(f)
                y1 = self._conv([ConvSrc(f)], b.c1, Hi, Wi)
                a1, m1, i1 = self._bn_relu(b.c1, y1)
                sd = b.c2.stride
                Ho, Wo = (Hi + 2 - 3) // sd + 1, (Wi + 2 - 3) // sd + 1
                y2 = self._conv([ConvSrc(a1, sd)], b.c2, Ho, Wo)
                a2, m2, i2 = self._bn_relu(b.c2, y2)
                y3 = self._conv([ConvSrc(a2)], b.c3, Ho, Wo)
                m3, i3 = self._bn_stats(b.c3, y3)
                yd = md = idd = None
                if b.ds is not None:
                    yd = self._conv([ConvSrc(f, b.ds.stride)], b.ds, Ho, Wo)
                    md, idd = self._bn_stats(b.ds, yd)
                out = ops.act_empty(y3, Bq, Ho, Wo, b.c3.cout)
                bd = b.ds.bn if b.ds is not None else None
                check(getattr(lib, f"tcam_bn_add_relu_{self.lay}")(
                    y3.data_ptr(), m3.data_ptr(), i3.data_ptr(), b.c3.bn.weight.data_ptr(),
                    b.c3.bn.bias.data_ptr(), _p(yd), _p(md), _p(idd),
                    _p(bd.weight if bd is not None else None),
                    _p(bd.bias if bd is not None else None),
                    None if yd is not None else f.data_ptr(), out.data_ptr(), Bq * Ho * Wo,
                    b.c3.cout, _stream()), f"tcam_bn_add_relu_{self.lay}")
                st["blocks"].append(dict(x=f, y1=y1, a1=a1, m1=m1, i1=i1, y2=y2, a2=a2, m2=m2,
                                         i2=i2, y3=y3, m3=m3, i3=i3, yd=yd, md=md, idd=idd,
                                         out=out))
                f = out
        Bq, Hf, Wf, Cf = ops.s3_dims(f)
        K = self.fc.out_features
        pooled = torch.empty((Bq, Cf), device=self.dev, dtype=torch.float32)
        logits = torch.empty((Bq, K), device=self.dev, dtype=torch.float32)
        ws = self._workspace("pool", int(lib.tcam_cls_pool_ws_bytes(Bq, Cf)))
        check(getattr(lib, f"tcam_cls_fwd_{self.lay}")(
            f.data_ptr(), Bq, Hf * Wf, Cf, self.fc.weight.data_ptr(), self.fc.bias.data_ptr(), K,
            pooled.data_ptr(), logits.data_ptr(), ws.data_ptr(), _stream()),
            f"tcam_cls_fwd_{self.lay}")
        st["pooled"] = pooled
        st["feat"] = f
        self.model.x_in = images
        return logits, st

    # ----------------------------------------------------------- backward
    def backward(self, dlogits: torch.Tensor, st) -> None:
        """Gradients of every parameter into the flat buffer from d loss / d logits."""
        try:
            self._backward_impl(dlogits.contiguous().float(), st)
        finally:
            if self._wg_stream is not None:
                torch.cuda.current_stream(self.dev).wait_stream(self._wg_stream)

    def _backward_impl(self, dlogits: torch.Tensor, st) -> None:
        lib = _lib.load()
        f = st["feat"]
        B, Hf, Wf, Cf = ops.s3_dims(f)
        K = self.fc.out_features
        dpooled = torch.empty((B, Cf), device=self.dev, dtype=torch.float32)
        check(lib.tcam_cls_bwd(dlogits.data_ptr(), st["pooled"].data_ptr(),
                               self.fc.weight.data_ptr(), B, K, Cf, 1 if self.amp else 0,
                               self.g(self.fc.weight).data_ptr(), self.g(self.fc.bias).data_ptr(),
                               dpooled.data_ptr(), _stream()), "tcam_cls_bwd")
        dout = ops.lay_empty(self.glay, B, Hf, Wf, Cf, self.dev)
        check(getattr(lib, f"tcam_pool_bwd_{self.glay}")(dpooled.data_ptr(), B, Hf * Wf, Cf,
                                                         dout.data_ptr(), _stream()),
              f"tcam_pool_bwd_{self.glay}")
        blocks = [b for layer in self.layers for b in layer]
        for bi in range(len(blocks) - 1, -1, -1):
            b, s = blocks[bi], st["blocks"][bi]
            dout = self._block_backward(b, s, dout)
        # max-pool adjoint, stem BN-ReLU, stem weight gradient (the image needs none)
        a0 = st["pool_in"]
        _, Hp, Wp, Cp = ops.s3_dims(a0)
        _, Ho, Wo, _ = ops.s3_dims(st["pool_out"])
        ws = self._workspace("pool", int(lib.tcam_maxpool_bwd_ws_bytes(B, Cp, Ho, Wo)))
        da0 = ops.lay_empty(self.glay, B, Hp, Wp, Cp, self.dev)
        name = "tcam_maxpool3x3s2_bwd_s1" if self.amp else "tcam_maxpool3x3s2_bwd_s3s2"
        check(getattr(lib, name)(dout.data_ptr(), a0.data_ptr(), da0.data_ptr(), ws.data_ptr(),
                                 B, Cp, Hp, Wp, Ho, Wo, _stream()), name)
        y0, _, m0, i0 = st["stem"]
        s0, gw, x0 = self.stem, self.g(self.stem.conv.weight), st["x0"]
        if not self.stem_im2col:
            # the fp32-MFMA general path on the exact S3 dy (TCAM_STEM_IM2COL=0)
            dy0, _, _ = self._bn_bwd(s0, da0, a0, y0, m0, i0, scaled=False)
            if self._stem_dw is None:
                self._stem_dw = torch.empty((s0.cout, 8, s0.k, s0.k), device=self.dev,
                                            dtype=torch.float32)
            tmp = self._stem_dw

            def stem_wgrad():
                self._wgrad_conv(x0, s0, dy0, None, None, tmp)
                gw.copy_(tmp[:, :s0.cin])
            self._side(stem_wgrad, x0, dy0, tmp)
            return
        # the 7x7/2 stem's weight gradient as a 1x1 one: every output pixel's 7x7 patch of the
        # 8-channel (3 real) image as 49 groups (tcam_im2col), then wgrad11's GEMM over pixels
        # (dW (64, 49 x 8) on the fp16 MFMA, f16x3 or AMP) — the general fp32-MFMA path took
        # ~2.2 ms at the end of the backward, with nothing left to overlap it
        dy0, dy0s, sc0 = self._bn_bwd(s0, da0, a0, y0, m0, i0, masky=True)
        op0 = dy0 if self.amp else dy0s
        _, Hx, Wx, Cx = ops.s3_dims(x0)
        _, Ho0, Wo0, Co = ops.s3_dims(op0)
        taps = s0.k * s0.k
        if self._stem_dw is None or self._stem_dw.shape != (Co, taps * Cx):
            self._stem_dw = torch.empty((Co, taps * Cx), device=self.dev, dtype=torch.float32)
        tmp = self._stem_dw
        lay = ops._lay(x0)

        def stem_wgrad():
            col = ops.lay_empty(lay, B, Ho0, Wo0, taps * Cx, self.dev)
            check(lib.tcam_im2col(x0.data_ptr(), col.data_ptr(), {"s1": 16, "s2": 32}[lay], B,
                                  Cx, Hx, Wx, s0.k, s0.k, s0.stride, s0.pad, Ho0, Wo0,
                                  _stream()), "tcam_im2col")
            self._wgrad11(col, 1, op0, sc0, tmp)
            # (co, tap, c) -> PyTorch's (co, c, kh, kw), the real input channels
            gw.copy_(tmp.view(Co, taps, Cx)[:, :, :s0.cin].permute(0, 2, 1)
                     .reshape(Co, s0.cin, s0.k, s0.k))
        self._side(stem_wgrad, x0, op0, sc0, tmp)

    def _block_backward(self, b: _Block, s, dout: torch.Tensor) -> torch.Tensor:
        """One Bottleneck's backward: its weight / BN gradients, returns d loss / d x."""
        out, x = s["out"], s["x"]
        B, Hin, Win, Cin = ops.s3_dims(x)
        _, Ho, Wo, _ = ops.s3_dims(out)
        # bn3 (+ the projection's BN): the mask is the block output's relu3
        dy3, dy3s, sc3 = self._bn_bwd(b.c3, dout, out, s["y3"], s["m3"], s["i3"])
        a2, a1 = s["a2"], s["a1"]
        g3 = self.g(b.c3.conv.weight).view(b.c3.cout, b.c3.cin)
        op3 = dy3 if self.amp else dy3s
        self._side(lambda: self._wgrad11(a2, 1, op3, sc3, g3), a2, op3, sc3)
        if b.ds is not None:
            dyd, dyds, scd = self._bn_bwd(b.ds, dout, out, s["yd"], s["md"], s["idd"])
            gd = self.g(b.ds.conv.weight).view(b.ds.cout, b.ds.cin)
            opd = dyd if self.amp else dyds
            sdd = b.ds.stride
            self._side(lambda: self._wgrad11(x, sdd, opd, scd, gd), x, opd, scd)
        # conv3 data gradient -> bn2
        da2 = self._dgrad([ConvSrc(op3)], b.c3.conv.weight.data, sc3, b.c3.cin, Ho, Wo, 1, 0,
                          c=b.c3)
        dy2, dy2s, sc2 = self._bn_bwd(b.c2, da2, a2, s["y2"], s["m2"], s["i2"], masky=True)
        g2 = self.g(b.c2.conv.weight)
        op2 = dy2 if self.amp else dy2s
        # stride 2: dy spread onto the input grid (dy_up[2o] = dy[o], zeros between) turns both
        # gradients of the conv into stride-1 3x3 ones — dW[k] = sum_q dy_up[q] x[q - 1 + k],
        # the fast MFMA weight gradient instead of the fp32-MFMA general path
        src2 = op2 if b.c2.stride == 1 else self._zero_up2(op2, Hin, Win)
        if b.c2.stride == 1:
            self._side(lambda: self._wgrad_conv(a1, b.c2, dy2, dy2s, sc2, g2), a1, dy2, dy2s, sc2)
        else:
            wdy, wdy2 = (src2, None) if self.amp else (None, src2)
            self._side(lambda: self._wgrad_conv(a1, b.c2, wdy, wdy2, sc2, g2, stride=1),
                       a1, src2, sc2)
        # conv2 data gradient -> bn1
        da1 = self._dgrad([ConvSrc(src2)], b.c2.conv.weight.data, sc2, b.c2.cin, Hin, Win, 3, 1,
                          c=b.c2)
        dy1, dy1s, sc1 = self._bn_bwd(b.c1, da1, a1, s["y1"], s["m1"], s["i1"], masky=True)
        g1 = self.g(b.c1.conv.weight).view(b.c1.cout, b.c1.cin)
        op1 = dy1 if self.amp else dy1s
        self._side(lambda: self._wgrad11(x, 1, op1, sc1, g1), x, op1, sc1)
        # d x: conv1's data gradient + the shortcut's
        if b.ds is None:
            dxc = self._dgrad([ConvSrc(op1)], b.c1.conv.weight.data, sc1, Cin, Hin, Win, 1, 0,
                              c=b.c1)
            dx = ops.lay_empty(self.glay, B, Hin, Win, Cin, self.dev)
            name = "tcam_grad_add_mask_s1" if self.amp else "tcam_grad_add_mask_s3s2"
            check(getattr(_lib.load(), name)(dxc.data_ptr(), dout.data_ptr(), out.data_ptr(),
                                             dx.data_ptr(), B * Hin * Win, Cin, _stream()), name)
            return dx
        # projection shortcut: one K-concatenated conv over [dy1 | dyd] (dyd zero-inserted
        # onto the input grid when the projection has stride 2)
        srcd = opd if b.ds.stride == 1 else self._zero_up2(opd, Hin, Win)
        wcat = torch.cat([b.c1.conv.weight.data, b.ds.conv.weight.data], dim=0)
        kdiv = None if self.amp else torch.cat([sc1, scd])
        return self._dgrad([ConvSrc(op1), ConvSrc(srcd)], wcat, kdiv, Cin, Hin, Win, 1, 0)

    # ------------------------------------------------------------- the step
    def loss_and_grad(self, logits: torch.Tensor, labels: torch.Tensor):
        """ClLoss on the device: (loss (1,), d loss / d logits (times the AMP scale))."""
        lab = labels.to(device=self.dev, dtype=torch.int32).contiguous()
        B, K = logits.shape
        loss = torch.empty(1, device=self.dev, dtype=torch.float32)
        dl = torch.empty_like(logits)
        check(_lib.load().tcam_ce_loss(logits.data_ptr(), lab.data_ptr(), B, K, self.cl_lambda,
                                       _p(self.scale) if self.amp else None, loss.data_ptr(),
                                       dl.data_ptr(), _stream()), "tcam_ce_loss")
        return loss, dl

    def step(self, images: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """One optimisation step on a batch; returns the device loss (1,)."""
        logits, st = self.forward(images)
        loss, dl = self.loss_and_grad(logits, labels)
        self.loss_gate.copy_(loss)
        self.backward(dl, st)
        if self.amp:   # scaler.unscale_: 1/scale, non-finite check (device)
            self.found_inf.zero_()
            check(_lib.load().tcam_amp_unscale(self.grad.data_ptr(), self.grad.numel(),
                                               self.scale.data_ptr(),
                                               self.found_inf.data_ptr(), _stream()),
                  "tcam_amp_unscale")
        else:
            # an f16x3 operand beyond the fp16 range made this step invalid: skip it on the
            # device on every rank (check_overflow() reports it)
            self.loss_gate.masked_fill_(ops.f16_overflow_flag(self.dev).bool(), float("nan"))
        self.all_reduce_and_step()
        self.steps += 1
        self.last_logits = logits
        return loss

    def all_reduce_and_step(self) -> None:
        """DDP average (RCCL all-reduce of the flat gradient + loss slot), rank 0's BN
        statistics broadcast, the gated SGD step of both parameter groups, repack."""
        scale = 1.0
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(self._gbuf, op=dist.ReduceOp.SUM)
            bn = self.bn_flat
            dist.broadcast(bn, src=0)
            self.set_bn_flat(bn)
            scale = 1.0 / dist.get_world_size()
        lib = _lib.load()
        n = self.flat.numel()
        groups = ((0, self.split, self.lrs[0], self._counts_g1),
                  (self.split, n, self.lrs[1], self.step_counts))
        for gi, (a, e, lr, cnt) in enumerate(groups):
            if e <= a:
                continue
            p, g, m = self.flat[a:e], self.grad[a:e], self.mom[a:e]
            if self.amp:
                gcfg = self.scaler_cfg
                sc, tr = (self.scale, self.growth_tracker) if gi == 1 else \
                    (self._scale_shadow, self._tracker_shadow)
                check(lib.tcam_sgd_step_amp(p.data_ptr(), g.data_ptr(), m.data_ptr(), e - a, lr,
                                            self.momentum, self.dampening, self.weight_decay,
                                            1 if self.nesterov else 0, scale,
                                            self._gbuf[-2:].data_ptr(), cnt.data_ptr(),
                                            cnt.data_ptr() + 4, sc.data_ptr(), tr.data_ptr(),
                                            gcfg[0], gcfg[1], gcfg[2], _stream()),
                      "tcam_sgd_step_amp")
            else:
                check(lib.tcam_sgd_step_gated(p.data_ptr(), g.data_ptr(), m.data_ptr(), e - a, lr,
                                              self.momentum, self.dampening, self.weight_decay,
                                              1 if self.nesterov else 0, scale,
                                              self.loss_gate.data_ptr(), cnt.data_ptr(),
                                              cnt.data_ptr() + 4, _stream()),
                      "tcam_sgd_step_gated")
        # one multi-tensor launch for every BN's counter
        torch._foreach_add_([bn.num_batches_tracked for bn in self.bns], 1)
        self.repack()
        self.model.invalidate_plans(ENCODER_PLANS)

    def check_overflow(self) -> None:
        """Raise (a host sync; a collective under torch.distributed) when an f16x3 operand
        left the fp16 range since the last check: those steps were skipped on the device."""
        if self.amp:
            return
        try:
            ops.check_f16_overflow(self.dev, all_ranks=True)
        except FloatingPointError:
            raise FloatingPointError(
                "an f16x3 operand exceeded the fp16 range |x| <= 65504 during stage-1 "
                "training: the affected steps were skipped; train with amp=True") from None

    @property
    def applied_steps(self) -> int:
        return int(self.step_counts[0].item())

    @property
    def skipped_steps(self) -> int:
        return int(self.step_counts[1].item())


class _TrainForwardCl(torch.autograd.Function):
    """STDClassifier.forward in train mode as one autograd node: forward =
    ClassifierTrainer.forward, backward = ClassifierTrainer.backward from d loss / d logits;
    the gradients reach every Parameter through autograd, so the reference's loop
    (``loss = ClLoss(model(x), y); loss.backward(); optimizer.step()``,
    train_wsol.py:1162-1184) and DDP's hooks work unchanged."""

    @staticmethod
    def forward(ctx, engine, images, *params):
        logits, st = engine.forward(images)
        ctx.engine, ctx.st = engine, st
        return logits

    @staticmethod
    def backward(ctx, g_logits):
        eng, st = ctx.engine, ctx.st
        ctx.st = None
        if st is None:
            raise RuntimeError("STDClassifier train-mode forward: backward called twice")
        eng.grad.zero_()
        eng.backward(g_logits.contiguous().float(), st)
        return (None, None) + tuple(eng.g(p).clone() for p in eng.params)


def train_forward(model: STDClassifier, images: torch.Tensor) -> torch.Tensor:
    """cl_logits of a ResNet50 STDClassifier in train mode (batch-statistics BatchNorm,
    running statistics updated), differentiable w.r.t. every parameter when grad mode is
    on.  Used by STDClassifier.forward when ``model.training``."""
    eng = model.__dict__.get("_train_engine")
    amp = getattr(model, "conv_precision", None) == "amp"
    if eng is None or not eng.views_intact() or eng.amp != amp:
        eng = ClassifierTrainer(model, amp=amp)
        model.__dict__["_train_engine"] = eng
    elif eng.param_version() != eng._packed_version:
        eng.repack()
    if torch.is_grad_enabled() and any(p.requires_grad for p in eng.params):
        logits = _TrainForwardCl.apply(eng, images, *eng.params)
    else:
        logits, _ = eng.forward(images)
    # one multi-tensor launch for every BN's counter
    torch._foreach_add_([bn.num_batches_tracked for bn in eng.bns], 1)
    model.invalidate_plans(ENCODER_PLANS)
    return logits


class _ClStepLR:
    """MyStepLR (learning/lr_scheduler.py:6-35) over the reference's two SGD groups
    (instantiators.py:806-807): each group's rate is max(base_g * gamma ** (epoch //
    step_size), min_lr); ``trainer.lrs`` follows every ``step()`` (once per epoch,
    main.py:114).  ``state_dict()`` is what the reference checkpoints as 'lr_scheduler'."""

    def __init__(self, trainer: ClassifierTrainer, step_size: int, gamma: float,
                 min_lr: float):
        from .training import MyStepLR
        self._trainer = trainer
        shadow = torch.optim.SGD([{"params": [torch.zeros(1, requires_grad=True)], "lr": lr}
                                  for lr in trainer.lrs], lr=trainer.lrs[0])
        self._sched = MyStepLR(shadow, step_size=step_size, gamma=gamma, min_lr=min_lr)

    def step(self) -> None:
        self._sched.optimizer.step()   # no gradients: keeps the scheduler's order check
        self._sched.step()
        self._trainer.lrs = [float(v) for v in self._sched.get_last_lr()]

    def state_dict(self):
        return self._sched.state_dict()

    def load_state_dict(self, sd) -> None:
        self._sched.load_state_dict(sd)
        for g, lr in zip(self._sched.optimizer.param_groups, self._sched.get_last_lr()):
            g["lr"] = lr
        self._trainer.lrs = [float(v) for v in self._sched.get_last_lr()]


def lr_schedule(trainer: ClassifierTrainer, step_size: int, gamma: float,
                min_lr: float) -> _ClStepLR:
    """The stage-1 trainer's per-epoch schedule (opt__lr_scheduler 'mystep')."""
    return _ClStepLR(trainer, step_size, gamma, min_lr)
