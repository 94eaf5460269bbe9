"""TEST INFRASTRUCTURE ONLY — torch-CPU autograd restatement of one TCAM training step
(and of the stage-1 STD_CL step, :func:`stdcl_step`)
(learning/train_wsol.py:685-884 for task TCAM, freeze_cl=True) over a reference-named
state_dict: frozen eval-mode encoder + WGAP, train-mode (batch-statistics) decoder BN,
SelfLearningTcams + ConRanFieldTcams + MaxSizePositiveTcams (losses/tcam.py:48-278,
elb.py:119-137, crf/dense_crf_loss.py:33-77), then torch.optim.SGD(momentum, dampening,
weight_decay, nesterov) — torch's own optimizer, i.e. the reference's.

``amp=True`` restates the reference's ``--amp True`` step (train_wsol.py:1077, 1155-1184:
``autocast`` + ``GradScaler``) in fp64 with autocast's fp16 tensors made explicit: every
tensor that is fp16 under autocast (conv inputs / weights / outputs, the BatchNorm-ReLU
outputs, the seg head's output) is rounded to fp16 in the forward AND its gradient is rounded
to fp16 in the backward (:class:`_R16`); the loss is scaled by the GradScaler scale before
the backward and the gradients are divided by it before the SGD step.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import crf_ref
from . import model_ref as R


class _CRF(torch.autograd.Function):
    """DenseCRFLossFunction (crf/dense_crf_loss.py:33-77): forward -sum(S AS)/N with AS from
    the reference permutohedral filter; backward -2 g AS / N."""

    @staticmethod
    def forward(ctx, images, S, sigma_rgb, sigma_xy):
        n = S.shape[0]
        s_np = S.detach().numpy().astype(np.float32)
        if crf_ref.ref_available():
            AS = crf_ref.ref_bilateral(images.numpy(), s_np, sigma_rgb, sigma_xy)
        else:
            AS = crf_ref.port_bilateral(images.numpy(), s_np, sigma_rgb, sigma_xy)
        AS = torch.from_numpy(AS).to(S.dtype)
        ctx.save_for_backward(AS)
        ctx.n = n
        return (-(S.detach() * AS).sum() / n).view(1)

    @staticmethod
    def backward(ctx, g):
        (AS,) = ctx.saved_tensors
        return None, -2 * g * AS / ctx.n, None, None


class _ColorCRF(torch.autograd.Function):
    """ColorDenseCRFLossFunction (crf/color_dense_crf_loss.py:31-78): the colour-only
    filter with DIM = the image's planes; forward -sum(S AS)/N, backward -2 g AS / N."""

    @staticmethod
    def forward(ctx, images, S, sigma_rgb):
        n = S.shape[0]
        s_np = S.detach().numpy().astype(np.float32)
        im = images.detach().numpy().astype(np.float32)
        if crf_ref.ref_available("color"):
            AS = crf_ref.ref_colorbilateral(im, s_np, sigma_rgb, im.shape[1])
        else:
            AS = crf_ref.port_bilateral(im, s_np, sigma_rgb, dim=im.shape[1])
        AS = torch.from_numpy(AS).to(S.dtype)
        ctx.save_for_backward(AS)
        ctx.n = n
        return (-(S.detach() * AS).sum() / n).view(1)

    @staticmethod
    def backward(ctx, g):
        (AS,) = ctx.saved_tensors
        return None, -2 * g * AS / ctx.n, None


def group_ordered_frames(seq_iter, frm_iter):
    """losses/tcam.py:32-45: batch positions per sequence id (ascending), each ordered by
    frame id with a stable sort."""
    seq = torch.as_tensor(seq_iter).reshape(-1)
    frm = torch.as_tensor(frm_iter).reshape(-1)
    out = []
    for sv in torch.unique(seq, sorted=True):
        idx = torch.nonzero(seq == sv, as_tuple=False).view(-1).tolist()
        out.append(sorted(idx, key=lambda i: float(frm[i])))
    return out


def rgb_joint_crf(fcams: torch.Tensor, raw: torch.Tensor, seq_iter, frm_iter,
                  lam: float = 2e-9, sigma_rgb: float = 15.0) -> torch.Tensor:
    """RgbJointConRanFieldTcams.forward (losses/tcam.py:186-205) with pair_samples'
    width mosaic (:207-232) and ColorDenseCRFLoss at scale_factor 1
    (color_dense_crf_loss.py:104-127): mean over the groups of >= 2 frames of
    lam * ColorDenseCRF(mosaic); 0 / 0 when there is none."""
    S = F.softmax(fcams, dim=1)
    loss = fcams.sum() * 0
    c = 0.0
    for item in group_ordered_frames(seq_iter, frm_iter):
        if len(item) < 2:
            continue
        im = torch.cat([raw[i:i + 1] for i in item], dim=3)
        pc = torch.cat([S[i:i + 1] for i in item], dim=3)
        loss = loss + lam * _ColorCRF.apply(im, pc, sigma_rgb).sum()
        c += 1.0
    return loss / c if c else loss * float("nan")


class _R16(torch.autograd.Function):
    """An fp16 tensor of the autocast graph: the value and its gradient rounded to fp16."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.float16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.float16).to(g.dtype)


def r16(x: torch.Tensor) -> torch.Tensor:
    return _R16.apply(x)


def _elb(fx: torch.Tensor, t: float) -> torch.Tensor:
    # ELB.forward (elb.py:119-137), elementwise then mean
    ct = -(1. / t ** 2)
    less = -(1. / t) * torch.log(-fx.clamp(max=ct))
    great = t * fx - (1. / t) * np.log(1. / t ** 2) + (1. / t)
    return torch.where(fx <= ct, less, great).mean()


def _bn_train(x, w, b, rm, rv, eps=1e-5, momentum=0.1):
    return F.batch_norm(x, rm, rv, w, b, True, momentum, eps)


def decoder_train(p: Dict[str, torch.Tensor], bufs: Dict[str, torch.Tensor], feats,
                  n_blocks: int, center: bool, masks: Optional[Dict[str, torch.Tensor]] = None,
                  amp: bool = False):
    """UnetTCAMDecoder.forward (unet/decoder.py:267-283) in train mode.

    ``masks`` (optional, {"decoder.blocks.i.convj": bool NCHW}): the ReLU branch taken at
    every pixel by the device forward under test.  relu(z) becomes z * mask, so the
    oracle differentiates the SAME piecewise-linear branch as the device step; without it
    a pre-activation within fp32 rounding of 0 may take the other branch, which moves
    that pixel's gradient discontinuously (not a kernel error).
    ``amp``: autocast's fp16 tensors (see the module docstring)."""
    q = r16 if amp else (lambda t: t)

    def c2r(x, pre):
        y = q(F.conv2d(q(x), q(p[pre + ".0.weight"]), padding=1))
        z = _bn_train(y, p[pre + ".1.weight"], p[pre + ".1.bias"],
                      bufs[pre + ".1.running_mean"], bufs[pre + ".1.running_var"])
        if masks is not None:
            return q(z * masks[pre].to(z.dtype))
        return q(F.relu(z))
    fs = feats[1:][::-1]
    x, skips = fs[0], fs[1:]
    if center:
        x = c2r(x, "decoder.center.0")
        x = c2r(x, "decoder.center.1")
    for i in range(n_blocks):
        skip = skips[i] if i < len(skips) else None
        x = F.interpolate(x, scale_factor=2, mode="nearest")
        if skip is not None:
            if x.shape[2:] != skip.shape[2:]:
                x = q(F.interpolate(x, size=skip.shape[2:], mode="bilinear",
                                    align_corners=True))
            x = torch.cat([x, skip], dim=1)
        x = c2r(x, f"decoder.blocks.{i}.conv1")
        x = c2r(x, f"decoder.blocks.{i}.conv2")
    return x


def tcam_losses(fcams: torch.Tensor, raw: torch.Tensor, seeds: Optional[torch.Tensor],
                lam_sl=1.0, lam_crf=2e-9, lam_size=0.01, elb_t=1.0, sigma_rgb=15.0,
                sigma_xy=100.0):
    """MasterLoss over SelfLearningTcams + ConRanFieldTcams + MaxSizePositiveTcams
    (losses/master.py:59-67, losses/tcam.py:48-115, 235-278; DenseCRFLoss with
    scale_factor 1, dense_crf_loss.py:95-123).  Returns (total, sl, crf, size) as
    autograd tensors; a zero lambda drops the term, like the reference's loss list."""
    S = F.softmax(fcams, dim=1)
    zero = fcams.sum() * 0
    sl = lam_sl * F.cross_entropy(fcams, seeds.long(), reduction="mean", ignore_index=-255) \
        if lam_sl else zero
    crf = (lam_crf * _CRF.apply(raw, S, sigma_rgb, sigma_xy)).sum() if lam_crf else zero
    size = zero
    if lam_size:
        n = S.shape[0]
        size = None
        for c in (0, 1):
            bl = S[:, c].reshape(n, -1).sum(dim=-1)
            v = _elb(-bl, elb_t)
            size = v if size is None else size + v
        size = lam_size * size * 0.5
    return sl + crf + size, sl, crf, size


def train_step(sd: Dict[str, torch.Tensor], x: torch.Tensor, raw: torch.Tensor,
               seeds: torch.Tensor, lr=0.01, momentum=0.9, dampening=0.0, weight_decay=1e-4,
               nesterov=True, lam_sl=1.0, lam_crf=2e-9, lam_size=0.01, elb_t=1.0,
               sigma_rgb=15.0, sigma_xy=100.0, dtype=torch.float64,
               masks: Optional[Dict[str, torch.Tensor]] = None, amp: bool = False,
               scale: float = 2.0 ** 16, feats=None
               ) -> Tuple[Dict[str, float], Dict, Dict, Dict]:
    """Returns (losses, grads, new_params, new_buffers) for the trainable decoder + seg head.
    dtype float64 (default): the accurate reference the fp32 GPU step is checked against.
    ``masks``: see :func:`decoder_train`.  ``amp``: the --amp step (module docstring) with
    GradScaler scale ``scale``; the grads returned are the unscaled ones the optimizer sees.
    ``feats``: the frozen encoder's features [x, f1 .. f5] (NCHW) to use instead of
    computing them (the amp check feeds the device's autocast encoder features)."""
    sd = {k: (v.detach().clone().to(dtype) if v.is_floating_point() else v.clone())
          for k, v in sd.items()}
    x = x.to(dtype)
    with torch.no_grad():
        if feats is None:
            feats = R.encoder_features(sd, x)
        else:
            feats = [f.detach().to(dtype) for f in feats]
    train_keys = [k for k in sd if k.startswith(("decoder.", "segmentation_head.")) and
                  not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
    params = {k: sd[k].clone().requires_grad_(True) for k in train_keys}
    bufs = {k: sd[k].clone() for k in sd if k.startswith("decoder.") and
            k.endswith(("running_mean", "running_var"))}
    n_blocks = sum(1 for k in sd if k.startswith("decoder.blocks.") and
                   k.endswith(".conv1.0.weight"))
    d = decoder_train(params, bufs, feats, n_blocks, "decoder.center.0.0.weight" in sd, masks,
                      amp)
    q = r16 if amp else (lambda t: t)
    fcams = q(F.conv2d(q(d), q(params["segmentation_head.0.weight"]),
                       q(params["segmentation_head.0.bias"]), padding=1))
    if fcams.shape[2:] != x.shape[2:]:   # base/model.py:148-154
        fcams = q(F.interpolate(fcams, size=x.shape[2:], mode="bilinear", align_corners=True))
    # (autocast: softmax / the losses run in fp32 on the fp16 fcams, losses/tcam.py)
    total, sl, crf, size = tcam_losses(fcams, raw, seeds, lam_sl, lam_crf, lam_size, elb_t,
                                       sigma_rgb, sigma_xy)
    if amp:   # scaler.scale(loss).backward(); scaler.unscale_(optimizer)
        (total * scale).backward()
        for k in train_keys:
            params[k].grad /= scale
    else:
        total.backward()
    grads = {k: params[k].grad.detach().clone() for k in train_keys}
    opt = torch.optim.SGD([params[k] for k in train_keys], lr=lr, momentum=momentum,
                          dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
    opt.step()
    new = {k: params[k].detach().clone() for k in train_keys}
    losses = {"total": float(total.detach()), "sl": float(sl.detach()),
              "crf": float(crf.detach().sum()), "size": float(size.detach())}
    return losses, grads, new, bufs


# ---------------------------------------------------------------- stage 1 (STD_CL)
def resnet50_train_features(p: Dict[str, torch.Tensor], bufs: Dict[str, torch.Tensor],
                            x: torch.Tensor, masks: Optional[Dict[str, torch.Tensor]] = None,
                            amp: bool = False, pre: str = "encoder.") -> torch.Tensor:
    """The WSOL ResNet50 encoder in train mode (encoders/resnet.py:140-153, 214-232:
    batch-statistics BatchNorm, running statistics updated in ``bufs``) -> layer4's output.

    ``masks`` ({"<pre>relu" | "<pre>layerL.B.relu{1,2,3}": bool NCHW}): the ReLU branch the
    device forward under test took (relu(z) -> z * mask), as :func:`decoder_train`.
    ``amp``: autocast's fp16 tensors (conv inputs / weights / outputs, every BatchNorm output,
    the residual sum, the ReLU outputs) rounded to fp16, values and gradients."""
    q = r16 if amp else (lambda t: t)

    def bn(y, name):
        return q(_bn_train(y, p[name + ".weight"], p[name + ".bias"],
                           bufs[name + ".running_mean"], bufs[name + ".running_var"]))

    def relu(z, name):
        if masks is not None:
            return q(z * masks[name].to(z.dtype))
        return q(F.relu(z))

    def conv(t, name, stride=1, padding=0):
        return q(F.conv2d(q(t), q(p[name]), stride=stride, padding=padding))

    f = relu(bn(conv(x, pre + "conv1.weight", 2, 3), pre + "bn1"), pre + "relu")
    f = F.max_pool2d(f, 3, 2, 1)
    for li, (nblk, stride) in enumerate(((3, 1), (4, 2), (6, 1), (3, 1)), start=1):
        for bi in range(nblk):
            b = f"{pre}layer{li}.{bi}"
            s = stride if bi == 0 else 1
            o = relu(bn(conv(f, b + ".conv1.weight"), b + ".bn1"), b + ".relu1")
            o = relu(bn(conv(o, b + ".conv2.weight", s, 1), b + ".bn2"), b + ".relu2")
            o = bn(conv(o, b + ".conv3.weight"), b + ".bn3")
            if b + ".downsample.0.weight" in p:
                idn = bn(conv(f, b + ".downsample.0.weight", s), b + ".downsample.1")
            else:
                idn = f
            f = relu(q(o + idn), b + ".relu3")
    return f


def stdcl_param_groups(keys):
    """process/instantiators.py:736-807 for resnet50: ``encoder.layer4.*`` and
    ``classification_head.*`` at lr * lr_classifier_ratio, the rest at lr."""
    cls = [k for k in keys if k.startswith(("encoder.layer4.", "classification_head."))]
    feat = [k for k in keys if k not in cls]
    return feat, cls


def stdcl_step(sd: Dict[str, torch.Tensor], x: torch.Tensor, labels: torch.Tensor,
               lr=0.001, lr_classifier_ratio=10.0, momentum=0.9, dampening=0.0,
               weight_decay=1e-4, nesterov=True, cl_lambda=1.0, dtype=torch.float64,
               masks: Optional[Dict[str, torch.Tensor]] = None, amp: bool = False,
               scale: float = 2.0 ** 16):
    """One stage-1 step (learning/train_wsol.py:700-714 task STD_CL, --freeze_encoder False):
    ``cl_logits = STDClassifier(x)`` in train mode (encoder + WGAP, poolings/core.py:109-115),
    ``loss = ClLoss`` (lambda * nn.CrossEntropyLoss, losses/std.py:19-53), backward, and
    torch.optim.SGD over the reference's two parameter groups.  Returns (loss, logits, grads,
    new_params, new_buffers).  ``amp``: autocast (fp16 convs / BN outputs / pool / fc, CE in
    fp32 on the fp16 logits) with the GradScaler scale ``scale``; grads are unscaled."""
    sd = {k: (v.detach().clone().to(dtype) if v.is_floating_point() else v.clone())
          for k, v in sd.items()}
    x = x.to(dtype)
    keys = [k for k in sd if not k.endswith(("running_mean", "running_var",
                                              "num_batches_tracked"))]
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    bufs = {k: sd[k].clone() for k in sd if k.endswith(("running_mean", "running_var"))}
    q = r16 if amp else (lambda t: t)
    f = resnet50_train_features(params, bufs, x, masks, amp)
    pooled = q(F.adaptive_avg_pool2d(f, 1).flatten(1))
    logits = q(F.linear(q(pooled), q(params["classification_head.fc.weight"]),
                        q(params["classification_head.fc.bias"])))
    loss = cl_lambda * F.cross_entropy(logits, labels.long(), reduction="mean")
    if amp:
        (loss * scale).backward()
        for k in keys:
            params[k].grad /= scale
    else:
        loss.backward()
    grads = {k: params[k].grad.detach().clone() for k in keys}
    feat, cls = stdcl_param_groups(keys)
    opt = torch.optim.SGD([{"params": [params[k] for k in feat], "lr": lr},
                           {"params": [params[k] for k in cls],
                            "lr": lr * lr_classifier_ratio}],
                          lr=lr, momentum=momentum, dampening=dampening,
                          weight_decay=weight_decay, nesterov=nesterov)
    opt.step()
    new = {k: params[k].detach().clone() for k in keys}
    return float(loss.detach()), logits.detach(), grads, new, bufs
