"""Drop-in TCAM / STD_CL models whose forward runs on the gfx950 kernels.

Module and parameter names reproduce the reference exactly so that strict
``state_dict`` loads of reference checkpoints work and CAM hook names
resolve:

* ``UnetTCAM``       dlib/unet/model.py:280-417 (TCAMModel = FCAMModel,
                     base/model.py:109-259); decoder dlib/unet/decoder.py.
* ``STDClassifier``  dlib/stdcl/classifier.py:19-59 (STDClModel,
                     base/model.py:15-107).
* ``ResNetEncoder``  dlib/encoders/resnet.py:57-153 (+ Bottleneck 175-232,
                     torchvision 0.12 ``_make_layer``): WSOL variant with
                     stride 1 in layer3 and layer4.
* ``WGAP``           dlib/poolings/core.py:96-115.
* ``SegmentationHead`` dlib/base/heads.py:19-36.

``forward`` keeps the reference contract — ``UnetTCAM.forward(x) ->
(cl_logits, fcams, None)`` and sets ``self.x_in`` / ``self.cams`` — but the
whole batch goes through hand-written HIP kernels (ops.py) with BatchNorm
folded into the convolution weights (eval mode only; see DESIGN.md for the
training-path status).  There is no CPU path: CPU inputs raise.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import ops
from .ops import ConvSrc

TCAM = "TCAM"
STD_CL = "STD_CL"
F_CL = "F_CL"

RESNET50 = "resnet50"
# constants.py:276-285
TRG_LAYERS = {RESNET50: "encoder.layer4.2.relu3", "vgg16": "encoder.relu",
              "inceptionv3": "encoder.SPG_A3_2b.2"}
FC_LAYERS = {RESNET50: "classification_head.fc", "vgg16": "classification_head.fc",
             "inceptionv3": "classification_head.fc"}


def count_params(model: nn.Module) -> int:
    """utils/shared.py:208-209."""
    return sum(p.numel() for p in model.parameters())


# --------------------------------------------------------------- modules
class Bottleneck(nn.Module):
    """encoders/resnet.py:175-232 (torchvision V1.5 layout: stride on conv2)."""
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu1 = nn.ReLU(inplace=False)
        self.relu2 = nn.ReLU(inplace=False)
        self.relu3 = nn.ReLU(inplace=False)
        self.downsample = downsample
        self.stride = stride


class ResNetEncoder(nn.Module):
    """WSOL ResNet50 encoder (encoders/resnet.py:57-153): layer3/layer4 stride 1."""

    def __init__(self, layers=(3, 4, 6, 3), out_channels=(3, 64, 256, 512, 1024, 2048),
                 depth: int = 5):
        super().__init__()
        self._depth = depth
        self._out_channels = tuple(out_channels)
        self._in_channels = 3
        self.name = RESNET50
        self.task = None
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=False)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0], 1)
        self.layer2 = self._make_layer(128, layers[1], 2)
        self.layer3 = self._make_layer(256, layers[2], 1)   # WSOL: stride_l3 = 1
        self.layer4 = self._make_layer(512, layers[3], 1)   # WSOL: z_stride = 1

    def _make_layer(self, planes: int, blocks: int, stride: int) -> nn.Sequential:
        # torchvision==0.12 ResNet._make_layer semantics (no dilation, groups=1).
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, 1, stride=stride,
                          bias=False),
                nn.BatchNorm2d(planes * Bottleneck.expansion))
        mods = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            mods.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*mods)

    @property
    def out_channels(self):
        return self._out_channels[: self._depth + 1]

    def set_task(self, task: str):
        self.task = task

    def set_model_name(self, name: str):
        self.name = name


    def load_state_dict(self, state_dict, strict: bool = True, **kw):
        """encoders/resnet.py:155-158: drops torchvision's ``fc.*`` (ImageNet weights)."""
        state_dict = dict(state_dict)
        state_dict.pop("fc.bias", None)
        state_dict.pop("fc.weight", None)
        return super().load_state_dict(state_dict, strict=strict, **kw)

    def super_load_state_dict(self, state_dict, **kw):
        """encoders/resnet.py:160-161 (checkpoint loads, instantiators.py:664-667)."""
        return super().load_state_dict(state_dict, **kw)

class Conv2dReLU(nn.Sequential):
    """base/modules.py:10-49 with use_batchnorm=True: (conv, bn, relu)."""

    def __init__(self, cin: int, cout: int, kernel_size: int, padding: int = 0):
        super().__init__(nn.Conv2d(cin, cout, kernel_size, padding=padding, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class DecoderBlock(nn.Module):
    """unet/decoder.py:14-57 (attention_type=None -> Identity)."""

    def __init__(self, in_channels: int, skip_channels: int, out_channels: int):
        super().__init__()
        self.conv1 = Conv2dReLU(in_channels + skip_channels, out_channels, 3, padding=1)
        self.attention1 = nn.Identity()
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1)
        self.attention2 = nn.Identity()


class CenterBlock(nn.Sequential):
    """unet/decoder.py:60-76 (VGG encoders only)."""

    def __init__(self, cin: int, cout: int):
        super().__init__(Conv2dReLU(cin, cout, 3, padding=1), Conv2dReLU(cout, cout, 3, padding=1))


class UnetTCAMDecoder(nn.Module):
    """unet/decoder.py:164-287 (UnetTCAMDecoder = UnetFCAMDecoder)."""

    def __init__(self, encoder_channels: Sequence[int], decoder_channels: Sequence[int],
                 n_blocks: int = 5, center: bool = False):
        super().__init__()
        if n_blocks != len(decoder_channels):
            raise ValueError(f"Model depth is {n_blocks}, but you provide `decoder_channels` "
                             f"for {len(decoder_channels)} blocks.")
        enc = list(encoder_channels[1:])[::-1]
        head = enc[0]
        in_ch = [head] + list(decoder_channels[:-1])
        skip_ch = list(enc[1:]) + [0]
        self.center = CenterBlock(head, head) if center else nn.Identity()
        self.blocks = nn.ModuleList([DecoderBlock(i, s, o) for i, s, o in
                                     zip(in_ch, skip_ch, decoder_channels)])


class WGAP(nn.Module):
    """poolings/core.py:96-115: AdaptiveAvgPool2d(1) + Linear."""

    def __init__(self, in_channels: int, classes: int, support_background: bool = False,
                 **unused):
        super().__init__()
        self.in_channels = in_channels
        self.classes = classes
        self.support_background = support_background
        self.cams = None
        self.name = "WGAP"
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(in_channels, classes)

    @property
    def builtin_cam(self):
        return False


class SegmentationHead(nn.Sequential):
    """base/heads.py:19-36 (activation=None, upsampling=1)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3):
        super().__init__(nn.Conv2d(in_channels, out_channels, kernel_size,
                                   padding=kernel_size // 2),
                         nn.Identity(), nn.Identity())


POOLINGS = {"WGAP": WGAP}


# ------------------------------------------------------------ BN folding
def fold_conv_bn(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Eval-mode BatchNorm folded into the conv: returns (W' (Cout,K) fp64, b' (Cout,) fp64).

    y = gamma * (conv(x) + b - mean) / sqrt(var + eps) + beta.
    """
    w = conv.weight.detach().double()
    cout = w.shape[0]
    w = w.reshape(cout, -1)
    b = conv.bias.detach().double() if conv.bias is not None else torch.zeros(cout, dtype=torch.float64,
                                                                              device=w.device)
    if bn is None:
        return w, b
    scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    return w * scale[:, None], bn.bias.detach().double() + (b - bn.running_mean.detach().double()) * scale


# ------------------------------------------- f16x3 activation exponents
# S2 keeps x = h + l in two fp16 parts; below |x| ~ 2^-3 the low part drops into fp16's
# subnormal range and the split loses bits (2^-25 absolute floor per element).  The f16x3
# plans therefore store each activation channel times a power of two 2^e (e >= 0) chosen at
# plan time from the BatchNorm that produced it: under the running statistics an eval-mode
# BN output has mean beta and std |gamma|, so its magnitude is ~ |beta| + 3 |gamma|; a channel
# whose estimate is below 2^-2 gets e with 2^e * estimate in [1, 2).  Every consumer absorbs
# the exponents exactly (power-of-two scaling of the fp64 folded weights): a conv multiplies
# weight [m, c] by 2^(e_out[m] - e_in[c]) and its bias by 2^e_out[m]; pools, the up-sampling
# and the concat act per channel; a residual add requires equal exponents (a ResNet stage's
# stream shares one vector); the classifier / CAM / seg-head weights divide by 2^e.  Layers
# of ordinary O(1) range get e = 0: their arithmetic is unchanged.  TCAM_F16_ACT_SCALE=0
# turns the exponents off (A/B and tests).
F16_SCALE_BELOW = 2.0 ** -2
F16_MAX_EXP = 16


def bn_magnitude(bn: nn.BatchNorm2d) -> torch.Tensor:
    """|beta| + 3 |gamma| per channel (fp64, CPU): the eval-mode BN output's range."""
    return (bn.bias.detach().double().abs() + 3.0 * bn.weight.detach().double().abs()).cpu()


def act_exponents(mag: torch.Tensor) -> Optional[torch.Tensor]:
    """Per-channel e >= 0 (int64, CPU) with 2^e * mag in [1, 2) where mag < 2^-2, else 0;
    None when every channel keeps e = 0 (or TCAM_F16_ACT_SCALE=0)."""
    if os.environ.get("TCAM_F16_ACT_SCALE", "1") == "0":
        return None
    mag = mag.double().cpu()
    e = torch.zeros(mag.numel(), dtype=torch.int64)
    small = (mag < F16_SCALE_BELOW) & (mag > 0)
    if bool(small.any()):
        e[small] = (-torch.floor(torch.log2(mag[small]))).clamp(max=F16_MAX_EXP).long()
    return e if bool((e != 0).any()) else None


def cat_exponents(parts: Sequence[Tuple[Optional[torch.Tensor], int]]) -> Optional[torch.Tensor]:
    """Concatenate per-source exponent vectors ((vector or None, channels) pairs)."""
    if all(e is None for e, _ in parts):
        return None
    return torch.cat([e if e is not None else torch.zeros(n, dtype=torch.int64)
                      for e, n in parts])


def unscale_in(w: torch.Tensor, e_in: Optional[torch.Tensor]) -> torch.Tensor:
    """A consumer weight (Cout, Cin, ...) over activations stored times 2^e_in[c]:
    w[:, c] * 2^-e_in[c] (exact)."""
    if e_in is None:
        return w
    f = torch.pow(2.0, -e_in.double()).to(device=w.device, dtype=w.dtype)
    return (w * f.reshape((1, -1) + (1,) * (w.dim() - 2))).contiguous()


def exps_signature(exps: Sequence[Optional[torch.Tensor]]) -> str:
    """A plan-cache key suffix for a feature-exponent list ("" when all are zero)."""
    if all(e is None for e in exps):
        return ""
    return ":" + "|".join("" if e is None else ",".join(map(str, e.tolist())) for e in exps)


def features_fc_weight(model) -> torch.Tensor:
    """The classifier weight to apply to ``model.features`` (the CAM hook's activations,
    which the f16x3 plans store times 2^features_exp)."""
    w = model.classification_head.fc.weight.detach().contiguous()
    return unscale_in(w, getattr(model, "features_exp", None))


class FoldedConv:
    """A conv (+BN) ready for the conv kernels: packed tap-major weights and bias.

    fmt "fp32": (Kpad, Mpad) fp32 for ``tcam_conv2d``; "x6": the split
    (Kpad/32, 4, 3, Mpad, 8) bf16 operand of ``tcam_conv2d_x6``; "f16x3": the split
    (Kpad/32, 4, 2, Mpad, 8) fp16 operand of ``tcam_conv2d_f16x3`` with its per-channel
    scales ``wscale`` (None for the other formats); "amp": the (Kpad/32, 4, 1, Mpad, 8)
    fp16 operand of ``tcam_conv2d_f16`` (the folded weight rounded to fp16).  ``cin_pad``
    zero-pads the input channels of a single-source conv (the stem reads the
    image padded to 8 channels on the x6 path).
    """

    __slots__ = ("wt", "wscale", "bias", "cout", "k", "pad", "stride")

    def __init__(self, parts: Sequence[Tuple[nn.Conv2d, Optional[nn.BatchNorm2d]]],
                 device: torch.device, fmt: str = "fp32", cin_pad: Optional[int] = None,
                 ein: Optional[Sequence[Optional[torch.Tensor]]] = None,
                 eout: Optional[torch.Tensor] = None):
        """``ein`` (per part: its input channels' exponents or None) / ``eout`` (output
        channels'): activations stored times 2^e (f16x3 plans, see act_exponents); the
        folded weights and bias absorb them exactly."""
        ws, bsum = [], None
        for i, (conv, bn) in enumerate(parts):
            w, b = fold_conv_bn(conv, bn)
            w = w.reshape(conv.weight.shape)
            e_in = ein[i] if ein is not None else None
            if e_in is not None or eout is not None:
                d = torch.zeros((w.shape[0], w.shape[1]), dtype=torch.float64)
                if eout is not None:
                    d += eout.double()[:, None]
                    b = b * torch.pow(2.0, eout.double()).to(b.device)
                if e_in is not None:
                    d -= e_in.double()[None, :]
                w = w * torch.pow(2.0, d).to(w.device)[:, :, None, None]
            w = w.float().to(device)
            if cin_pad is not None and cin_pad > w.shape[1]:
                w = torch.cat([w, w.new_zeros((w.shape[0], cin_pad - w.shape[1]) +
                                              tuple(w.shape[2:]))], dim=1)
            ws.append(w)
            bsum = b if bsum is None else bsum + b
        self.wscale = None
        if fmt == "f16x3":
            self.wt, self.wscale = ops.pack_conv_weight_f16(ws)
        elif fmt == "amp":
            self.wt = ops.pack_conv_weight_h1(ws)
        elif fmt == "x6":
            self.wt = ops.pack_conv_weight_x6(ws)
        else:
            self.wt = ops.pack_conv_weight(ws)
        self.bias = bsum.float().contiguous().to(device)
        conv0 = parts[0][0]
        self.cout = conv0.out_channels
        self.k = conv0.kernel_size[0]
        self.pad = conv0.padding[0]
        self.stride = conv0.stride[0]


def _param_version(m: nn.Module) -> int:
    v = 0
    for t in list(m.parameters()) + list(m.buffers()):
        v += t._version + t.data_ptr() % 9973
    return v


# -------------------------------------------------------- HIP executors
class _ResNetPlan:
    """Folded weights of the WSOL ResNet50 encoder for the HIP forward."""

    def __init__(self, enc: ResNetEncoder, device):
        self.stem = FoldedConv([(enc.conv1, enc.bn1)], device)
        self.layers: List[List[Tuple[FoldedConv, FoldedConv, FoldedConv, bool, int]]] = []
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
            blocks = []
            for blk in layer:
                c1 = FoldedConv([(blk.conv1, blk.bn1)], device)
                c2 = FoldedConv([(blk.conv2, blk.bn2)], device)
                if blk.downsample is not None:
                    # conv3 and the projection shortcut share one GEMM over a
                    # concatenated K; their folded biases add.
                    c3 = FoldedConv([(blk.conv3, blk.bn3),
                                     (blk.downsample[0], blk.downsample[1])], device)
                    ds_stride = blk.downsample[0].stride[0]
                else:
                    c3 = FoldedConv([(blk.conv3, blk.bn3)], device)
                    ds_stride = 0
                blocks.append((c1, c2, c3, blk.downsample is not None, ds_stride))
            self.layers.append(blocks)

    def forward(self, x: torch.Tensor, keep_all: bool = True) -> List[torch.Tensor]:
        B, _, H, W = x.shape
        feats = [x]
        s = self.stem
        H1, W1 = (H + 2 * 3 - 7) // 2 + 1, (W + 2 * 3 - 7) // 2 + 1
        f = ops.conv2d([ConvSrc(x, 2)], s.wt, s.bias, s.cout, H1, W1, 7, 3, True)
        feats.append(f)
        f = ops.maxpool3x3s2(f)
        for blocks in self.layers:
            for c1, c2, c3, has_ds, ds_stride in blocks:
                Hi, Wi = f.shape[2], f.shape[3]
                h1 = ops.conv2d([ConvSrc(f)], c1.wt, c1.bias, c1.cout, Hi, Wi, 1, 0, True)
                st = c2.stride
                Ho, Wo = (Hi + 2 - 3) // st + 1, (Wi + 2 - 3) // st + 1
                h2 = ops.conv2d([ConvSrc(h1, st)], c2.wt, c2.bias, c2.cout, Ho, Wo, 3, 1, True)
                if has_ds:
                    f = ops.conv2d([ConvSrc(h2), ConvSrc(f, ds_stride)], c3.wt, c3.bias,
                                   c3.cout, Ho, Wo, 1, 0, True)
                else:
                    f = ops.conv2d([ConvSrc(h2)], c3.wt, c3.bias, c3.cout, Ho, Wo, 1, 0, True,
                                   residual=f)
            feats.append(f)
        return feats


class _DecoderPlan:
    def __init__(self, dec: UnetTCAMDecoder, device):
        self.center = None
        if isinstance(dec.center, CenterBlock):
            self.center = [FoldedConv([(c[0], c[1])], device) for c in dec.center]
        self.blocks = [(FoldedConv([(b.conv1[0], b.conv1[1])], device),
                        FoldedConv([(b.conv2[0], b.conv2[1])], device)) for b in dec.blocks]

    def forward(self, feats: Sequence[torch.Tensor]) -> torch.Tensor:
        fs = list(feats[1:])[::-1]
        x, skips = fs[0], fs[1:]
        if self.center is not None:
            for c in self.center:
                x = ops.conv2d([ConvSrc(x)], c.wt, c.bias, c.cout, x.shape[2], x.shape[3], 3, 1,
                               True)
        for i, (c1, c2) in enumerate(self.blocks):
            skip = skips[i] if i < len(skips) else None
            h, w = x.shape[2], x.shape[3]
            if skip is None:
                srcs = [ConvSrc(x, up2=True)]
                Ho, Wo = 2 * h, 2 * w
            else:
                Ho, Wo = skip.shape[2], skip.shape[3]
                if (2 * h, 2 * w) == (Ho, Wo):
                    srcs = [ConvSrc(x, up2=True), ConvSrc(skip)]
                else:  # nearest x2 then bilinear(align_corners=True) to the skip size
                    srcs = [ConvSrc(ops.up2_resize(x, (Ho, Wo))), ConvSrc(skip)]
            x = ops.conv2d(srcs, c1.wt, c1.bias, c1.cout, Ho, Wo, 3, 1, True)
            x = ops.conv2d([ConvSrc(x)], c2.wt, c2.bias, c2.cout, Ho, Wo, 3, 1, True)
        return x


class _ResNetPlanX6:
    """The encoder on the x6 path: S3 activations, ``tcam_conv2d_x6`` (fmt "x6"), or on the
    f16x3 path: S2 activations, ``tcam_conv2d_f16x3`` (fmt "f16x3")."""

    def __init__(self, enc: ResNetEncoder, device, fmt: str = "x6"):
        self.fmt = fmt
        # f16x3: per-channel activation exponents (act_exponents); a stage's residual
        # stream shares one vector, from the summed magnitudes of its blocks' bn3 (+ the
        # projection shortcut's BN)
        scaled = fmt == "f16x3"

        def ex(bn):
            return act_exponents(bn_magnitude(bn)) if scaled else None
        e0 = ex(enc.bn1)
        self.stem = FoldedConv([(enc.conv1, enc.bn1)], device, fmt, cin_pad=8, eout=e0)
        # f16x3: the stem reads the fp32 image directly over its 147 real K (tcam_stem_f16x3)
        # instead of an NCHW -> S2 pass and 49 taps x 8 padded channels
        self.stem_direct = None
        if fmt == "f16x3" and os.environ.get("TCAM_STEM_DIRECT", "1") != "0":
            w, b = fold_conv_bn(enc.conv1, enc.bn1)
            if e0 is not None:
                f = torch.pow(2.0, e0.double()).to(w.device)
                w, b = w * f[:, None], b * f
            self.stem_direct = ops.StemF16(w.reshape(enc.conv1.weight.shape).float().to(device),
                                           b, enc.conv1.stride[0], enc.conv1.padding[0])
        self.layers = []
        # f16x3 / amp: layer 1's bottlenecks fused into one launch each
        # (ops.bottleneck_f16x3; TCAM_FUSED_L1=0 runs the three convs per block)
        self.fused_l1 = fmt in ("f16x3", "amp") and os.environ.get("TCAM_FUSED_L1", "1") != "0"
        e_prev = e0
        self.out_exps: List[Optional[torch.Tensor]] = [None, e0]
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
            blocks = []
            e_stream = None
            if scaled:
                mag = None
                for blk in layer:
                    m = bn_magnitude(blk.bn3)
                    if blk.downsample is not None:
                        m = m + bn_magnitude(blk.downsample[1])
                    mag = m if mag is None else mag + m
                e_stream = act_exponents(mag)
                if layer[0].downsample is None:   # the stream continues the input's
                    e_stream = e_prev
            for bi, blk in enumerate(layer):
                e_in = e_prev if bi == 0 else e_stream
                e1, e2 = ex(blk.bn1), ex(blk.bn2)
                c1 = FoldedConv([(blk.conv1, blk.bn1)], device, fmt, ein=[e_in], eout=e1)
                c2 = FoldedConv([(blk.conv2, blk.bn2)], device, fmt, ein=[e1], eout=e2)
                if blk.downsample is not None:
                    c3 = FoldedConv([(blk.conv3, blk.bn3),
                                     (blk.downsample[0], blk.downsample[1])], device, fmt,
                                    ein=[e2, e_in], eout=e_stream)
                    ds_stride = blk.downsample[0].stride[0]
                else:
                    c3 = FoldedConv([(blk.conv3, blk.bn3)], device, fmt, ein=[e2],
                                    eout=e_stream)
                    ds_stride = 0
                blocks.append((c1, c2, c3, blk.downsample is not None, ds_stride))
            self.layers.append(blocks)
            e_prev = e_stream
            self.out_exps.append(e_stream)

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        """x: (B, 3, H, W) fp32 image -> [x, stem, layer1..layer4] (S3 / S2 features)."""
        B, _, H, W = x.shape
        feats = [x]
        s = self.stem
        H1, W1 = (H + 2 * 3 - 7) // 2 + 1, (W + 2 * 3 - 7) // 2 + 1
        if self.stem_direct is not None:
            f = ops.stem_f16x3(x, self.stem_direct)
        else:
            xs = ops.s3_from_nchw(x, 8, self.fmt)
            f = ops.conv2d_x6([ConvSrc(xs, 2)], s.wt, s.bias, s.cout, H1, W1, 7, 3, True,
                              wscale=s.wscale)
        feats.append(f)
        f = ops.maxpool3x3s2_s3(f)
        for li, blocks in enumerate(self.layers):
            for c1, c2, c3, has_ds, ds_stride in blocks:
                if li == 0 and self.fused_l1 and c2.stride == 1 and (not has_ds or ds_stride == 1):
                    # f16x3 / amp: the whole stride-1 layer-1 block in one launch (round 5)
                    f = ops.bottleneck_f16x3(f, c1, c2, c3, has_ds)
                    continue
                Hi, Wi = f.shape[1], f.shape[2]
                h1 = ops.conv2d_x6([ConvSrc(f)], c1.wt, c1.bias, c1.cout, Hi, Wi, 1, 0, True,
                                   wscale=c1.wscale)
                st = c2.stride
                Ho, Wo = (Hi + 2 - 3) // st + 1, (Wi + 2 - 3) // st + 1
                h2 = ops.conv2d_x6([ConvSrc(h1, st)], c2.wt, c2.bias, c2.cout, Ho, Wo, 3, 1,
                                   True, wscale=c2.wscale)
                if has_ds:
                    f = ops.conv2d_x6([ConvSrc(h2), ConvSrc(f, ds_stride)], c3.wt, c3.bias,
                                      c3.cout, Ho, Wo, 1, 0, True, wscale=c3.wscale)
                else:
                    f = ops.conv2d_x6([ConvSrc(h2)], c3.wt, c3.bias, c3.cout, Ho, Wo, 1, 0,
                                      True, residual=f, wscale=c3.wscale)
            feats.append(f)
        return feats


class _DecoderPlanX6:
    def __init__(self, dec: UnetTCAMDecoder, device, fmt: str = "x6",
                 enc_exps: Optional[Sequence[Optional[torch.Tensor]]] = None):
        """``enc_exps``: the encoder plan's feature exponents ([x, f1 .. f5], f16x3 plans);
        the decoder's own activations get theirs from its BNs, and ``out_exp`` (the last
        block's) is for the seg head's weights."""
        scaled = fmt == "f16x3"

        def ex(bn):
            return act_exponents(bn_magnitude(bn)) if scaled else None
        fe = list(enc_exps[1:])[::-1] if (scaled and enc_exps is not None) else None
        x_e = fe[0] if fe else None
        self.center = None
        if isinstance(dec.center, CenterBlock):
            self.center = []
            for c in dec.center:
                e = ex(c[1])
                self.center.append(FoldedConv([(c[0], c[1])], device, fmt, ein=[x_e], eout=e))
                x_e = e
        self.blocks = []
        for i, b in enumerate(dec.blocks):
            conv1 = b.conv1[0]
            skip_e = fe[1 + i] if (fe and 1 + i < len(fe)) else None
            n_x = conv1.in_channels
            if skip_e is not None or x_e is not None:
                n_skip = skip_e.numel() if skip_e is not None else 0
                xin = n_x - n_skip if skip_e is not None else (
                    x_e.numel() if x_e is not None else n_x)
                ein = cat_exponents([(x_e, xin), (skip_e, n_x - xin)])
            else:
                ein = None
            e1, e2 = ex(b.conv1[1]), ex(b.conv2[1])
            self.blocks.append((FoldedConv([(conv1, b.conv1[1])], device, fmt, ein=[ein],
                                           eout=e1),
                                FoldedConv([(b.conv2[0], b.conv2[1])], device, fmt, ein=[e1],
                                           eout=e2)))
            x_e = e2
        self.out_exp = x_e

    def forward(self, feats: Sequence[torch.Tensor]) -> torch.Tensor:
        fs = list(feats[1:])[::-1]
        x, skips = fs[0], fs[1:]
        if self.center is not None:
            for c in self.center:
                x = ops.conv2d_x6([ConvSrc(x)], c.wt, c.bias, c.cout, x.shape[1], x.shape[2], 3,
                                  1, True, wscale=c.wscale)
        for i, (c1, c2) in enumerate(self.blocks):
            skip = skips[i] if i < len(skips) else None
            h, w = x.shape[1], x.shape[2]
            if skip is None:
                srcs = [ConvSrc(x, up2=True)]
                Ho, Wo = 2 * h, 2 * w
            else:
                Ho, Wo = skip.shape[1], skip.shape[2]
                if (2 * h, 2 * w) == (Ho, Wo):
                    srcs = [ConvSrc(x, up2=True), ConvSrc(skip)]
                else:
                    srcs = [ConvSrc(ops.up2_resize_s3(x, (Ho, Wo))), ConvSrc(skip)]
            x = ops.conv2d_x6(srcs, c1.wt, c1.bias, c1.cout, Ho, Wo, 3, 1, True, wscale=c1.wscale)
            x = ops.conv2d_x6([ConvSrc(x)], c2.wt, c2.bias, c2.cout, Ho, Wo, 3, 1, True,
                              wscale=c2.wscale)
        return x


# "f16x3" (the default for the eval plans): fp16-split MFMA on S2 (22-bit operands, three
# products: half the MFMA work and 2/3 of the bytes of x6; |activations| <= 65504, checked;
# per-layer error vs fp64 at or below x6's, profiles/round3_f16x3_layer_error.txt);
# "x6": fp32-accurate bf16-split MFMA on S3 (exact operands, six products; the training
# path's decoder); "fp32": native fp32 MFMA on NCHW (ResNet50 only); "amp": autocast's fp16
# convolutions (--amp / --amp_eval, train_wsol.py:1155-1184): fp16 operands on S1, one
# fp16 product per MAC accumulated in fp32, fp16 outputs — NOT fp32-accurate
CONV_PRECISIONS = ("x6", "f16x3", "fp32", "amp")
HIP_PRECISIONS = ("x6", "f16x3", "amp")


def _precision(m) -> str:
    p = getattr(m, "conv_precision", None) or os.environ.get("TCAM_CONV_PRECISION", "f16x3")
    if p not in CONV_PRECISIONS:
        raise ValueError(f"conv_precision must be one of {CONV_PRECISIONS}, got {p!r}")
    return p


def _check_f16(m, prec: str, device) -> None:
    """A direct forward on the f16x3 path raises when an activation left the S2 range
    (a host sync).  CAMComputer defers the check to the end of its evaluation
    (``_defer_f16_check``), so its pipelined clips do not synchronise."""
    if prec == "f16x3" and not m.__dict__.get("_defer_f16_check", False):
        # a direct forward raises on this rank only (no collective per call); the batched
        # evaluation (CAMComputer) and the trainer check all ranks together
        ops.check_f16_overflow(device, all_ranks=False)


# ---------------------------------------------------------------- models
def _check_input(x: torch.Tensor):
    if not isinstance(x, torch.Tensor) or x.dim() != 4:
        raise ValueError("expected a (B, 3, H, W) tensor")
    if not x.is_cuda:
        raise RuntimeError("tcam models run on the MI355X HIP path only; move the model and "
                           "input to 'cuda' (there is no CPU fallback)")


class _HipModelMixin:
    """Caches folded weights; rebuilt when any parameter/buffer changes."""

    def _plan_get(self, key: str, build, module: Optional[nn.Module] = None):
        """The folded plan ``key`` of ``module`` (default: the whole model), rebuilt when
        any parameter / buffer of that module changed (version counter or storage)."""
        ver = _param_version(self if module is None else module)
        cache = self.__dict__.setdefault("_plans", {})
        ent = cache.get(key)
        if ent is None or ent[0] != ver:
            # plans are shared by every stream that runs the model (CAMComputer pipelines
            # clips over several): drain users of the old plan, and finish the packing
            # kernels before any other stream may read the new one
            if torch.cuda.is_initialized():
                torch.cuda.synchronize()
            with torch.no_grad():
                ent = (ver, build())
            if torch.cuda.is_initialized():
                torch.cuda.synchronize()
            cache[key] = ent
        return ent[1]

    def invalidate_plans(self, keys: Optional[Sequence[str]] = None):
        """Drop cached plans (all, or ``keys``): needed after weights or BN statistics
        were written by a kernel (no tensor version bump)."""
        if keys is None:
            self.__dict__["_plans"] = {}
        else:
            plans = self.__dict__.setdefault("_plans", {})
            for k in list(plans):   # a key and its exponent-keyed variants ("<key>:...")
                if any(k == p or k.startswith(p + ":") for p in keys):
                    plans.pop(k)


class STDClassifier(nn.Module, _HipModelMixin):
    """dlib/stdcl/classifier.py:19-59 — encoder + WGAP head (stage-1 CAM model)."""

    # "f16x3" (default): fp16-split MFMA convs on S2 activations; "x6": exact bf16-split MFMA
    # convs on S3; "fp32": native fp32 MFMA convs on NCHW (see CONV_PRECISIONS).
    # None -> $TCAM_CONV_PRECISION or "f16x3".
    conv_precision: Optional[str] = None

    def __init__(self, task: str = STD_CL, encoder_name: str = RESNET50, encoder_depth: int = 5,
                 encoder_weights: Optional[str] = None, in_channels: int = 3,
                 aux_params: Optional[dict] = None, scale_in: float = 1.):
        super().__init__()
        _check_arch(encoder_name, encoder_weights, in_channels)
        self.encoder_name = encoder_name
        self.task = STD_CL
        assert scale_in > 0.
        self.scale_in = float(scale_in)
        self.x_in = None
        self.encoder = _make_encoder(encoder_name, encoder_depth)
        self.encoder.set_task(task)
        assert aux_params is not None
        aux = dict(aux_params)
        pooling_head = aux.pop("pooling_head")
        self.classification_head = POOLINGS[pooling_head](
            in_channels=self.encoder.out_channels[-1], **aux)
        self.name = f"u-{encoder_name}"
        self.features = None
        self.features_exp = None

    # base/model.py:36-50 (STDClModel)
    def __str__(self):
        return "{}. Task: {}.".format(self.name, self.task)

    def get_info_nbr_params(self) -> str:
        info = self.__str__() + " \n NBR-PARAMS: \n"
        info += "\tEncoder [{}]: {}. \n".format(self.encoder.name, count_params(self.encoder))
        info += "\tClassification head [{}]: {}. \n".format(
            self.classification_head.name, count_params(self.classification_head))
        info += "\tTotal: {}. \n".format(count_params(self))
        return info

    def free_mem(self):
        self.x_in = None
        self.features = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _check_input(x)
        if self.scale_in != 1.:
            raise NotImplementedError("scale_in != 1 is not on the TCAM hot path")
        self.x_in = x
        x = x.contiguous().float()
        if self.training and self.encoder_name == RESNET50:
            # stage-1 training (train_wsol.py:700-714, --freeze_encoder False): batch-statistics
            # BatchNorm, logits differentiable w.r.t. every parameter (cl_training)
            from .cl_training import train_forward
            self.features = self.features_exp = None
            return train_forward(self, x)
        head = self.classification_head
        fw, fb = head.fc.weight.detach().contiguous(), head.fc.bias.detach().contiguous()
        prec = _precision(self)
        if prec in HIP_PRECISIONS:
            plan = self._plan_get("enc_" + prec,
                                  lambda: _encoder_plan_x6(self.encoder, x.device, prec),
                                  self.encoder)
            feats = plan.forward(x)
            # TRG_LAYERS output (layer4.2.relu3 / relu / SPG_A3_2b.2: CAM hook), S3 layout
            # (stored times 2^features_exp per channel on the f16x3 path)
            self.features = feats[-1]
            self.features_exp = _plan_exps(plan, len(feats))[-1]
            logits = ops.wgap_s3(feats[-1], unscale_in(fw, self.features_exp), fb)
            _check_f16(self, prec, x.device)
            return logits
        _require_resnet_fp32(self.encoder)
        plan = self._plan_get("enc", lambda: _ResNetPlan(self.encoder, x.device), self.encoder)
        feats = plan.forward(x)
        self.features = feats[-1]  # == output of encoder.layer4.2.relu3 (CAM hook)
        self.features_exp = None
        return ops.wgap(feats[-1], fw, fb)


class UnetTCAM(nn.Module, _HipModelMixin):
    """dlib/unet/model.py:280-417 — frozen WSOL encoder + WGAP head, U-Net decoder,
    2-channel segmentation head whose softmax channel 1 is the TCAM CAM."""

    conv_precision: Optional[str] = None  # see STDClassifier.conv_precision

    def __init__(self, task: str = TCAM, encoder_name: str = RESNET50, encoder_depth: int = 5,
                 encoder_weights: Optional[str] = None, decoder_use_batchnorm: bool = True,
                 decoder_channels: Sequence[int] = (256, 128, 64, 32, 16),
                 decoder_attention_type: Optional[str] = None, in_channels: int = 3,
                 seg_h_out_channels: int = 2, activation=None,
                 aux_params: Optional[dict] = None, scale_in: float = 1.,
                 freeze_cl: bool = False, im_rec: bool = False, img_range: str = "tanh"):
        super().__init__()
        _check_arch(encoder_name, encoder_weights, in_channels)
        if decoder_use_batchnorm is not True or decoder_attention_type is not None:
            raise NotImplementedError("TCAM hot path uses BN decoders without attention")
        if seg_h_out_channels != 2 or activation is not None or im_rec:
            raise NotImplementedError("TCAM hot path: 2-channel seg head, no activation, "
                                      "no reconstruction head")
        self.freeze_cl = freeze_cl
        self.task = TCAM
        assert scale_in > 0.
        self.scale_in = float(scale_in)
        self.im_rec = im_rec
        self.img_range = img_range
        self.x_in = None
        self.encoder = _make_encoder(encoder_name, encoder_depth)
        self.encoder.set_task(task)
        self.decoder = UnetTCAMDecoder(self.encoder.out_channels, decoder_channels,
                                       n_blocks=encoder_depth,
                                       center=encoder_name.startswith("vgg"))
        assert aux_params is not None, "ERROR"
        aux = dict(aux_params)
        pooling_head = aux.pop("pooling_head")
        self.classification_head = POOLINGS[pooling_head](
            in_channels=self.encoder.out_channels[-1], **aux)
        self.segmentation_head = SegmentationHead(decoder_channels[-1], seg_h_out_channels, 3)
        self.reconstruction_head = None
        self.cams = None
        self.cam = None      # (B, H, W) softmax channel 1 (fused kernel output)
        self.cam_u8 = None   # (B, H, W) uint8(cam * 255) for the bbox sweep
        self.name = f"u-{encoder_name}"

    # base/model.py:124-162
    def forward(self, x: torch.Tensor, want_fcams: bool = True, argmax: bool = False):
        """Eval mode: the fused inference plan (folded BN) -> (cl_logits, fcams, None) and
        ``cams`` / ``cam`` / ``cam_u8``.  Train mode (``model.train()``): the decoder runs
        on batch statistics (running statistics updated) and ``fcams`` is differentiable
        w.r.t. the decoder and segmentation head (training.train_forward)."""
        _check_input(x)
        if self.scale_in != 1.:
            raise ValueError
        x = x.contiguous().float()
        self.x_in = x
        if self.training:
            from .training import train_forward
            cl_logits, fcams = train_forward(self, x)
            self.cams = fcams.detach()
            self.cam = self.cam_u8 = None
            return cl_logits, fcams, None
        head = self.classification_head
        fw, fb = head.fc.weight.detach().contiguous(), head.fc.bias.detach().contiguous()
        conv = self.segmentation_head[0]
        sw, sb = conv.weight.detach().contiguous(), conv.bias.detach().contiguous()
        prec = _precision(self)
        if prec in HIP_PRECISIONS:
            enc = self._plan_get("enc_" + prec,
                                 lambda: _encoder_plan_x6(self.encoder, x.device, prec),
                                 self.encoder)
            feats = enc.forward(x)
            exps = _plan_exps(enc, len(feats))
            dec = self._plan_get("dec_" + prec + exps_signature(exps),
                                 lambda: _DecoderPlanX6(self.decoder, x.device, prec, exps),
                                 self.decoder)
            cl_logits = ops.wgap_s3(feats[-1], unscale_in(fw, exps[-1]), fb)
            d = dec.forward(feats)
            sw = unscale_in(sw, dec.out_exp)
            dhw = tuple(d.shape[1:3])
            if dhw != tuple(x.shape[2:]):
                # base/model.py:148-154: fcams resized (bilinear, align_corners=True) to the
                # input size before the CAM (InceptionV3 at 299 decodes to 300).
                f0, _, _ = ops.seghead_cam_s3(d, sw, sb, want_fcams=True, want_u8=False)
                fcams, cam, u8 = ops.resize_cam(f0, tuple(x.shape[2:]),
                                                want_fcams=want_fcams, argmax=argmax)
                dhw = tuple(x.shape[2:])
            else:
                fcams, cam, u8 = ops.seghead_cam_s3(d, sw, sb, want_fcams=want_fcams,
                                                    argmax=argmax)
            _check_f16(self, prec, x.device)
        else:
            _require_resnet_fp32(self.encoder)
            enc = self._plan_get("enc", lambda: _ResNetPlan(self.encoder, x.device),
                                 self.encoder)
            dec = self._plan_get("dec", lambda: _DecoderPlan(self.decoder, x.device),
                                 self.decoder)
            feats = enc.forward(x)
            cl_logits = ops.wgap(feats[-1], fw, fb)
            d = dec.forward(feats)
            dhw = tuple(d.shape[2:])
            fcams, cam, u8 = ops.seghead_cam(d, sw, sb, want_fcams=want_fcams, argmax=argmax)
        if dhw != tuple(x.shape[2:]):
            raise NotImplementedError("seg-head resize runs on the x6 / f16x3 paths only")
        self.cams = fcams
        self.cam = cam
        self.cam_u8 = u8
        return cl_logits, fcams, None

    # base/model.py:164-215
    def train(self, mode: bool = True):
        super().train(mode)
        if self.freeze_cl:
            self.freeze_classifier()
        return self

    def freeze_classifier(self):
        assert self.freeze_cl
        for m in list(self.encoder.modules()) + list(self.classification_head.modules()):
            for p in m.parameters():
                p.requires_grad = False
            if isinstance(m, (nn.BatchNorm2d, nn.Dropout)):
                m.eval()

    def assert_cl_is_frozen(self):
        assert self.freeze_cl
        for m in list(self.encoder.modules()) + list(self.classification_head.modules()):
            for p in m.parameters():
                assert not p.requires_grad
            if isinstance(m, (nn.BatchNorm2d, nn.Dropout)):
                assert not m.training
        return True

    def free_mem(self):
        self.x_in = None
        self.cams = None
        self.cam = None
        self.cam_u8 = None

    # base/model.py:220-256 (FCAMModel = TCAMModel)
    def __str__(self):
        return "{}. Task: {}. Supp.BACK: {}. Freeze CL: {}. IMG-RECON: {}:".format(
            self.name, self.task, self.classification_head.support_background,
            self.freeze_cl, self.im_rec)

    def get_info_nbr_params(self) -> str:
        """The parameter report the reference's get_model logs right after create_model
        (process/instantiators.py:568)."""
        info = self.__str__() + " \n NBR-PARAMS: \n"
        info += "\tEncoder [{}]: {}. \n".format(self.encoder.name, count_params(self.encoder))
        info += "\tClassification head [{}]: {}. \n".format(
            self.classification_head.name, count_params(self.classification_head))
        info += "\tDecoder: {}. \n".format(count_params(self.decoder))
        info += "\tSegmentation head: {}. \n".format(count_params(self.segmentation_head))
        if self.reconstruction_head:
            info += "\tReconstruction head: {}. \n".format(
                count_params(self.reconstruction_head))
        info += "\tTotal: {}. \n".format(count_params(self))
        return info


def _make_encoder(encoder_name: str, depth: int) -> nn.Module:
    """encoders/__init__.py:50-85 (get_encoder) for the three WSOL backbones."""
    from .backbones import ENCODERS
    if encoder_name == RESNET50:
        return ResNetEncoder(depth=depth)
    enc = ENCODERS[encoder_name](depth=depth)
    enc.set_model_name(encoder_name)
    return enc


def _plan_exps(plan, n: int) -> List[Optional[torch.Tensor]]:
    """An encoder plan's per-feature activation exponents (None = all zero)."""
    e = getattr(plan, "out_exps", None)
    return list(e) if e is not None else [None] * n


def _encoder_plan_x6(enc: nn.Module, device, fmt: str = "x6"):
    from .backbones import InceptionV3Encoder, VGGEncoder, _InceptionPlanX6, _VGGPlanX6
    if isinstance(enc, ResNetEncoder):
        return _ResNetPlanX6(enc, device, fmt)
    if isinstance(enc, VGGEncoder):
        return _VGGPlanX6(enc, device, fmt)
    if isinstance(enc, InceptionV3Encoder):
        return _InceptionPlanX6(enc, device, fmt)
    raise TypeError(type(enc))


def _require_resnet_fp32(enc: nn.Module) -> None:
    if not isinstance(enc, ResNetEncoder):
        raise NotImplementedError("conv_precision='fp32' (native fp32 MFMA, NCHW) is built for "
                                  "the ResNet50 encoder only; VGG16/InceptionV3 run on 'x6'")


def _check_arch(encoder_name, encoder_weights, in_channels):
    if encoder_name not in (RESNET50, "vgg16", "inceptionv3"):
        raise NotImplementedError(f"encoder {encoder_name!r}: the TCAM family is resnet50, "
                                  f"vgg16 and inceptionv3")
    if encoder_weights not in (None,):
        raise ValueError("pretrained downloads are unavailable; load a state_dict instead")
    if in_channels != 3:
        raise NotImplementedError("in_channels != 3")


def create_model(task: str, arch: str, encoder_name: str, encoder_weights=None,
                 in_channels: int = 3, **kw) -> nn.Module:
    """dlib/__init__.py:36-75 registry restricted to the TCAM hot path."""
    if task == TCAM and arch in ("UnetTCAM",):
        return UnetTCAM(task=task, encoder_name=encoder_name, encoder_weights=encoder_weights,
                        in_channels=in_channels, **kw)
    if task == STD_CL and arch in ("STDClassifier",):
        return STDClassifier(task=task, encoder_name=encoder_name,
                             encoder_weights=encoder_weights, in_channels=in_channels, **kw)
    raise NotImplementedError(f"task={task!r} arch={arch!r} is outside the TCAM hot path")


def build_r50_tcam(classes: int = 10, seed: Optional[int] = None) -> UnetTCAM:
    """The configuration of the README TCAM runs (README.md:273-340)."""
    m = UnetTCAM(task=TCAM, encoder_name=RESNET50, encoder_depth=5, encoder_weights=None,
                 decoder_channels=(256, 128, 64, 32, 16), in_channels=3, seg_h_out_channels=2,
                 aux_params=dict(pooling_head="WGAP", classes=classes,
                                 support_background=False), freeze_cl=True)
    if seed is not None:
        from .utils.seeding import seed_module_
        seed_module_(m, seed)
    return m.eval()


def build_r50_stdcl(classes: int = 10, seed: Optional[int] = None) -> STDClassifier:
    m = STDClassifier(task=STD_CL, encoder_name=RESNET50, encoder_depth=5,
                      encoder_weights=None, in_channels=3,
                      aux_params=dict(pooling_head="WGAP", classes=classes,
                                      support_background=False))
    if seed is not None:
        from .utils.seeding import seed_module_
        seed_module_(m, seed)
    return m.eval()


def _build_tcam(encoder_name: str, classes: int, seed: Optional[int]) -> UnetTCAM:
    from .backbones import encoder_depth_channels
    depth, dec = encoder_depth_channels(encoder_name)
    m = UnetTCAM(task=TCAM, encoder_name=encoder_name, encoder_depth=depth, encoder_weights=None,
                 decoder_channels=dec, in_channels=3, seg_h_out_channels=2,
                 aux_params=dict(pooling_head="WGAP", classes=classes,
                                 support_background=False), freeze_cl=True)
    if seed is not None:
        from .utils.seeding import seed_module_
        seed_module_(m, seed)
    return m.eval()


def build_vgg16_tcam(classes: int = 10, seed: Optional[int] = None) -> UnetTCAM:
    """VGG16-TCAM (configs[3]): WSOL16 encoder depth 3, CenterBlock, decoder (256, 128, 64)."""
    return _build_tcam("vgg16", classes, seed)


def build_inceptionv3_tcam(classes: int = 10, seed: Optional[int] = None) -> UnetTCAM:
    """InceptionV3-TCAM (configs[4]): SPG InceptionV3 encoder, decoder (256, 128, 64, 32, 16)."""
    return _build_tcam("inceptionv3", classes, seed)


def build_stdcl(encoder_name: str = RESNET50, classes: int = 10,
                seed: Optional[int] = None) -> STDClassifier:
    from .backbones import encoder_depth_channels
    depth, _ = encoder_depth_channels(encoder_name)
    m = STDClassifier(task=STD_CL, encoder_name=encoder_name, encoder_depth=depth,
                      encoder_weights=None, in_channels=3,
                      aux_params=dict(pooling_head="WGAP", classes=classes,
                                      support_background=False))
    if seed is not None:
        from .utils.seeding import seed_module_
        seed_module_(m, seed)
    return m.eval()
