"""VGG16 (WSOL16) and InceptionV3 (SPG) encoders of the TCAM model family, with their
HIP executors on the x6 path (S3 activations, ``tcam_conv2d_x6``).

Module and parameter names reproduce the reference so strict ``state_dict`` loads of
reference checkpoints work and the CAM hooks resolve:

* ``VGGEncoder``          dlib/encoders/vgg.py:61-161 (torchvision VGG's ``features`` /
                          ``avgpool``; ``conv6`` 512->1024 + ``relu``; ``full_features``
                          re-registers the same modules, so its keys repeat in the
                          state_dict exactly as in the reference).
* ``InceptionV3Encoder``  dlib/encoders/inceptionv3.py:50-100 over
                          dlib/encoders/wsol_backbones/inceptionv3.py:52-304 (SPG variant:
                          stride-1 Mixed_6a, SPG_A3_1b/2b 1024-channel 3x3 heads, every
                          3x3 conv padded 1, every MaxPool2d padded 1, BN eps 1e-3).

Each concatenating block (InceptionA/B/C) has its branches write straight into their
channel slice of the block output (fused ``torch.cat``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import os

import torch
import torch.nn as nn

from . import ops
from .ops import ConvSrc

VGG16 = "vgg16"
INCEPTIONV3 = "inceptionv3"

# encoders/vgg.py:47-58
WSOL16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, 512, 512, 512]


# ------------------------------------------------------------------- VGG
def make_layers(cfg) -> nn.Sequential:
    """encoders/vgg.py:146-161 (conv3x3 pad 1 + ReLU; 'M' = MaxPool2d(2, 2))."""
    layers: List[nn.Module] = []
    cin = 3
    for v in cfg:
        if v == "M1":
            layers.append(nn.MaxPool2d(kernel_size=3, stride=2, padding=1))
        elif v == "M2":
            layers.append(nn.MaxPool2d(kernel_size=3, stride=1, padding=1))
        elif v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=False)]
            cin = v
    return nn.Sequential(*layers)


class VGGEncoder(nn.Module):
    """encoders/vgg.py:61-110 with the 'vgg16' params (out_channels (64, 128, 256, 1024),
    WSOL16, depth 3, vgg.py:234-242).  torchvision's VGG registers ``features`` then
    ``avgpool`` (no state); the classifier is deleted (vgg.py:80)."""

    def __init__(self, out_channels=(64, 128, 256, 1024), config=WSOL16, depth: int = 3):
        super().__init__()
        self.features = make_layers(config)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.conv6 = nn.Conv2d(512, 1024, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=False)
        self.full_features = nn.Sequential(*list(self.features.children()), self.conv6,
                                           self.relu)
        self._out_channels = tuple(out_channels)
        self._depth = depth
        self._in_channels = 3
        self.name = "null-name"
        self.task = None

    @property
    def out_channels(self):
        return self._out_channels[: self._depth + 1]

    def set_task(self, task: str):
        self.task = task

    def set_model_name(self, name: str):
        self.name = name


    def super_load_state_dict(self, state_dict, **kw):
        """encoders/vgg.py:124-125 (checkpoint loads, instantiators.py:664-667)."""
        return super().load_state_dict(state_dict, **kw)

class _VGGPlanX6:
    """Folded weights + the S3 forward of the WSOL16 encoder.  Stages split at the
    max-pools (vgg.py:86-95): [64@H, 128@H/2, 256@H/4, 1024@H/8]."""

    def __init__(self, enc: VGGEncoder, device, fmt: str = "x6"):
        from .models import FoldedConv
        self.fmt = fmt
        self.ops: List = []   # ("conv", FoldedConv) | ("pool", None)
        first = True
        for m in list(enc.full_features.children()):
            if isinstance(m, nn.Conv2d):
                self.ops.append(("conv", FoldedConv([(m, None)], device, fmt,
                                                    cin_pad=8 if first else None)))
                first = False
            elif isinstance(m, nn.MaxPool2d):
                self.ops.append(("pool", (m.kernel_size, m.stride, m.padding)))

    def forward(self, x: torch.Tensor, keep_all: bool = True) -> List[torch.Tensor]:
        f = ops.s3_from_nchw(x, 8, self.fmt)
        feats = []
        for kind, c in self.ops:
            if kind == "pool":
                feats.append(f)
                k, st, pd = c
                f = ops.pool2d_s3(f, k, st, pd, "max")
            else:
                H, W = f.shape[1], f.shape[2]
                f = ops.conv2d_x6([ConvSrc(f)], c.wt, c.bias, c.cout, H, W, 3, 1, True,
                                  wscale=c.wscale)
        feats.append(f)
        return feats if keep_all else feats[-1:]


# ------------------------------------------------------------- Inception
class BasicConv2d(nn.Module):
    """wsol_backbones/inceptionv3.py:52-64: conv (no bias) + BN(eps 1e-3) + ReLU."""

    def __init__(self, cin: int, cout: int, kernel_size, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size, bias=False, **kw)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)


class InceptionA(nn.Module):
    """inceptionv3.py:67-96."""

    def __init__(self, cin: int, pool_features: int):
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 64, 1)
        self.branch5x5_1 = BasicConv2d(cin, 48, 1)
        self.branch5x5_2 = BasicConv2d(48, 64, 5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, padding=1)
        self.branch_pool = BasicConv2d(cin, pool_features, 1)


class InceptionB(nn.Module):
    """inceptionv3.py:99-125 (SPG: Mixed_6a with kernel 3, stride 1, padding 1)."""

    def __init__(self, cin: int, kernel_size: int = 3, stride: int = 2, padding: int = 0):
        super().__init__()
        self.branch3x3 = BasicConv2d(cin, 384, kernel_size, stride=stride, padding=padding)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, stride=stride, padding=padding)
        self.stride = stride


class InceptionC(nn.Module):
    """inceptionv3.py:128-170."""

    def __init__(self, cin: int, channels_7x7: int):
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(cin, 192, 1)
        self.branch7x7_1 = BasicConv2d(cin, c7, 1)
        self.branch7x7_2 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, (7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(cin, c7, 1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, (1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(cin, 192, 1)


class InceptionV3Encoder(nn.Module):
    """encoders/inceptionv3.py:50-100 over wsol_backbones/inceptionv3.py:245-290 with the
    registry params (stage_idxs (3, 5, 9, 15), out_channels (3, 64, 80, 288, 768, 1024),
    inceptionv3.py:119-129).  Registration order (hence state_dict order) follows the
    reference: the named blocks, then ``features`` (which repeats them), ``avgpool``."""

    def __init__(self, stage_idxs=(3, 5, 9, 15), out_channels=(3, 64, 80, 288, 768, 1024),
                 depth: int = 5):
        super().__init__()
        self.large_feature_map = True
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, 3, stride=2, padding=1)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, 3, stride=1, padding=0)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, 3, stride=1, padding=1)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, 1, stride=1, padding=0)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, 3, stride=1, padding=0)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288, kernel_size=3, stride=1, padding=1)
        self.Mixed_6b = InceptionC(768, channels_7x7=128)
        self.Mixed_6c = InceptionC(768, channels_7x7=160)
        self.Mixed_6d = InceptionC(768, channels_7x7=160)
        self.Mixed_6e = InceptionC(768, channels_7x7=192)
        self.SPG_A3_1b = nn.Sequential(nn.Dropout(p=0.5), nn.Conv2d(768, 1024, 3, padding=1),
                                       nn.ReLU(inplace=False))
        self.SPG_A3_2b = nn.Sequential(nn.Dropout(p=0.5), nn.Conv2d(1024, 1024, 3, padding=1),
                                       nn.ReLU(inplace=False))
        self.features = nn.Sequential(
            self.Conv2d_1a_3x3, self.Conv2d_2a_3x3, self.Conv2d_2b_3x3,
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1, ceil_mode=True),
            self.Conv2d_3b_1x1, self.Conv2d_4a_3x3,
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1, ceil_mode=True),
            self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b,
            self.Mixed_6c, self.Mixed_6d, self.Mixed_6e, self.SPG_A3_1b, self.SPG_A3_2b)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.last_linear = None
        # "correct paddings" (encoders/inceptionv3.py:61-67)
        for m in self.modules():
            if isinstance(m, nn.Conv2d) and m.kernel_size == (3, 3):
                m.padding = (1, 1)
            if isinstance(m, nn.MaxPool2d):
                m.padding = (1, 1)
        del self.last_linear
        self._stage_idxs = tuple(stage_idxs)
        self._out_channels = tuple(out_channels)
        self._depth = depth
        self._in_channels = 3
        self.name = "null-name"
        self.task = None

    @property
    def out_channels(self):
        return self._out_channels[: self._depth + 1]

    def set_task(self, task: str):
        self.task = task

    def set_model_name(self, name: str):
        self.name = name


    def super_load_state_dict(self, state_dict, **kw):
        """encoders/inceptionv3.py:108-109 (checkpoint loads, instantiators.py:664-667)."""
        return super().load_state_dict(state_dict, **kw)

def _conv_out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


class _BC:
    """A folded BasicConv2d (or SPG conv + bias) with its geometry."""

    def __init__(self, conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], device, cin_pad=None,
                 fmt: str = "x6"):
        from .models import FoldedConv
        self.f = FoldedConv([(conv, bn)], device, fmt, cin_pad=cin_pad)
        self.k = tuple(conv.kernel_size)
        self.p = tuple(conv.padding)
        self.s = conv.stride[0]
        self.cout = conv.out_channels

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                 coff: int = 0) -> torch.Tensor:
        H, W = x.shape[1], x.shape[2]
        Ho = _conv_out(H, self.k[0], self.s, self.p[0])
        Wo = _conv_out(W, self.k[1], self.s, self.p[1])
        return ops.conv2d_x6([ConvSrc(x, self.s)], self.f.wt, self.f.bias, self.cout, Ho, Wo,
                             self.k, self.p, True, out=out, out_coff=coff, wscale=self.f.wscale)


    def member(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
               coff: int = 0) -> "ops.ConvMember":
        """This conv as one member of a grouped launch (ops.conv2d_group)."""
        H, W = x.shape[1], x.shape[2]
        Ho = _conv_out(H, self.k[0], self.s, self.p[0])
        Wo = _conv_out(W, self.k[1], self.s, self.p[1])
        return ops.ConvMember(ConvSrc(x, self.s), self.f.wt, self.f.bias, self.cout, Ho, Wo,
                              self.k, self.p, True, wscale=self.f.wscale, out=out,
                              out_coff=coff)


def _bc(m: BasicConv2d, device, cin_pad=None, fmt: str = "x6") -> _BC:
    return _BC(m.conv, m.bn, device, cin_pad, fmt)


class _BCGroup:
    """Branch-parallel 1x1 BasicConv2d's reading one input (an Inception block's
    branch1x1 / branch5x5_1 / branch3x3dbl_1, inceptionv3.py:86-96, or branch1x1 /
    branch7x7_1 / branch7x7dbl_1, :150-170) as ONE grouped launch: the folded weights are
    stacked along the output channels and each member's channels go to its own tensor
    (tcam_conv2d_x6_multi)."""

    def __init__(self, members: Sequence[BasicConv2d], device, fmt: str = "x6"):
        from .models import fold_conv_bn
        ws, bs = [], []
        for m in members:
            assert tuple(m.conv.kernel_size) == (1, 1) and m.conv.stride[0] == 1
            w, b = fold_conv_bn(m.conv, m.bn)
            ws.append(w.reshape(m.conv.weight.shape).float().to(device))
            bs.append(b.float().to(device))
        self.wscale = None
        if fmt == "f16x3":
            self.wt, self.wscale = ops.pack_conv_weight_f16([torch.cat(ws, 0)])
        else:
            self.wt = ops.pack_conv_weight_x6([torch.cat(ws, 0)])
        self.bias = torch.cat(bs).contiguous()
        self.couts = [m.conv.out_channels for m in members]

    def __call__(self, x: torch.Tensor, outs) -> List[torch.Tensor]:
        B, H, W, _ = ops.s3_dims(x)
        return ops.conv2d_x6_multi([ConvSrc(x, 1)], self.wt, self.bias, self.couts, H, W, 1, 0,
                                   True, outs, wscale=self.wscale)


class _InceptionPlanX6:
    """The SPG InceptionV3 encoder forward on S3 (stages of encoders/inceptionv3.py:76-84:
    [x, 64@S/2, 80, 288, 768, 1024])."""

    def __init__(self, enc: InceptionV3Encoder, device, fmt: str = "x6"):
        self.fmt = fmt
        bc = lambda m, **kw: _bc(m, device, fmt=fmt, **kw)  # noqa: E731
        self.c1a = bc(enc.Conv2d_1a_3x3, cin_pad=8)
        self.c2a = bc(enc.Conv2d_2a_3x3)
        self.c2b = bc(enc.Conv2d_2b_3x3)
        self.c3b = bc(enc.Conv2d_3b_1x1)
        self.c4a = bc(enc.Conv2d_4a_3x3)
        self.pools = [m for m in enc.features if isinstance(m, nn.MaxPool2d)]
        self.a = [self._plan_a(m, device, fmt)
                  for m in (enc.Mixed_5b, enc.Mixed_5c, enc.Mixed_5d)]
        m = enc.Mixed_6a
        self.b = dict(b3=bc(m.branch3x3), d1=bc(m.branch3x3dbl_1), d2=bc(m.branch3x3dbl_2),
                      d3=bc(m.branch3x3dbl_3), stride=m.stride)
        self.c = [self._plan_c(m, device, fmt)
                  for m in (enc.Mixed_6b, enc.Mixed_6c, enc.Mixed_6d, enc.Mixed_6e)]
        self.spg1 = _BC(enc.SPG_A3_1b[1], None, device, fmt=fmt)
        self.spg2 = _BC(enc.SPG_A3_2b[1], None, device, fmt=fmt)

    # TCAM_INCEPTION_NOGROUP=1: the branch-parallel 1x1 convs as separate launches (A/B)
    GROUP = os.environ.get("TCAM_INCEPTION_NOGROUP", "0") != "1"
    # TCAM_INCEPTION_STAGES=0: each block's independent branch convs as separate launches
    # instead of one heterogeneous grouped launch per stage (A/B); TCAM_INCEPTION_STAGE_TILE:
    # the grouped launches' tile (-1 = automatic; 18, the 128x64 register-staged tile, measured
    # best: profiles/round4_inception_stage_ab.jsonl)
    STAGES = os.environ.get("TCAM_INCEPTION_STAGES", "1") != "0"
    STAGE_TILE = int(os.environ.get("TCAM_INCEPTION_STAGE_TILE", "18"))

    @classmethod
    def _plan_a(cls, m: InceptionA, device, fmt: str):
        bc = lambda mm: _bc(mm, device, fmt=fmt)  # noqa: E731
        p = dict(b5_2=bc(m.branch5x5_2), d2=bc(m.branch3x3dbl_2), d3=bc(m.branch3x3dbl_3),
                 bp=bc(m.branch_pool))
        if cls.GROUP and fmt != "amp":
            p["g1"] = _BCGroup([m.branch1x1, m.branch5x5_1, m.branch3x3dbl_1], device, fmt)
        else:
            p.update(b1=bc(m.branch1x1), b5_1=bc(m.branch5x5_1), d1=bc(m.branch3x3dbl_1))
        return p

    @classmethod
    def _plan_c(cls, m: InceptionC, device, fmt: str):
        first = ["branch1x1", "branch7x7_1", "branch7x7dbl_1"]
        names = ["branch7x7_2", "branch7x7_3", "branch7x7dbl_2", "branch7x7dbl_3",
                 "branch7x7dbl_4", "branch7x7dbl_5", "branch_pool"]
        p = {n: _bc(getattr(m, n), device, fmt=fmt) for n in names}
        if cls.GROUP and fmt != "amp":   # (grouped launches: x6 / f16x3)
            p["g1"] = _BCGroup([getattr(m, n) for n in first], device, fmt)
        else:
            p.update({n: _bc(getattr(m, n), device, fmt=fmt) for n in first})
        return p

    @staticmethod
    def _maxpool(x, m: nn.MaxPool2d):
        one = lambda v: v[0] if isinstance(v, (tuple, list)) else v  # noqa: E731
        return ops.pool2d_s3(x, m.kernel_size, one(m.stride), one(m.padding), "max",
                             ceil_mode=m.ceil_mode)

    def _stage(self, calls):
        """Independent branch convs [(bc, input, out, coff)] of one block: ONE grouped
        launch (ops.conv2d_group) on the x6 / f16x3 formats, else one launch each.
        Returns the outputs."""
        if self.STAGES and self.fmt != "amp" and len(calls) > 1:
            return ops.conv2d_group([bc.member(x, o, c) for bc, x, o, c in calls],
                                    self.STAGE_TILE)
        return [bc(x, o, c) for bc, x, o, c in calls]

    def _block_a(self, x, p):
        """inceptionv3.py:80-94; stages: the three 1x1 convs on x (grouped along Cout), the
        avg pool, then branch5x5_2 | branch3x3dbl_2 | branch_pool, then branch3x3dbl_3."""
        B, H, W, _ = ops.s3_dims(x)
        cout = 64 + 64 + 96 + p["bp"].cout
        out = ops.act_empty(x, B, H, W, cout)
        if "g1" in p:
            _, t5, td = p["g1"](x, [(out, 0), None, None])
        else:
            p["b1"](x, out, 0)
            t5, td = p["b5_1"](x), p["d1"](x)
        pooled = ops.pool2d_s3(x, 3, 1, 1, "avg")
        _, d2, _ = self._stage([(p["b5_2"], t5, out, 64), (p["d2"], td, None, 0),
                                (p["bp"], pooled, out, 224)])
        p["d3"](d2, out, 128)
        return out

    def _block_b(self, x, p):
        """inceptionv3.py:109-120: branch3x3 | branch3x3dbl_1 on x, then the dbl chain."""
        B, H, W, Cin = ops.s3_dims(x)
        st = p["stride"]
        b3 = p["b3"]
        Ho = _conv_out(H, b3.k[0], st, b3.p[0])
        Wo = _conv_out(W, b3.k[1], st, b3.p[1])
        out = ops.act_empty(x, B, Ho, Wo, 384 + 96 + Cin)
        _, d1 = self._stage([(b3, x, out, 0), (p["d1"], x, None, 0)])
        p["d3"](p["d2"](d1), out, 384)
        ops.pool2d_s3(x, 3, st, 1, "max", out=out, out_coff=480)   # inceptionv3.py:120-121
        return out

    def _block_c(self, x, p):
        """inceptionv3.py:141-158; stages: the three 1x1 convs on x, the avg pool, then
        branch7x7_2 | branch7x7dbl_2 | branch_pool, branch7x7_3 | branch7x7dbl_3, then
        branch7x7dbl_4, branch7x7dbl_5."""
        B, H, W, _ = ops.s3_dims(x)
        out = ops.act_empty(x, B, H, W, 768)
        if "g1" in p:
            _, t7, d = p["g1"](x, [(out, 0), None, None])
        else:
            p["branch1x1"](x, out, 0)
            t7, d = p["branch7x7_1"](x), p["branch7x7dbl_1"](x)
        pooled = ops.pool2d_s3(x, 3, 1, 1, "avg")
        t7, d, _ = self._stage([(p["branch7x7_2"], t7, None, 0), (p["branch7x7dbl_2"], d, None, 0),
                                (p["branch_pool"], pooled, out, 576)])
        _, d = self._stage([(p["branch7x7_3"], t7, out, 192), (p["branch7x7dbl_3"], d, None, 0)])
        d = p["branch7x7dbl_4"](d)
        p["branch7x7dbl_5"](d, out, 384)
        return out

    def forward(self, x: torch.Tensor, keep_all: bool = True) -> List[torch.Tensor]:
        feats = [x]
        f = ops.s3_from_nchw(x, 8, self.fmt)
        f = self.c2b(self.c2a(self.c1a(f)))
        feats.append(f)                                   # 64 @ S/2      features[:3]
        f = self.c3b(self._maxpool(f, self.pools[0]))
        feats.append(f)                                   # 80            features[3:5]
        f = self._maxpool(self.c4a(f), self.pools[1])
        f = self._block_a(f, self.a[0])
        f = self._block_a(f, self.a[1])
        feats.append(f)                                   # 288           features[5:9]
        f = self._block_a(f, self.a[2])
        f = self._block_b(f, self.b)
        for p in self.c:
            f = self._block_c(f, p)
        feats.append(f)                                   # 768           features[9:15]
        f = self.spg2(self.spg1(f))                       # dropout = identity in eval
        feats.append(f)                                   # 1024          features[15:]
        return feats if keep_all else feats[-1:]


ENCODERS = {VGG16: VGGEncoder, INCEPTIONV3: InceptionV3Encoder}


def encoder_depth_channels(encoder_name: str):
    """process/instantiators.py:46-55 (get_encoder_d_c)."""
    if encoder_name == VGG16:
        return 3, (256, 128, 64)
    return 5, (256, 128, 64, 32, 16)
