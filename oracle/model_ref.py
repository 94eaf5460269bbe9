"""TEST INFRASTRUCTURE ONLY: torch-CPU fp32 restatement of the TCAM model path.

Functional forward over a reference-named ``state_dict``; no module classes
from the product are used, so it checks names and math independently.
Pinned against the reference itself by tests/golden/r50_*.npz.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]
BN_EPS = 1e-5


def _bn(x: torch.Tensor, sd: SD, p: str) -> torch.Tensor:
    # nn.BatchNorm2d in eval mode (frozen classifier, base/model.py:170-194).
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], False, 0.0, BN_EPS)


def _bottleneck(x: torch.Tensor, sd: SD, p: str, stride: int) -> torch.Tensor:
    # encoders/resnet.py:214-232 (stride on conv2, torchvision V1.5).
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1"))
    out = F.relu(_bn(F.conv2d(out, sd[p + ".conv2.weight"], stride=stride, padding=1), sd,
                     p + ".bn2"))
    out = _bn(F.conv2d(out, sd[p + ".conv3.weight"]), sd, p + ".bn3")
    if p + ".downsample.0.weight" in sd:
        idn = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd,
                  p + ".downsample.1")
    else:
        idn = x
    return F.relu(out + idn)


def resnet50_wsol_features(sd: SD, x: torch.Tensor, pre: str = "encoder.") -> List[torch.Tensor]:
    """encoders/resnet.py:126-153: stages [Identity, conv1-bn1-relu, maxpool+layer1,
    layer2, layer3, layer4]; WSOL strides (layer2 2, layer3 1, layer4 1)."""
    feats = [x]
    f = F.relu(_bn(F.conv2d(x, sd[pre + "conv1.weight"], stride=2, padding=3), sd, pre + "bn1"))
    feats.append(f)
    f = F.max_pool2d(f, 3, 2, 1)
    for li, (nblk, stride) in enumerate(((3, 1), (4, 2), (6, 1), (3, 1)), start=1):
        for bi in range(nblk):
            f = _bottleneck(f, sd, f"{pre}layer{li}.{bi}", stride if bi == 0 else 1)
        feats.append(f)
    return feats


def _conv2d_relu(x: torch.Tensor, sd: SD, p: str) -> torch.Tensor:
    # base/modules.py:10-49 (conv no bias, BN, ReLU)
    return F.relu(_bn(F.conv2d(x, sd[p + ".0.weight"], padding=1), sd, p + ".1"))


def unet_tcam_decoder(sd: SD, feats: List[torch.Tensor], n_blocks: int = 5,
                      pre: str = "decoder.") -> torch.Tensor:
    """unet/decoder.py:267-283 + DecoderBlock.forward 41-57."""
    fs = feats[1:][::-1]
    x, skips = fs[0], fs[1:]
    if pre + "center.0.0.weight" in sd:
        x = _conv2d_relu(x, sd, pre + "center.0")
        x = _conv2d_relu(x, sd, pre + "center.1")
    for i in range(n_blocks):
        skip = skips[i] if i < len(skips) else None
        x = F.interpolate(x, scale_factor=2, mode="nearest")
        if skip is not None:
            if x.shape[2:] != skip.shape[2:]:
                x = F.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=True)
            x = torch.cat([x, skip], dim=1)
        x = _conv2d_relu(x, sd, f"{pre}blocks.{i}.conv1")
        x = _conv2d_relu(x, sd, f"{pre}blocks.{i}.conv2")
    return x


def wgap(sd: SD, f: torch.Tensor, pre: str = "classification_head.") -> torch.Tensor:
    # poolings/core.py:109-115
    return F.linear(F.adaptive_avg_pool2d(f, 1).flatten(1), sd[pre + "fc.weight"],
                    sd[pre + "fc.bias"])


# encoders/vgg.py:47-58 ('WSOL16') — conv3x3 (bias) + ReLU, 'M' = MaxPool2d(2, 2)
WSOL16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, 512, 512, 512]


def vgg16_wsol_features(sd: SD, x: torch.Tensor, pre: str = "encoder.") -> List[torch.Tensor]:
    """VGGEncoder.forward (encoders/vgg.py:86-106): stages split at each max-pool,
    conv6 512->1024 + ReLU closing the last one; depth 3 -> 4 features."""
    feats, idx, f = [], 0, x
    for v in WSOL16:
        if v == "M":
            feats.append(f)
            f = F.max_pool2d(f, 2, 2)
            idx += 1
        else:
            f = F.relu(F.conv2d(f, sd[f"{pre}features.{idx}.weight"],
                                sd[f"{pre}features.{idx}.bias"], padding=1))
            idx += 2
    f = F.relu(F.conv2d(f, sd[pre + "conv6.weight"], sd[pre + "conv6.bias"], padding=1))
    feats.append(f)
    return feats


def _bconv(x: torch.Tensor, sd: SD, p: str, stride=1, padding=0) -> torch.Tensor:
    # BasicConv2d (wsol_backbones/inceptionv3.py:52-64): conv, BN(eps 1e-3), ReLU
    y = F.conv2d(x, sd[p + ".conv.weight"], stride=stride, padding=padding)
    y = F.batch_norm(y, sd[p + ".bn.running_mean"], sd[p + ".bn.running_var"],
                     sd[p + ".bn.weight"], sd[p + ".bn.bias"], False, 0.0, 1e-3)
    return F.relu(y)


def _inc_a(x, sd, p):
    # InceptionA.forward (inceptionv3.py:81-96); 3x3 paddings already 1
    b1 = _bconv(x, sd, p + ".branch1x1")
    b5 = _bconv(_bconv(x, sd, p + ".branch5x5_1"), sd, p + ".branch5x5_2", padding=2)
    d = _bconv(x, sd, p + ".branch3x3dbl_1")
    d = _bconv(d, sd, p + ".branch3x3dbl_2", padding=1)
    d = _bconv(d, sd, p + ".branch3x3dbl_3", padding=1)
    bp = _bconv(F.avg_pool2d(x, 3, 1, 1), sd, p + ".branch_pool")
    return torch.cat([b1, b5, d, bp], 1)


def _inc_b(x, sd, p, stride=1):
    # InceptionB.forward (inceptionv3.py:114-125), SPG Mixed_6a: k3 s1 p1
    b3 = _bconv(x, sd, p + ".branch3x3", stride=stride, padding=1)
    d = _bconv(x, sd, p + ".branch3x3dbl_1")
    d = _bconv(d, sd, p + ".branch3x3dbl_2", padding=1)
    d = _bconv(d, sd, p + ".branch3x3dbl_3", stride=stride, padding=1)
    bp = F.max_pool2d(x, 3, stride, 1)
    return torch.cat([b3, d, bp], 1)


def _inc_c(x, sd, p):
    # InceptionC.forward (inceptionv3.py:148-170)
    b1 = _bconv(x, sd, p + ".branch1x1")
    b7 = _bconv(x, sd, p + ".branch7x7_1")
    b7 = _bconv(b7, sd, p + ".branch7x7_2", padding=(0, 3))
    b7 = _bconv(b7, sd, p + ".branch7x7_3", padding=(3, 0))
    d = _bconv(x, sd, p + ".branch7x7dbl_1")
    d = _bconv(d, sd, p + ".branch7x7dbl_2", padding=(3, 0))
    d = _bconv(d, sd, p + ".branch7x7dbl_3", padding=(0, 3))
    d = _bconv(d, sd, p + ".branch7x7dbl_4", padding=(3, 0))
    d = _bconv(d, sd, p + ".branch7x7dbl_5", padding=(0, 3))
    bp = _bconv(F.avg_pool2d(x, 3, 1, 1), sd, p + ".branch_pool")
    return torch.cat([b1, b7, d, bp], 1)


def inceptionv3_spg_features(sd: SD, x: torch.Tensor,
                             pre: str = "encoder.") -> List[torch.Tensor]:
    """InceptionV3Encoder.forward (encoders/inceptionv3.py:76-100) with the corrected
    paddings (every 3x3 conv and MaxPool2d padded 1, inceptionv3.py:61-67) over
    wsol_backbones/inceptionv3.py:245-290; dropout is identity in eval."""
    feats = [x]
    f = _bconv(x, sd, pre + "Conv2d_1a_3x3", stride=2, padding=1)
    f = _bconv(f, sd, pre + "Conv2d_2a_3x3", padding=1)
    f = _bconv(f, sd, pre + "Conv2d_2b_3x3", padding=1)
    feats.append(f)
    f = F.max_pool2d(f, 3, 2, 1, ceil_mode=True)
    f = _bconv(f, sd, pre + "Conv2d_3b_1x1")
    feats.append(f)
    f = _bconv(f, sd, pre + "Conv2d_4a_3x3", padding=1)
    f = F.max_pool2d(f, 3, 2, 1, ceil_mode=True)
    f = _inc_a(f, sd, pre + "Mixed_5b")
    f = _inc_a(f, sd, pre + "Mixed_5c")
    feats.append(f)
    f = _inc_a(f, sd, pre + "Mixed_5d")
    f = _inc_b(f, sd, pre + "Mixed_6a")
    for b in ("6b", "6c", "6d", "6e"):
        f = _inc_c(f, sd, pre + "Mixed_" + b)
    feats.append(f)
    f = F.relu(F.conv2d(f, sd[pre + "SPG_A3_1b.1.weight"], sd[pre + "SPG_A3_1b.1.bias"],
                        padding=1))
    f = F.relu(F.conv2d(f, sd[pre + "SPG_A3_2b.1.weight"], sd[pre + "SPG_A3_2b.1.bias"],
                        padding=1))
    feats.append(f)
    return feats


def encoder_features(sd: SD, x: torch.Tensor) -> List[torch.Tensor]:
    if "encoder.conv6.weight" in sd:
        return vgg16_wsol_features(sd, x)
    if "encoder.Mixed_5b.branch1x1.conv.weight" in sd:
        return inceptionv3_spg_features(sd, x)
    return resnet50_wsol_features(sd, x)


@torch.no_grad()
def tcam_forward(sd: SD, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, List[torch.Tensor]]:
    """FCAMModel.forward (base/model.py:124-162): (cl_logits, fcams, features)."""
    feats = encoder_features(sd, x)
    logits = wgap(sd, feats[-1])
    n_blocks = sum(1 for k in sd if k.startswith("decoder.blocks.") and
                   k.endswith(".conv1.0.weight"))
    d = unet_tcam_decoder(sd, feats, n_blocks=n_blocks)
    fcams = F.conv2d(d, sd["segmentation_head.0.weight"], sd["segmentation_head.0.bias"],
                     padding=1)
    if fcams.shape[2:] != x.shape[2:]:
        fcams = F.interpolate(fcams, size=x.shape[2:], mode="bilinear", align_corners=True)
    return logits, fcams, feats


def segmentation_cam(fcams: torch.Tensor, argmax: bool = False) -> torch.Tensor:
    """SegmentationCam.compute_cams (cams/builtincam.py:201-225), batched; then
    nan_to_num (inference_wsol.py:323)."""
    if argmax:
        cam = torch.argmax(fcams, dim=1).float()
    else:
        cam = torch.softmax(fcams, dim=1)[:, 1]
    return torch.nan_to_num(cam, nan=0.0, posinf=1., neginf=0.0)


def cam_to_scoremap(cam: torch.Tensor, size) -> np.ndarray:
    """inference_wsol.py:342-346 + t2n (utils/tools.py:253-254): bilinear
    (align_corners=False) to image size, float64 numpy."""
    out = F.interpolate(cam[:, None], size, mode="bilinear", align_corners=False)[:, 0]
    return out.numpy().astype(float)


def quantize_u8(scoremap: np.ndarray) -> np.ndarray:
    """wsol_metrics.py:153: (scoremap * 255).astype(np.uint8)."""
    return (scoremap * 255).astype(np.uint8)


@torch.no_grad()
def stdcl_forward(sd: SD, x: torch.Tensor):
    """STDClModel.forward (base/model.py:20-34) with the layer4 output kept (the
    CAM hook encoder.layer4.2.relu3, constants.py:276-285)."""
    feats = resnet50_wsol_features(sd, x)
    return wgap(sd, feats[-1]), feats[-1]


@torch.no_grad()
def std_cam(sd: SD, A: torch.Tensor, class_idx: int, size) -> Tuple[torch.Tensor, np.ndarray]:
    """CAM (cams/cam.py:31-99, core.py:162-193, normalized=True), nan_to_num,
    then bilinear to size.  A: (1, C, h, w) or (C, h, w)."""
    if A.dim() == 4:
        A = A[0]
    w = sd["classification_head.fc.weight"][class_idx][:, None, None]
    low = torch.nansum(w * A, dim=0)
    low = low - low.min()
    low = low / low.max()
    low = torch.nan_to_num(low, nan=0.0, posinf=1., neginf=0.0)
    return low, cam_to_scoremap(low[None], size)[0]


def re_normalize_cam(cam: torch.Tensor, h: float) -> torch.Tensor:
    # datasets/wsol_loader.py:630-635
    e = torch.exp((cam + 1e-6) * h)
    e = e / e.max()
    return torch.nan_to_num(e, nan=0.0, posinf=1., neginf=0.0)


def temporal_max(cams: List[torch.Tensor], t: float = 0.0, sl_tc_knn: int = 1) -> torch.Tensor:
    """datasets/wsol_loader.py:591-601: std_cam = max over temporal frames of stage-1
    CAMs, each re-normalised first when ``_is_tmp and sl_tc_knn_t > 0`` (:571, 594;
    ``_is_tmp = sl_tc_knn > 0``)."""
    std = None
    for c in cams:
        if sl_tc_knn > 0 and t > 0:
            c = re_normalize_cam(c, t)
        std = c if std is None else torch.maximum(std, c)
    return std


def knn_frames(lframes: List[str], frame: str, k: int, mode: str) -> List[str]:
    """The temporal frames of one item: datasets/wsol_loader.py:544-569 with
    _get_lef_knn / _get_right_knn (447-458) — left + [frame] + right."""
    idx = lframes.index(frame)
    n = len(lframes)
    left, right = [], []
    if mode in ("before", "before-after"):
        left = lframes[max(0, idx - k): idx]
    if mode in ("after", "before-after"):
        right = lframes[min(idx + 1, n - 1): min(idx + k + 1, n)]
    return left + [frame] + right
