"""Generate the golden vectors in tests/golden/ from the REFERENCE code.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py

What is imported from the reference (read-only, not copied):
  dlib/encoders/resnet.py (ResNetEncoder, Bottleneck, resnet_encoders),
  dlib/unet/{model,decoder}.py (UnetTCAM, UnetTCAMDecoder, DecoderBlock),
  dlib/base/{model,heads,modules}.py, dlib/poolings/core.py (WGAP),
  dlib/stdcl/classifier.py (STDClassifier), dlib/cams/{builtincam,cam,core}.py
  (SegmentationCam, CAM), dlib/learning/inference_wsol.py semantics for the
  per-frame CAM (softmax ch-1, bilinear to image size, t2n float64).

Third-party modules absent from this image are stubbed:
  pynvml / cv2 (imported but not exercised by the model path),
  pretrainedmodels.pretrained_settings (a dict only read for URLs), and
  torchvision 0.12 ``ResNet`` whose ``_make_layer`` (the only method the WSOL
  encoder inherits) is restated below from its published algorithm.  Parity of
  that restatement is structural: the strict ``state_dict`` key/shape match
  against our own modules is asserted here.

Outputs (small, committed): ``r50_tcam.npz`` and ``r50_stdcl.npz``.
"""
from __future__ import annotations

import os
import sys
sys.dont_write_bytecode = True  # nothing may be written under /root/reference
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from tcam_wsol_video_amd.utils.seeding import seeded_state_dict  # noqa: E402


def _install_stubs():
    # -- third-party stubs ---------------------------------------------------
    for name in ("pynvml", "pynvml.smi", "cv2"):
        m = types.ModuleType(name)
        sys.modules[name] = m
    sys.modules["pynvml.smi"].nvidia_smi = object
    sys.modules["cv2"].__version__ = "4.5.5"

    class _AnyDict(dict):
        def __missing__(self, k):
            v = {}
            self[k] = v
            return v

    pm = types.ModuleType("pretrainedmodels")
    pmm = types.ModuleType("pretrainedmodels.models")
    pmt = types.ModuleType("pretrainedmodels.models.torchvision_models")
    pmt.pretrained_settings = _AnyDict()
    sys.modules["pretrainedmodels"] = pm
    sys.modules["pretrainedmodels.models"] = pmm
    sys.modules["pretrainedmodels.models.torchvision_models"] = pmt

    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvr = types.ModuleType("torchvision.models.resnet")
    tvv = types.ModuleType("torchvision.models.vgg")

    class ResNet(nn.Module):
        """torchvision==0.12 ResNet: only ``_make_layer`` is inherited by the
        WSOL encoder (resnet.py:57-133 calls nn.Module.__init__ directly)."""

        def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
            norm_layer = self._norm_layer
            downsample = None
            previous_dilation = self.dilation
            if dilate:
                self.dilation *= stride
                stride = 1
            if stride != 1 or self.inplanes != planes * block.expansion:
                downsample = nn.Sequential(
                    nn.Conv2d(self.inplanes, planes * block.expansion, 1,
                              stride=stride, bias=False),
                    norm_layer(planes * block.expansion))
            layers = [block(self.inplanes, planes, stride, downsample,
                            self.groups, self.base_width, previous_dilation,
                            norm_layer)]
            self.inplanes = planes * block.expansion
            for _ in range(1, blocks):
                layers.append(block(self.inplanes, planes, groups=self.groups,
                                    base_width=self.base_width,
                                    dilation=self.dilation,
                                    norm_layer=norm_layer))
            return nn.Sequential(*layers)

    class VGG(nn.Module):
        """torchvision==0.12 VGG.__init__ (the WSOL VGGEncoder inherits only the module
        layout: ``features``, ``avgpool``, ``classifier`` — deleted by vgg.py:80)."""

        def __init__(self, features, num_classes=1000, init_weights=True, dropout=0.5):
            super().__init__()
            self.features = features
            self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
            self.classifier = nn.Sequential(
                nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(p=dropout),
                nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(p=dropout),
                nn.Linear(4096, num_classes))

    tvv.VGG = VGG
    tvr.ResNet = ResNet
    tv.models = tvm
    tvm.resnet = tvr
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    sys.modules["torchvision.models.resnet"] = tvr
    sys.modules["torchvision.models.vgg"] = tvv

    # -- reference package stubs: skip the heavy package __init__s ----------
    sys.path.insert(0, REF)
    for pkg in ("dlib", "dlib.encoders", "dlib.cams"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, *pkg.split("."))]
        sys.modules[pkg] = m

    import importlib
    resnet = importlib.import_module("dlib.encoders.resnet")

    vgg = importlib.import_module("dlib.encoders.vgg")
    inc = importlib.import_module("dlib.encoders.inceptionv3")
    registry = dict(resnet.resnet_encoders)
    registry.update(vgg.vgg_encoders)
    registry.update(inc.inceptionv3_encoders)

    def get_encoder(task, name, in_channels=3, depth=5, weights=None):
        # encoders/__init__.py:50-85 with weights=None (no network here).
        assert weights is None
        enc = registry[name]
        encoder = enc["encoder"](**dict(enc["params"], depth=depth))
        encoder.set_in_channels(in_channels)
        encoder.set_model_name(name)
        encoder.set_task(task)
        return encoder

    sys.modules["dlib.encoders"].get_encoder = get_encoder
    sys.modules["dlib.encoders"].resnet = resnet
    sys.modules["dlib.encoders"].vgg = vgg
    sys.modules["dlib.encoders"].inceptionv3 = inc
    sys.modules["dlib.encoders"].vgg_encoders = vgg.vgg_encoders
    sys.modules["dlib"].encoders = sys.modules["dlib.encoders"]


def reference_models():
    _install_stubs()
    import importlib
    unet = importlib.import_module("dlib.unet.model")
    stdcl = importlib.import_module("dlib.stdcl.classifier")
    const = importlib.import_module("dlib.configure.constants")
    return unet, stdcl, const


def build_ref_tcam(unet, const, classes=10):
    m = unet.UnetTCAM(
        task=const.TCAM, encoder_name="resnet50", encoder_depth=5,
        encoder_weights=None, decoder_channels=(256, 128, 64, 32, 16),
        in_channels=3, seg_h_out_channels=2, scale_in=1.,
        aux_params=dict(pooling_head="WGAP", classes=classes,
                        support_background=False),
        freeze_cl=True, im_rec=False)
    return m


def build_ref_family_tcam(unet, const, encoder_name, classes=10):
    # process/instantiators.py:46-55 (get_encoder_d_c) + :495-529
    depth, dec = (3, (256, 128, 64)) if encoder_name == "vgg16" else (5, (256, 128, 64, 32, 16))
    return unet.UnetTCAM(
        task=const.TCAM, encoder_name=encoder_name, encoder_depth=depth,
        encoder_weights=None, decoder_channels=dec, in_channels=3, seg_h_out_channels=2,
        scale_in=1., aux_params=dict(pooling_head="WGAP", classes=classes,
                                     support_background=False),
        freeze_cl=True, im_rec=False)


def build_ref_stdcl(stdcl, const, classes=10):
    return stdcl.STDClassifier(
        task=const.STD_CL, encoder_name="resnet50", encoder_depth=5,
        encoder_weights=None, in_channels=3, scale_in=1.,
        aux_params=dict(pooling_head="WGAP", classes=classes,
                        support_background=False))


def ref_tcam_cam(model, frame):
    """inference_wsol.py:248-346 for TCAM: forward, SegmentationCam
    (builtincam.py:201-225), nan_to_num, bilinear to image size, t2n."""
    import importlib
    builtincam = importlib.import_module("dlib.cams.builtincam")
    ext = builtincam.SegmentationCam(model=model)
    with torch.no_grad():
        cl_logits, fcams, _ = model(frame[None])
        cam = ext(argmax=False)
        cam = torch.nan_to_num(cam, nan=0.0, posinf=1., neginf=0.0)
        cam = F.interpolate(cam[None, None], frame.shape[1:], mode="bilinear",
                            align_corners=False)[0, 0]
    return cl_logits[0].numpy(), fcams[0].numpy(), cam.numpy().astype(float)


def ref_std_cam(model, frame, class_idx):
    """STD_CL CAM: cam.py:31-99 + core.py:139-193 (normalized=True), then
    bilinear (align_corners=False) to image size (inference_wsol.py:342-346)."""
    import importlib
    cam_mod = importlib.import_module("dlib.cams.cam")
    ext = cam_mod.CAM(model=model, target_layer="encoder.layer4.2.relu3",
                      fc_layer="classification_head.fc")
    with torch.no_grad():
        logits = model(frame[None])
        low = ext(class_idx=class_idx, scores=logits, normalized=True)
        cam = F.interpolate(low[None, None].clone(), frame.shape[1:],
                            mode="bilinear", align_corners=False)[0, 0]
    ext.clear_hooks()
    return logits[0].numpy(), low.numpy(), cam.numpy().astype(float)


def normalized_frames(n, size, seed):
    from tcam_wsol_video_amd.utils.seeding import synthetic_clip
    clip = synthetic_clip(n, seed=seed, height=size, width=size)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    mean = torch.tensor([0.485, .456, .406])[None, :, None, None]
    std = torch.tensor([.229, .224, .225])[None, :, None, None]
    return ((x - mean) / std).contiguous(), clip


def family_goldens(unet, const, seed=1234):
    """VGG16-TCAM (configs[3]) and InceptionV3-TCAM (configs[4]) goldens: full outputs at
    a small size, logits + CAM at the configs' size (224 / 299)."""
    for name, small, big in (("vgg16", 64, 224), ("inceptionv3", 96, 299)):
        m = build_ref_family_tcam(unet, const, name)
        m.load_state_dict(seeded_state_dict(m, seed), strict=True)
        m.eval()
        out = {"keys": np.array(list(m.state_dict().keys())),
               "shapes": np.array([",".join(map(str, v.shape))
                                   for v in m.state_dict().values()])}
        for size, n, full in ((small, 2, True), (big, 1, False)):
            x, _ = normalized_frames(n, size, seed=11 + size)
            out[f"x{size}"] = x.numpy()
            res = [ref_tcam_cam(m, x[i]) for i in range(n)]
            out[f"logits{size}"] = np.stack([r[0] for r in res])
            out[f"cam{size}"] = np.stack([r[2] for r in res]).astype(np.float32)
            if full:
                out[f"fcams{size}"] = np.stack([r[1] for r in res])
        np.savez_compressed(os.path.join(HERE, f"{name}_tcam.npz"), seed=seed, **out)


def main():
    torch.set_num_threads(8)
    unet, stdcl, const = reference_models()
    if "--family" in sys.argv:
        family_goldens(unet, const)
        print("wrote", os.listdir(HERE))
        return
    seed = 1234
    out = {}

    tcam = build_ref_tcam(unet, const)
    tcam.load_state_dict(seeded_state_dict(tcam, seed), strict=True)
    tcam.eval()
    keys = list(tcam.state_dict().keys())
    shapes = [tuple(v.shape) for v in tcam.state_dict().values()]
    out["tcam_keys"] = np.array(keys)
    out["tcam_shapes"] = np.array([",".join(map(str, s)) for s in shapes])
    for size, n in ((64, 2), (224, 1)):
        x, _ = normalized_frames(n, size, seed=7 + size)
        out[f"tcam_x{size}"] = x.numpy()
        logits, fcams, cams = [], [], []
        for i in range(n):
            lo, fc, cm = ref_tcam_cam(tcam, x[i])
            logits.append(lo), fcams.append(fc), cams.append(cm)
        out[f"tcam_logits{size}"] = np.stack(logits)
        out[f"tcam_fcams{size}"] = np.stack(fcams)
        out[f"tcam_cam{size}"] = np.stack(cams)
    np.savez_compressed(os.path.join(HERE, "r50_tcam.npz"), seed=seed, **out)

    out = {}
    std = build_ref_stdcl(stdcl, const)
    std.load_state_dict(seeded_state_dict(std, seed), strict=True)
    std.eval()
    out["std_keys"] = np.array(list(std.state_dict().keys()))
    x, _ = normalized_frames(1, 224, seed=99)
    lo, low, cam = ref_std_cam(std, x[0], class_idx=3)
    out.update(std_x224=x.numpy(), std_logits224=lo[None], std_low224=low[None],
               std_cam224=cam[None], std_class=np.array([3]))
    np.savez_compressed(os.path.join(HERE, "r50_stdcl.npz"), seed=seed, **out)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
