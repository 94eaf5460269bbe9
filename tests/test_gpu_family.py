"""GPU parity of the VGG16-TCAM and InceptionV3-TCAM forwards
against the reference's own golden outputs and the oracle, plus the ops they add:
rectangular-tap / strided-output x6 convolutions, S3 pooling, the seg-head resize."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import model_ref as R
from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.inference import CAM, CAMComputer
from tcam_wsol_video_amd.models import (TRG_LAYERS, build_inceptionv3_tcam, build_stdcl,
                                        build_vgg16_tcam)
from tcam_wsol_video_amd.ops import ConvSrc
from tcam_wsol_video_amd.utils.seeding import synthetic_clip

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
CAM_TOL = 1e-4   # north_star: CAMs within 1e-4 fp32 of the reference CPU path
X6_TOL = 2e-6


def _s3(x, cuda, cpad=None):
    return ops.s3_from_nchw(x.to(cuda).contiguous(), cpad)


@pytest.mark.parametrize("kh,kw,ph,pw,stride", [(1, 7, 0, 3, 1), (7, 1, 3, 0, 1),
                                                (1, 3, 0, 1, 1), (3, 1, 1, 0, 1),
                                                (5, 5, 2, 2, 1), (3, 3, 1, 1, 2),
                                                (3, 3, 0, 0, 1)])
@pytest.mark.parametrize("coff", [0, 24])
def test_conv_rect_taps_and_concat_offset(cuda, kh, kw, ph, pw, stride, coff):
    g = torch.Generator().manual_seed(kh * 10 + kw + stride)
    B, C, H, W, cout = 2, 48, 17, 19, 40
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(cout, C, kh, kw, generator=g) / np.sqrt(C * kh * kw)
    b = torch.randn(cout, generator=g)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=(ph, pw))
    absd = F.conv2d(x.double().abs(), w.double().abs(), stride=stride, padding=(ph, pw))
    ref = ref.clamp_min(0)
    Ho, Wo = ref.shape[2:]
    wt = ops.pack_conv_weight_x6([w.to(cuda)])
    ctot = coff + cout + 16
    out = ops.s3_empty(B, Ho, Wo, ctot, cuda)
    out.zero_()
    ops.conv2d_x6([ConvSrc(_s3(x, cuda), stride)], wt, b.to(cuda), cout, Ho, Wo, (kh, kw),
                  (ph, pw), True, out=out, out_coff=coff)
    full = ops.s3_to_nchw(out).cpu().double()
    got = full[:, coff:coff + cout]
    assert bool(((got - ref).abs() <= X6_TOL * (absd + 1.0)).all())
    # channels outside the slice untouched
    assert float(full[:, :coff].abs().max() if coff else 0.0) == 0.0
    assert float(full[:, coff + cout:].abs().max()) == 0.0


@pytest.mark.parametrize("k,s,p,mode,ceil", [(2, 2, 0, "max", False), (3, 2, 1, "max", True),
                                             (3, 1, 1, "max", False), (3, 1, 1, "avg", False),
                                             (3, 2, 1, "avg", True), (3, 2, 0, "max", False)])
@pytest.mark.parametrize("hw", [(57, 57), (29, 30), (112, 112), (8, 9)])
def test_pool2d_s3_matches_torch(cuda, k, s, p, mode, ceil, hw):
    g = torch.Generator().manual_seed(hw[0] + k)
    x = torch.randn(2, 24, hw[0], hw[1], generator=g)
    if mode == "max":
        ref = F.max_pool2d(x, k, s, p, ceil_mode=ceil)
    else:
        ref = F.avg_pool2d(x, k, s, p, ceil_mode=ceil, count_include_pad=True)
    out = ops.pool2d_s3(_s3(x, cuda), k, s, p, mode, ceil_mode=ceil)
    got = ops.s3_to_nchw(out).cpu()
    assert got.shape == ref.shape
    if mode == "max":
        assert torch.equal(got, ref)
    else:
        assert (got - ref).abs().max().item() <= 1e-6 * max(1.0, ref.abs().max().item())


def test_pool2d_s3_concat_offset(cuda):
    x = torch.randn(1, 16, 11, 13)
    out = ops.s3_empty(1, 11, 13, 40, cuda)
    out.zero_()
    ops.pool2d_s3(_s3(x, cuda), 3, 1, 1, "max", out=out, out_coff=16)
    full = ops.s3_to_nchw(out).cpu()
    assert torch.equal(full[:, 16:32], F.max_pool2d(x, 3, 1, 1))
    assert full[:, :16].abs().max() == 0 and full[:, 32:].abs().max() == 0


def test_resize_cam_matches_torch(cuda):
    f = torch.randn(2, 2, 30, 30)
    fo, cam, u8 = ops.resize_cam(f.to(cuda), (29, 29))
    ref = F.interpolate(f, size=(29, 29), mode="bilinear", align_corners=True)
    assert (fo.cpu() - ref).abs().max().item() < 1e-5
    rc = torch.softmax(ref, 1)[:, 1]
    assert (cam.cpu() - rc).abs().max().item() < 1e-5


FAMILY = {"vgg16": (build_vgg16_tcam, 64, 224), "inceptionv3": (build_inceptionv3_tcam, 96, 299)}


@pytest.fixture(scope="module", params=[(n, p) for n in sorted(FAMILY) for p in ("x6", "f16x3")],
                ids=lambda v: f"{v[0]}-{v[1]}")
def family(request, cuda):
    name, prec = request.param
    build, small, big = FAMILY[name]
    d = np.load(os.path.join(G, f"{name}_tcam.npz"))
    m = build(seed=int(d["seed"])).to(cuda)
    m.conv_precision = prec
    return name, m, d, small, big


def test_family_matches_reference_golden(cuda, family):
    name, model, d, small, big = family
    for size in (small, big):
        x = torch.from_numpy(d[f"x{size}"]).to(cuda)
        with torch.no_grad():
            logits, fcams, _ = model(x)
        torch.cuda.synchronize()
        assert fcams.shape[2:] == x.shape[2:]
        assert np.abs(logits.cpu().numpy() - d[f"logits{size}"]).max() < 1e-3, name
        if f"fcams{size}" in d.files:
            assert np.abs(fcams.cpu().numpy() - d[f"fcams{size}"]).max() < 1e-3, name
        cam = model.cam.cpu().double().numpy()
        assert np.abs(cam - d[f"cam{size}"]).max() < CAM_TOL, name
        assert model.cam_u8.shape == cam.shape


def test_family_batch_matches_oracle(cuda, family):
    name, model, d, small, big = family
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    size = 224
    clip = synthetic_clip(3, seed=5, height=size, width=size)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    x = ((x - torch.tensor([0.485, .456, .406])[None, :, None, None]) /
         torch.tensor([.229, .224, .225])[None, :, None, None]).contiguous()
    with torch.no_grad():
        logits, fcams, _ = model(x.to(cuda))
    lo_ref, fc_ref, _ = R.tcam_forward(sd, x)
    assert (logits.cpu() - lo_ref).abs().max().item() < 1e-3
    cam_ref = R.segmentation_cam(fc_ref)
    assert (model.cam.cpu() - cam_ref).abs().max().item() < CAM_TOL


@pytest.mark.parametrize("prec", ["x6", "f16x3"])
@pytest.mark.parametrize("name", ["vgg16", "inceptionv3"])
def test_family_stdcl_cam_matches_oracle(cuda, name, prec):
    m = build_stdcl(name, seed=77).to(cuda)
    m.conv_precision = prec
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    clip = synthetic_clip(2, seed=3, height=224, width=224)
    x = (torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0 - 0.45) / 0.225
    x = x.contiguous()
    with torch.no_grad():
        logits = m(x.to(cuda))
    feats = R.encoder_features(sd, x)
    lo_ref = R.wgap(sd, feats[-1])
    assert (logits.cpu() - lo_ref).abs().max().item() < 1e-3
    ext = CAM(m, target_layer=TRG_LAYERS[name])
    cam = ext(class_idx=[1, 4], reshape=(224, 224))
    for b, c in enumerate((1, 4)):
        _, ref = R.std_cam(sd, feats[-1][b:b + 1], c, (224, 224))
        assert np.abs(cam[b].cpu().double().numpy() - ref).max() < CAM_TOL


def test_family_camcomputer_runs(cuda, family):
    name, model, d, small, big = family
    comp = CAMComputer(model, cam_curve_interval=0.01)
    clip = synthetic_clip(4, seed=9, height=224, width=224)
    x = (torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0 - 0.45) / 0.225
    gt = torch.tensor([[[20, 30, 150, 170]]] * 4, dtype=torch.int32, device=cuda)
    tg = torch.tensor([0, 1, 2, 3], device=cuda)
    comp.evaluate_batch(x.to(cuda).contiguous(), tg, gt)
    res = comp.compute_and_evaluate()
    assert res is not None
