"""ConRanFieldTcams at crf_tc_scale != 1 (losses/tcam.py:80-115 through
crf/dense_crf_loss.py:95-123): the fused training loss filters a nearest-resized image and
a bilinear-resized S at sigma_xy * scale, against the reference's filter (oracle/_ref) on
the same resized inputs and the reference's custom backward taken through the resize."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import crf_ref as R
from tcam_wsol_video_amd import losses as L
from tcam_wsol_video_amd.training import tcam_losses

pytestmark = pytest.mark.gpu


def _filter(img, seg, sr, sx):
    if R.ref_available("xy"):
        return R.ref_bilateral(img, seg, sr, sx)
    return R.port_bilateral(img, seg, sr, sx)


@pytest.mark.parametrize("scale,H,W", [(0.5, 64, 48), (0.75, 40, 56)])
def test_scaled_crf_term_matches_reference_semantics(cuda, scale, H, W):
    rng = np.random.default_rng(int(scale * 100) + H)
    B, lam, sr, sx = 3, 2e-3, 15.0, 100.0
    yy, xx = np.mgrid[0:H, 0:W]
    base = 128 + 100 * np.sin(xx / 9.0) * np.cos(yy / 7.0)
    raw = np.stack([base, 0.7 * base + 30, 255 - base], 0)[None].repeat(B, 0)
    raw = (raw + rng.normal(0, 6, raw.shape)).clip(0, 255).astype(np.float32)
    fcams = torch.from_numpy(rng.normal(0, 2, (B, 2, H, W)).astype(np.float32))
    losses, dF = tcam_losses(fcams.to(cuda), torch.from_numpy(raw).to(cuda), None,
                             lam=(0.0, lam, 0.0), crf_scale=scale)
    # reference semantics on the host: the same resizes (fp32, as the reference's own
    # F.interpolate on its device tensors), the reference filter, its custom backward
    S = torch.softmax(fcams, 1)
    si = F.interpolate(torch.from_numpy(raw), scale_factor=scale, mode="nearest",
                       recompute_scale_factor=False)
    S_req = S.clone().requires_grad_(True)
    ss = F.interpolate(S_req, scale_factor=scale, mode="bilinear",
                       recompute_scale_factor=False, align_corners=False)
    AS = _filter(si.numpy(), ss.detach().numpy(), sr, sx * scale).astype(np.float64)
    val = lam * -(ss.detach().double().numpy() * AS).sum() / B
    (gS,) = torch.autograd.grad(ss, S_req, torch.from_numpy(-2.0 * lam * AS / B).float())
    gS = gS.double()
    S64 = S.double()
    dF_ref = S64 * (gS - (gS * S64).sum(1, keepdim=True))
    lo = losses.cpu().double().numpy()
    assert losses.numel() == 4
    assert abs(lo[2] - val) <= 1e-5 * abs(val), (lo[2], val)
    assert abs(lo[0] - val) <= 1e-5 * abs(val)
    assert lo[1] == 0.0 and lo[3] == 0.0
    np.testing.assert_allclose(dF.cpu().double().numpy(), dF_ref.numpy(), rtol=1e-4,
                               atol=1e-5 * float(dF_ref.abs().max()))


def test_master_loss_takes_the_crf_scale(cuda):
    """MasterLoss with ConRanFieldTcams(scale_factor=0.5) reports the scaled term."""
    rng = np.random.default_rng(3)
    B, H, W = 2, 32, 32
    raw = torch.from_numpy((rng.random((B, 3, H, W)) * 255).astype(np.float32))
    fcams = torch.from_numpy(rng.normal(0, 1, (B, 2, H, W)).astype(np.float32)).to(cuda)
    fcams.requires_grad_(True)
    m = L.MasterLoss(cuda_id=0)
    m.add(L.ConRanFieldTcams(cuda_id=0, lambda_=2e-3, sigma_rgb=15.0, sigma_xy=100.0,
                             scale_factor=0.5))
    total = m(epoch=0, fcams=fcams, raw_img=raw)
    total.backward()
    direct, dF = tcam_losses(fcams.detach(), raw.to(cuda), None, lam=(0.0, 2e-3, 0.0),
                             crf_scale=0.5)
    assert torch.equal(total.detach().reshape(1), direct[:1])
    assert torch.equal(fcams.grad, dF)


def test_scaled_rgb_joint_term_matches_reference_semantics(cuda):
    """RgbJointConRanFieldTcams at rgb_jcrf_tc_scale 0.5: each group's width mosaic
    (pair_samples, losses/tcam.py:207-232) resized, the reference's colour filter (DIM 3),
    -sum(S' AS') per mosaic, the mean over groups; d / d S through the resize and the
    mosaic's concatenation."""
    from tcam_wsol_video_amd.losses import group_ordered_frames
    rng = np.random.default_rng(21)
    B, H, W, lam, sr, scale = 5, 24, 20, 2e-3, 15.0, 0.5
    raw = (rng.random((B, 3, H, W)) * 255).astype(np.float32)
    fcams = torch.from_numpy(rng.normal(0, 2, (B, 2, H, W)).astype(np.float32))
    seq, frm = [0, 0, 1, 1, 1], [1, 0, 2, 0, 1]
    groups = group_ordered_frames(seq, frm)
    losses, dF = tcam_losses(fcams.to(cuda), torch.from_numpy(raw).to(cuda), None,
                             lam=(0.0, 0.0, 0.0), rgb=(lam, sr, groups, scale))
    S = torch.softmax(fcams, 1)
    S_req = S.clone().requires_grad_(True)
    groups = [list(g) for g in groups if len(g) >= 2]
    c = float(len(groups))
    val = 0.0
    gS = torch.zeros_like(S)
    for g in groups:
        img_m = torch.cat([torch.from_numpy(raw[b]) for b in g], dim=2)[None]
        s_m = torch.cat([S_req[b] for b in g], dim=2)[None]
        si = F.interpolate(img_m, scale_factor=scale, mode="nearest",
                           recompute_scale_factor=False)
        ss = F.interpolate(s_m, scale_factor=scale, mode="bilinear",
                           recompute_scale_factor=False, align_corners=False)
        if R.ref_available("color"):
            AS = R.ref_colorbilateral(si.numpy(), ss.detach().numpy(), sr, 3)
        else:
            AS = R.port_bilateral(si.numpy(), ss.detach().numpy(), sr, 0.0, dim=3)
        AS = AS.astype(np.float64)
        val += -(ss.detach().double().numpy() * AS).sum()
        (gg,) = torch.autograd.grad(ss, S_req, torch.from_numpy(-2.0 * lam / c * AS).float())
        gS += gg
    val *= lam / c
    S64, gS = S.double(), gS.double()
    dF_ref = S64 * (gS - (gS * S64).sum(1, keepdim=True))
    lo = losses.cpu().double().numpy()
    assert losses.numel() == 5
    assert abs(lo[4] - val) <= 1e-5 * abs(val), (lo[4], val)
    assert abs(lo[0] - val) <= 1e-5 * abs(val)
    np.testing.assert_allclose(dF.cpu().double().numpy(), dF_ref.numpy(), rtol=1e-4,
                               atol=1e-5 * float(dF_ref.abs().max()))
