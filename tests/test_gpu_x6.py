"""GPU parity of the x6 path (bf16-split MFMA convolution on S3 activations)
and of the S3-layout kernels, against PyTorch fp64/fp32 references.

The x6 conv keeps the six split products of order <= 2 (csrc/conv_x6.hip), so
its error is an fp32-accumulation error: it is checked against fp64 with the
bound used for an fp32 FMA chain, relative to sum_k |w x|."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.ops import ConvSrc

pytestmark = pytest.mark.gpu

# |out - fp64| <= X6_TOL * sum_k |w_k x_k|  (fp32 FMA chains measure ~1e-7..4e-7)
X6_TOL = 2e-6


def _s3(x_nchw, cuda, cpad=None):
    return ops.s3_from_nchw(x_nchw.to(cuda).contiguous(), cpad)


X6_CASES = [
    # (B, [(C, H, W, stride, up2)], Cout, KS, pad, relu, residual)
    (2, [(8, 37, 41, 2, 0)], 64, 7, 3, True, False),            # stem (image padded to 8)
    (2, [(64, 14, 14, 1, 0)], 64, 1, 0, True, False),
    (2, [(64, 14, 14, 1, 0)], 256, 1, 0, True, True),           # conv3 + identity
    (3, [(32, 15, 15, 2, 0)], 32, 3, 1, True, False),           # strided 3x3
    (2, [(128, 7, 7, 1, 0)], 128, 3, 1, True, False),
    (2, [(128, 7, 7, 1, 0), (96, 14, 14, 2, 0)], 512, 1, 0, True, False),  # conv3 + ds
    (2, [(48, 7, 9, 1, 1), (40, 14, 18, 1, 0)], 64, 3, 1, True, False),    # up2 + skip
    (2, [(32, 9, 9, 1, 1)], 16, 3, 1, True, False),             # last decoder block
    (2, [(16, 18, 18, 1, 0)], 16, 3, 1, True, False),           # C = 16
    (2, [(16, 20, 17, 1, 0)], 8, 3, 1, False, False),           # Cout 8 on the 16-row thin kernel
    (1, [(200, 5, 6, 1, 0)], 136, 3, 1, True, False),           # ragged M, K tails
    (3, [(96, 9, 11, 1, 0)], 40, 3, 1, False, True),            # Cout % 32 != 0, residual
    (4, [(256, 14, 14, 1, 0)], 512, 3, 1, True, False),
    # thin 3x3 (halo-tiled kernel): two sources with up2, partial 16x16 tiles, Cout 24
    (2, [(64, 9, 10, 1, 1), (64, 18, 20, 1, 0)], 32, 3, 1, True, False),
    (1, [(32, 40, 37, 1, 0)], 32, 3, 1, True, False),
    (2, [(32, 17, 19, 1, 0)], 24, 3, 1, False, False),
    (2, [(64, 15, 13, 1, 0)], 64, 3, 1, True, False),
    (1, [(32, 8, 9, 1, 1), (64, 16, 18, 1, 0)], 40, 3, 1, True, False),
    # decoder-training dgrad shapes (ResNet50-TCAM at 64^2): no ReLU, wide Cout
    (2, [(256, 8, 8, 1, 0)], 3072, 3, 1, False, False),
    (2, [(128, 8, 8, 1, 0)], 768, 3, 1, False, False),
    (2, [(128, 8, 8, 1, 0)], 128, 3, 1, False, False),
    (2, [(256, 8, 8, 1, 0), (512, 8, 8, 1, 0)], 128, 3, 1, True, False),  # decoder block 1
    (2, [(768, 8, 8, 1, 0)], 128, 3, 1, True, False),
    # deep-K aligned 2-source up2 (the InceptionV3 decoder block 0): one partial wave of
    # LDS-DMA tiles -> automatic stream-K
    (1, [(1024, 5, 5, 1, 1), (768, 10, 10, 1, 0)], 256, 3, 1, True, False),
    (2, [(512, 6, 6, 1, 0)], 384, 3, 1, True, False),
    (2, [(256, 6, 6, 1, 1), (288, 12, 12, 1, 0)], 128, 3, 1, True, False),
    (2, [(288, 6, 6, 1, 1), (768, 12, 12, 1, 0)], 128, 3, 1, True, False),
    (2, [(256, 12, 12, 1, 0)], 256, 3, 1, True, False),
]


@pytest.mark.parametrize("sk", [-1, 0, 3, 7])
@pytest.mark.parametrize("tile", [-1] + list(range(30)))
@pytest.mark.parametrize("case", X6_CASES)
def test_conv2d_x6_matches_fp64(cuda, case, tile, sk):
    from tcam_wsol_video_amd import _lib
    B, srcs, cout, ks, pad, relu, use_res = case
    g = torch.Generator().manual_seed(hash(str(case)) % 1000)
    xs = [torch.randn(B, c, h, w, generator=g) for (c, h, w, s, u) in srcs]
    if srcs[0][0] == 8 and ks == 7:
        xs[0][:, 3:] = 0
    ws = [torch.randn(cout, c, ks, ks, generator=g) / np.sqrt(c * ks * ks)
          for (c, h, w, s, u) in srcs]
    bias = torch.randn(cout, generator=g)
    ref, absd = None, None
    for x, w, (c, h, wd, s, u) in zip(xs, ws, srcs):
        xx = F.interpolate(x, scale_factor=2, mode="nearest") if u else x
        y = F.conv2d(xx.double(), w.double(), stride=s, padding=pad)
        a = F.conv2d(xx.double().abs(), w.double().abs(), stride=s, padding=pad)
        ref = y if ref is None else ref + y
        absd = a if absd is None else absd + a
    ref = ref + bias.double()[None, :, None, None]
    Ho, Wo = ref.shape[2:]
    res = torch.randn(B, cout, Ho, Wo, generator=g) if use_res else None
    if res is not None:
        ref = ref + res.double()
    if relu:
        ref = ref.clamp_min(0)
    wt = ops.pack_conv_weight_x6([w.to(cuda) for w in ws])
    s3 = [ConvSrc(_s3(x, cuda), s, bool(u)) for x, (c, h, w, s, u) in zip(xs, srcs)]
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    lib.tcam_conv_x6_force_streamk(sk)
    try:
        out = ops.conv2d_x6(s3, wt, bias.to(cuda), cout, Ho, Wo, ks, pad, relu,
                            residual=_s3(res, cuda) if res is not None else None)
        if sk > 0:  # deterministic: a second run is bit-identical
            out2 = ops.conv2d_x6(s3, wt, bias.to(cuda), cout, Ho, Wo, ks, pad, relu,
                                 residual=_s3(res, cuda) if res is not None else None)
            assert torch.equal(out, out2)
    finally:
        lib.tcam_conv_x6_force_tile(-1)
        lib.tcam_conv_x6_force_streamk(-1)
    got = ops.s3_to_nchw(out).cpu().double()
    err = (got - ref).abs()
    bound = X6_TOL * (absd + (res.double().abs() if res is not None else 0) + 1.0)
    assert bool((err <= bound).all()), f"max err {err.max().item()}"
    # stored parts are the canonical split of the stored value
    hi, mid, lo = ops.split3(ops.s3_to_nchw(out).permute(0, 2, 3, 1).contiguous())
    parts = out.view(B, Ho, Wo, cout // 8, 3, 8)
    assert torch.equal(parts[..., 0, :].reshape(hi.shape), hi)
    assert torch.equal(parts[..., 1, :].reshape(mid.shape), mid)
    assert torch.equal(parts[..., 2, :].reshape(lo.shape), lo)


@pytest.mark.parametrize("sk", [-1, 3])
@pytest.mark.parametrize("tile", [-1, 3, 15, 17, 18, 23, 29])
@pytest.mark.parametrize("couts", [(64, 48, 64), (192, 128, 128), (24, 40), (32,)])
def test_grouped_launch_matches_fp64(cuda, couts, tile, sk):
    """tcam_conv2d_x6_multi (one launch over output-stacked 1x1 weights, the Inception
    branch-parallel convs): every member matches its own fp64 conv and lands in its own
    tensor / channel slice; channels outside the slices stay untouched.  Non-16x16 tiles
    (3) fall back to a 16x16x32 tile."""
    from tcam_wsol_video_amd import _lib
    g = torch.Generator().manual_seed(sum(couts) + tile)
    B, C, H, W = 2, 96, 9, 11
    x = torch.randn(B, C, H, W, generator=g)
    ws = [torch.randn(c, C, 1, 1, generator=g) / np.sqrt(C) for c in couts]
    bs = [torch.randn(c, generator=g) for c in couts]
    wt = ops.pack_conv_weight_x6([torch.cat(ws, 0).to(cuda)])
    bias = torch.cat(bs).to(cuda)
    wide = ops.s3_from_nchw(torch.full((B, couts[0] + 32, H, W), 7.0).to(cuda))
    outs = [(wide, 16)] + [None] * (len(couts) - 1)
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    lib.tcam_conv_x6_force_streamk(sk)
    try:
        got = ops.conv2d_x6_multi([ConvSrc(_s3(x, cuda), 1)], wt, bias, couts, H, W, 1, 0, True,
                                  outs)
    finally:
        lib.tcam_conv_x6_force_tile(-1)
        lib.tcam_conv_x6_force_streamk(-1)
    assert got[0] is wide
    full = ops.s3_to_nchw(wide).cpu().double()
    assert bool((full[:, :16] == 7.0).all()) and bool((full[:, 16 + couts[0]:] == 7.0).all())
    for i, (w, b) in enumerate(zip(ws, bs)):
        ref = (F.conv2d(x.double(), w.double()) + b.double()[None, :, None, None]).clamp_min(0)
        absd = F.conv2d(x.double().abs(), w.double().abs())
        y = full[:, 16:16 + couts[0]] if i == 0 else ops.s3_to_nchw(got[i]).cpu().double()
        assert y.shape == ref.shape
        assert bool(((y - ref).abs() <= X6_TOL * (absd + 1.0)).all()), (i, couts, tile)


def test_s3_roundtrip_exact(cuda):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 24, 9, 7, generator=g) * torch.logspace(-20, 20, 24)[None, :, None, None]
    s = _s3(x, cuda)
    assert s.shape == (2, 9, 7, 3, 3, 8)
    back = ops.s3_to_nchw(s).cpu()
    assert torch.equal(back, x)
    # channel padding (image -> 8 channels)
    img = torch.randn(2, 3, 5, 6, generator=g)
    s = _s3(img, cuda, 8)
    back = ops.s3_to_nchw(s).cpu()
    assert torch.equal(back[:, :3], img) and bool((back[:, 3:] == 0).all())


def test_maxpool_s3(cuda):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 16, 13, 10, generator=g)
    out = ops.s3_to_nchw(ops.maxpool3x3s2_s3(_s3(x, cuda))).cpu()
    assert torch.equal(out, F.max_pool2d(x, 3, 2, 1))


@pytest.mark.parametrize("hw,size", [((7, 7), (14, 14)), ((14, 14), (14, 14)),
                                     ((5, 6), (9, 13))])
def test_up2_resize_s3(cuda, hw, size):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 24, *hw, generator=g)
    ref = F.interpolate(F.interpolate(x, scale_factor=2, mode="nearest"), size=size,
                        mode="bilinear", align_corners=True)
    out = ops.s3_to_nchw(ops.up2_resize_s3(_s3(x, cuda), size)).cpu()
    assert (out - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("shape", [(3, 64, 28, 28), (2, 2048, 7, 9), (1, 8192, 3, 5),
                                   (2, 520, 1, 37)])
def test_wgap_s3(cuda, shape):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(*shape, generator=g).clamp_min(0)
    w = torch.randn(10, shape[1], generator=g) / shape[1] ** 0.5
    b = torch.randn(10, generator=g)
    ref = F.linear(x.double().mean(dim=(2, 3)), w.double(), b.double())
    out = ops.wgap_s3(_s3(x, cuda), w.to(cuda), b.to(cuda)).cpu().double()
    assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("shape", [(2, 16, 20, 24), (1, 64, 17, 33), (3, 8, 1, 1),
                                   (1, 16, 224, 224)])
@pytest.mark.parametrize("argmax", [False, True])
def test_seghead_cam_s3(cuda, argmax, shape):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(*shape, generator=g)
    w = torch.randn(2, shape[1], 3, 3, generator=g) * 0.3
    b = torch.randn(2, generator=g)
    fc_ref = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    absd = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    fcams, cam, u8 = ops.seghead_cam_s3(_s3(x, cuda), w.to(cuda), b.to(cuda), argmax=argmax)
    # fp32 fmaf chain over 9 Cin terms: relative to sum |w x| as the x6 bound
    assert bool(((fcams.cpu().double() - fc_ref).abs() <= X6_TOL * (absd + 1.0)).all())
    ref = (fc_ref.argmax(1).double() if argmax else torch.softmax(fc_ref, 1)[:, 1])
    if not argmax:
        assert (cam.cpu().double() - ref).abs().max().item() < 1e-5
    f, c2, u2 = ops.seghead_cam(x.to(cuda), w.to(cuda), b.to(cuda), argmax=argmax)
    assert (cam - c2).abs().max().item() < 1e-5


def test_std_cam_s3_matches_nchw(cuda):
    g = torch.Generator().manual_seed(8)
    A = torch.randn(2, 64, 28, 28, generator=g).clamp_min(0).to(cuda)
    w = torch.randn(5, 64, generator=g).to(cuda)
    cls = torch.tensor([1, 3], dtype=torch.int32, device=cuda)
    l1, c1, u1 = ops.std_cam(A, w, cls, (224, 224))
    l2, c2, u2 = ops.std_cam(ops.s3_from_nchw(A), w, cls, (224, 224))
    assert (l1 - l2).abs().max().item() < 1e-5
    assert (c1 - c2).abs().max().item() < 1e-5
