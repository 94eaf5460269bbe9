"""GPU parity of the fused ResNet50 layer-1 bottleneck (tcam_bottleneck_f16x3 / _f16 (AMP),
encoders/resnet.py:175-232 at stride 1): one launch against the three unfused f16x3 convs of
the same folded weights, BIT for bit (the same packed weights, K-step order, f16x3 terms and
epilogue), at the bench geometry (56^2), on frames whose size is not a multiple of the 14x14
tile, with the projection shortcut (first block) and with the residual (blocks 2-3); and a
whole ResNet50 encoder with the fusion on and off."""
import pytest
import torch
import torch.nn as nn

from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.models import FoldedConv
from tcam_wsol_video_amd.ops import ConvSrc

pytestmark = pytest.mark.gpu


def _bn(c, g):
    bn = nn.BatchNorm2d(c)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(c, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(c, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(c, generator=g) + 0.5)
    return bn.eval()


def _block(cin, ds, cuda, seed, fmt="f16x3", mods=None):
    """The block's three folded convs; ``mods`` (a list) receives the (conv, bn) modules."""
    g = torch.Generator().manual_seed(seed)

    def conv(ci, co, k):
        c = nn.Conv2d(ci, co, k, padding=k // 2, bias=False)
        with torch.no_grad():
            c.weight.copy_(torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5)
        return c
    p1 = [(conv(cin, 64, 1), _bn(64, g))]
    p2 = [(conv(64, 64, 3), _bn(64, g))]
    parts = [(conv(64, 256, 1), _bn(256, g))]
    if ds:
        parts.append((conv(cin, 256, 1), _bn(256, g)))
    if mods is not None:
        mods.extend(p1 + p2 + parts)
    c1 = FoldedConv(p1, cuda, fmt)
    c2 = FoldedConv(p2, cuda, fmt)
    c3 = FoldedConv(parts, cuda, fmt)
    return c1, c2, c3


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
@pytest.mark.parametrize("cin,ds", [(64, True), (256, False)])
@pytest.mark.parametrize("B,H,W", [(2, 56, 56), (3, 20, 31), (1, 1, 1)])
def test_bottleneck_matches_fp64_reference(cuda, cin, ds, B, H, W, fmt):
    """The fused launch against the reference Bottleneck itself (encoders/resnet.py:175-232,
    eval-mode BN) in float64 on the same (S2 / S1-rounded) input: f16x3 within 2e-5 of the
    output's largest magnitude (S2 intermediates keep ~22 bits), AMP (fp16 intermediates and
    products, fp32 sums) within 1e-2 — the direct oracle check beside the bit-identity with
    the unfused convs below."""
    g = torch.Generator().manual_seed(77 + cin + H)
    mods = []
    c1, c2, c3 = _block(cin, ds, cuda, seed=H * 7 + W + cin, fmt=fmt, mods=mods)
    x = ops.s3_from_nchw(torch.randn(B, cin, H, W, generator=g).relu().to(cuda), fmt=fmt)
    out = ops.bottleneck_f16x3(x, c1, c2, c3, ds)
    torch.cuda.synchronize()
    ops.check_f16_overflow(cuda)
    x64 = ops.s3_to_nchw(x).double().cpu()

    def cbn(v, m):
        conv, bn = m
        conv, bn = conv.double(), bn.double()
        with torch.no_grad():
            return bn(conv(v))
    h = torch.relu(cbn(x64, mods[0]))
    h = torch.relu(cbn(h, mods[1]))
    ref = torch.relu(cbn(h, mods[2]) + (cbn(x64, mods[3]) if ds else x64))
    got = ops.s3_to_nchw(out).double().cpu()
    tol = 2e-5 if fmt == "f16x3" else 1e-2
    err = float((got - ref).abs().max())
    assert err <= tol * float(ref.abs().max()), (err, float(ref.abs().max()))


def _unfused(x, c1, c2, c3, ds):
    B, H, W, _ = ops.s3_dims(x)
    h1 = ops.conv2d_x6([ConvSrc(x)], c1.wt, c1.bias, 64, H, W, 1, 0, True, stream_k=False,
                       wscale=c1.wscale)
    h2 = ops.conv2d_x6([ConvSrc(h1)], c2.wt, c2.bias, 64, H, W, 3, 1, True, stream_k=False,
                       wscale=c2.wscale)
    if ds:
        return ops.conv2d_x6([ConvSrc(h2), ConvSrc(x)], c3.wt, c3.bias, 256, H, W, 1, 0, True,
                             stream_k=False, wscale=c3.wscale)
    return ops.conv2d_x6([ConvSrc(h2)], c3.wt, c3.bias, 256, H, W, 1, 0, True, residual=x,
                         stream_k=False, wscale=c3.wscale)


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
@pytest.mark.parametrize("cin,ds", [(64, True), (256, False)])
@pytest.mark.parametrize("B,H,W", [(2, 56, 56), (1, 16, 16), (3, 20, 31), (1, 14, 14),
                                   (1, 1, 1), (2, 15, 43)])
def test_bottleneck_bit_identical_to_unfused(cuda, cin, ds, B, H, W, fmt):
    g = torch.Generator().manual_seed(1000 + cin + 7 * H + W)
    c1, c2, c3 = _block(cin, ds, cuda, seed=H * 131 + W, fmt=fmt)
    x = ops.s3_from_nchw(torch.randn(B, cin, H, W, generator=g).relu().to(cuda), fmt=fmt)
    ref = _unfused(x, c1, c2, c3, ds)
    out = ops.bottleneck_f16x3(x, c1, c2, c3, ds)
    torch.cuda.synchronize()
    ops.check_f16_overflow(cuda)
    assert out.shape == ref.shape and out.dtype == ref.dtype
    diff = (out.view(torch.int16) != ref.view(torch.int16))
    assert not bool(diff.any()), f"{int(diff.sum())} of {diff.numel()} words differ"


def test_bottleneck_flags_overflow(cuda):
    """A block whose conv3 output leaves the S2 range sets the shared overflow flag, as the
    unfused conv would."""
    c1, c2, c3 = _block(256, False, cuda, seed=5)
    c3.bias.fill_(1e6)
    g = torch.Generator().manual_seed(3)
    x = ops.s3_from_nchw(torch.randn(1, 256, 14, 14, generator=g).relu().to(cuda), fmt="f16x3")
    ops.check_f16_overflow(cuda)   # clear
    ops.bottleneck_f16x3(x, c1, c2, c3, False)
    torch.cuda.synchronize()
    with pytest.raises(Exception):
        ops.check_f16_overflow(cuda)


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
def test_resnet50_encoder_fused_layer1_matches_unfused(cuda, fmt):
    """The whole f16x3 ResNet50 encoder plan with layer 1 fused and unfused: every feature map
    bit-identical (stream-K off, so the unfused launches accumulate K in the fused order)."""
    from tcam_wsol_video_amd import _lib
    from tcam_wsol_video_amd.models import _ResNetPlanX6, build_r50_tcam
    model = build_r50_tcam(seed=0)
    plan = _ResNetPlanX6(model.encoder, cuda, fmt)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 3, 224, 224, generator=g).to(cuda)
    lib = _lib.load()
    lib.tcam_conv_x6_force_streamk(0)
    try:
        plan.fused_l1 = False
        ref = plan.forward(x)
        plan.fused_l1 = True
        out = plan.forward(x)
        torch.cuda.synchronize()
    finally:
        lib.tcam_conv_x6_force_streamk(-1)
    ops.check_f16_overflow(cuda)
    for i, (a, b) in enumerate(zip(out, ref)):
        assert torch.equal(a, b), f"feature {i} differs"


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
def test_bottleneck_batch_over_2gib_runs_in_frame_chunks(cuda, fmt):
    """A batch whose block output exceeds the kernel's 32-bit offsets (S2: > 668 frames of
    56 x 56 x 256; S1: > 1337) runs as frame chunks: every frame equals the unfused convs
    on that frame alone (frames are independent)."""
    B = 700 if fmt == "f16x3" else 1400
    c1, c2, c3 = _block(256, False, cuda, seed=5, fmt=fmt)
    g = torch.Generator(device=cuda).manual_seed(3)
    one = torch.randn(3, 256, 56, 56, generator=g, device=cuda).relu()
    x = ops.s3_from_nchw(one, fmt=fmt)
    big = x[torch.arange(B, device=cuda) % 3].contiguous()
    out = ops.bottleneck_f16x3(big, c1, c2, c3, False)
    ref = ops.bottleneck_f16x3(x, c1, c2, c3, False)
    torch.cuda.synchronize()
    ops.check_f16_overflow(cuda)
    for b in (0, 1, 2, B - 3, B - 2, B - 1, B // 2):
        assert torch.equal(out[b], ref[b % 3]), b
    del big, out
