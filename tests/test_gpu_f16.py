"""GPU parity of the f16x3 path (fp16-split MFMA convolution on S2 activations,
csrc/conv_x6.hip FmtF16) and of the S2-layout kernels (csrc/s3.hip over LayS2).

Operands are x = h + l with h = fp16(x), l = fp16(x - h) (22 significand bits; weights
carry a per-output-channel power-of-two scale), each product keeps al*bh + ah*bl + ah*bh,
accumulated in fp32.  Against fp64 the error is then the fp32-accumulation error plus
<= 3 * 2^-22 |w x| per product: the x6 path's bound X6_TOL (relative to sum_k |w x|) holds
for it as well, and is what these tests assert."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_x6 import X6_CASES, X6_TOL
from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.ops import ConvSrc

pytestmark = pytest.mark.gpu


def _s2(x_nchw, cuda, cpad=None):
    return ops.s3_from_nchw(x_nchw.to(cuda).contiguous(), cpad, fmt="f16x3")


def _split2(x):
    h = x.to(torch.float16)
    return h, (x - h.float()).to(torch.float16)


def _check_split(out):
    h = out[..., 0, :].float()
    lo = out[..., 1, :].float()
    ha = out[..., 0, :].abs()
    ulp = (torch.nextafter(ha, torch.full_like(ha, float("inf"))) - ha).float()
    assert bool((lo.abs() <= 0.5 * ulp).all()), "lo part exceeds half an ulp of hi"
    assert bool(torch.isfinite(h).all())


def _fp64_case(case, g):
    B, srcs, cout, ks, pad, relu, use_res = case
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
        absd = absd + res.double().abs()
    if relu:
        ref = ref.clamp_min(0)
    return xs, ws, bias, res, ref, absd


@pytest.mark.parametrize("sk", [-1, 3])
@pytest.mark.parametrize("tile", [-1] + list(range(38)))
@pytest.mark.parametrize("case", X6_CASES)
def test_conv2d_f16x3_matches_fp64(cuda, case, tile, sk):
    from tcam_wsol_video_amd import _lib
    B, srcs, cout, ks, pad, relu, use_res = case
    g = torch.Generator().manual_seed(hash(str(case)) % 1000)
    xs, ws, bias, res, ref, absd = _fp64_case(case, g)
    Ho, Wo = ref.shape[2:]
    wt, wscale = ops.pack_conv_weight_f16([w.to(cuda) for w in ws])
    s2 = [ConvSrc(_s2(x, cuda), s, bool(u)) for x, (c, h, w, s, u) in zip(xs, srcs)]
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    lib.tcam_conv_x6_force_streamk(sk)
    try:
        out = ops.conv2d_x6(s2, wt, bias.to(cuda), cout, Ho, Wo, ks, pad, relu,
                            residual=_s2(res, cuda) if res is not None else None,
                            wscale=wscale)
        if sk > 0:  # deterministic: a second run is bit-identical
            out2 = ops.conv2d_x6(s2, wt, bias.to(cuda), cout, Ho, Wo, ks, pad, relu,
                                 residual=_s2(res, cuda) if res is not None else None,
                                 wscale=wscale)
            assert torch.equal(out, out2)
    finally:
        lib.tcam_conv_x6_force_tile(-1)
        lib.tcam_conv_x6_force_streamk(-1)
    ops.check_f16_overflow(cuda)
    assert ops.is_s2(out)
    got = ops.s3_to_nchw(out).cpu().double()
    err = (got - ref).abs()
    bound = X6_TOL * (absd + 1.0)
    assert bool((err <= bound).all()), f"max err {err.max().item()}"
    # stored parts are a split of the kernel's fp32 result: |l| <= ulp(h) / 2 (l is itself
    # rounded, so h + l need not re-split to the same pair at ties)
    _check_split(out)


@pytest.mark.parametrize("tile", [-1, 3, 15, 17, 18, 23])
@pytest.mark.parametrize("couts", [(64, 48, 64), (192, 128, 128), (32,)])
def test_grouped_launch_f16x3_matches_fp64(cuda, couts, tile):
    from tcam_wsol_video_amd import _lib
    g = torch.Generator().manual_seed(sum(couts) + tile)
    B, C, H, W = 2, 96, 9, 11
    x = torch.randn(B, C, H, W, generator=g)
    ws = [torch.randn(c, C, 1, 1, generator=g) / np.sqrt(C) for c in couts]
    bs = [torch.randn(c, generator=g) for c in couts]
    wt, wscale = ops.pack_conv_weight_f16([torch.cat(ws, 0).to(cuda)])
    bias = torch.cat(bs).to(cuda)
    wide = _s2(torch.full((B, couts[0] + 32, H, W), 7.0), cuda)
    outs = [(wide, 16)] + [None] * (len(couts) - 1)
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    try:
        got = ops.conv2d_x6_multi([ConvSrc(_s2(x, cuda), 1)], wt, bias, couts, H, W, 1, 0,
                                  True, outs, wscale=wscale)
    finally:
        lib.tcam_conv_x6_force_tile(-1)
    full = ops.s3_to_nchw(wide).cpu().double()
    assert bool((full[:, :16] == 7.0).all()) and bool((full[:, 16 + couts[0]:] == 7.0).all())
    for i, (w, b) in enumerate(zip(ws, bs)):
        ref = (F.conv2d(x.double(), w.double()) + b.double()[None, :, None, None]).clamp_min(0)
        absd = F.conv2d(x.double().abs(), w.double().abs())
        y = full[:, 16:16 + couts[0]] if i == 0 else ops.s3_to_nchw(got[i]).cpu().double()
        assert bool(((y - ref).abs() <= X6_TOL * (absd + 1.0)).all()), (i, couts, tile)


def test_weight_pack_f16_is_exact_split():
    g = torch.Generator().manual_seed(2)
    w = torch.randn(40, 24, 3, 3, generator=g) * torch.logspace(-6, 2, 40)[:, None, None, None]
    wt, sc = ops.pack_conv_weight_f16([w])
    kp, mp = ops.conv_x6_weight_dims(24 * 9, 40)
    assert wt.shape == (kp // 32, 4, 2, mp, 8) and wt.dtype == torch.float16
    assert sc.shape == (mp,)
    # value = (h + l) * scale, per column; scale a power of two
    v = (wt[:, :, 0].float() + wt[:, :, 1].float()).permute(0, 1, 3, 2).reshape(kp, mp)
    v = v * sc[None, :]
    ref = w.permute(2, 3, 1, 0).reshape(24 * 9, 40).double()
    rel = ((v[:24 * 9, :40].double() - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
    assert rel <= 2.0 ** -21
    assert bool((torch.log2(sc) == torch.round(torch.log2(sc))).all())


def test_s2_roundtrip_is_the_canonical_split(cuda):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 24, 9, 7, generator=g) * torch.logspace(-3, 3.5, 24)[None, :, None, None]
    s = _s2(x, cuda)
    assert s.shape == (2, 9, 7, 3, 2, 8) and s.dtype == torch.float16
    back = ops.s3_to_nchw(s).cpu()
    h, lo = _split2(x)
    assert torch.equal(back, h.float() + lo.float())
    assert ((back.double() - x.double()).abs() <= 2.0 ** -22 * x.double().abs() + 2.0 ** -25).all()
    img = torch.randn(2, 3, 5, 6, generator=g)
    back = ops.s3_to_nchw(_s2(img, cuda, 8)).cpu()
    assert bool((back[:, 3:] == 0).all())


def test_s2_pools_resize_wgap_seghead_stdcam(cuda):
    """The S2 variants give the S3 kernels' results on the same (S2-representable) values."""
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 16, 13, 10, generator=g)
    xr = ops.s3_to_nchw(_s2(x, cuda)).cpu()        # the S2-representable input
    a, b = _s2(x, cuda), ops.s3_from_nchw(xr.to(cuda))
    # max picks an input value: exact on S2-representable inputs
    assert torch.equal(ops.s3_to_nchw(ops.maxpool3x3s2_s3(a)).cpu(), F.max_pool2d(xr, 3, 2, 1))
    for mode in ("max", "avg"):
        pa = ops.s3_to_nchw(ops.pool2d_s3(a, 3, 1, 1, mode)).cpu().double()
        pb = ops.s3_to_nchw(ops.pool2d_s3(b, 3, 1, 1, mode)).cpu().double()
        assert ((pa - pb).abs() <= 2.0 ** -21 * pb.abs() + 1e-7).all(), mode
    ua = ops.s3_to_nchw(ops.up2_resize_s3(a, (20, 17))).cpu().double()
    ub = ops.s3_to_nchw(ops.up2_resize_s3(b, (20, 17))).cpu().double()
    assert ((ua - ub).abs() <= 2.0 ** -21 * ub.abs() + 1e-7).all()
    w = torch.randn(10, 16, generator=g).to(cuda)
    bb = torch.randn(10, generator=g).to(cuda)
    assert torch.equal(ops.wgap_s3(a, w, bb), ops.wgap_s3(b, w, bb))
    ws = torch.randn(2, 16, 3, 3, generator=g).to(cuda) * 0.3
    f1, c1, u1 = ops.seghead_cam_s3(a, ws, bb[:2])
    f2, c2, u2 = ops.seghead_cam_s3(b, ws, bb[:2])
    assert torch.equal(f1, f2) and torch.equal(u1, u2)
    cls = torch.tensor([1, 3], dtype=torch.int32, device=cuda)
    l1, cc1, _ = ops.std_cam(a, w, cls, (40, 30))
    l2, cc2, _ = ops.std_cam(b, w, cls, (40, 30))
    assert torch.equal(l1, l2) and torch.equal(cc1, cc2)


def test_f16x3_overflow_is_flagged(cuda):
    """An output beyond the S2 range (|x| > 65504) sets the device flag; the check raises
    and resets it."""
    x = torch.full((1, 16, 4, 4), 100.0)
    w = torch.full((16, 16, 1, 1), 100.0)
    wt, sc = ops.pack_conv_weight_f16([w.to(cuda)])
    ops.check_f16_overflow(cuda)
    ops.conv2d_x6([ConvSrc(_s2(x, cuda))], wt, torch.zeros(16, device=cuda), 16, 4, 4, 1, 0,
                  True, wscale=sc)
    with pytest.raises(FloatingPointError):
        ops.check_f16_overflow(cuda)
    ops.check_f16_overflow(cuda)      # reset
    ops.conv2d_x6([ConvSrc(_s2(x / 100, cuda))], wt, torch.zeros(16, device=cuda), 16, 4, 4, 1,
                  0, True, wscale=sc)
    ops.check_f16_overflow(cuda)      # 16 * 100 = 1600: in range


def test_relayout_between_s2_and_s3(cuda):
    """S2 -> S3 is exact; S3 -> S2 gives the canonical S2 split of the S3 values."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 24, 5, 7, generator=g) * torch.logspace(-3, 3, 24)[None, :, None, None]
    s2 = _s2(x, cuda)
    s3 = ops.relayout(s2, "x6")
    assert ops.is_s3(s3) and ops.relayout(s3, "x6") is s3
    assert torch.equal(ops.s3_to_nchw(s3), ops.s3_to_nchw(s2))
    s3b = ops.s3_from_nchw(x.to(cuda))
    back = ops.relayout(s3b, "f16x3")
    assert ops.is_s2(back)
    assert torch.equal(back, _s2(x, cuda))


@pytest.mark.parametrize("cin,cout,k,stride,pad,hw", [(3, 64, 7, 2, 3, (61, 67)),    # R50 conv1
                                                     (3, 64, 7, 2, 3, (224, 224)),
                                                     (3, 32, 3, 2, 0, (45, 38)),     # SPG-I3 1a
                                                     (3, 64, 3, 1, 1, (33, 29)),     # VGG conv1
                                                     (5, 16, 5, 1, 2, (9, 40))])
def test_stem_f16x3_matches_fp64(cuda, cin, cout, k, stride, pad, hw):
    """tcam_stem_f16x3 (the image read directly, K = the real (tap, channel) pairs) against
    fp64, the f16x3 bound; and a second call is bit-identical."""
    g = torch.Generator().manual_seed(cout * k + hw[0])
    B = 2
    x = torch.randn(B, cin, *hw, generator=g) * 2
    w = torch.randn(cout, cin, k, k, generator=g) / np.sqrt(cin * k * k)
    bias = torch.randn(cout, generator=g)
    ref = F.conv2d(x.double(), w.double(), bias.double(), stride=stride, padding=pad)
    absd = F.conv2d(x.double().abs(), w.double().abs(), stride=stride, padding=pad)
    ref = ref.clamp_min(0)
    st = ops.StemF16(w.to(cuda), bias.to(cuda), stride, pad)
    out = ops.stem_f16x3(x.to(cuda), st)
    out2 = ops.stem_f16x3(x.to(cuda), st)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    ops.check_f16_overflow(cuda)
    assert ops.is_s2(out) and tuple(out.shape[1:3]) == tuple(ref.shape[2:])
    got = ops.s3_to_nchw(out).cpu().double()
    err = (got - ref).abs()
    assert bool((err <= X6_TOL * (absd + 1.0)).all()), f"max err {err.max().item()}"
    _check_split(out)


def test_r50_direct_stem_matches_generic_stem(cuda, monkeypatch):
    """The ResNet50 plan's direct stem against the generic f16x3 stem (NCHW -> S2, 49 taps x 8
    padded channels): the same products summed in another order."""
    from tcam_wsol_video_amd.models import _ResNetPlanX6, build_r50_tcam
    model = build_r50_tcam(seed=3).to(cuda).eval()
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(cuda)
    with torch.no_grad():
        direct = _ResNetPlanX6(model.encoder, cuda, "f16x3")
        assert direct.stem_direct is not None
        monkeypatch.setenv("TCAM_STEM_DIRECT", "0")
        generic = _ResNetPlanX6(model.encoder, cuda, "f16x3")
        assert generic.stem_direct is None
        fa, fb = direct.forward(x), generic.forward(x)
    torch.cuda.synchronize()
    for a, b in zip(fa[1:], fb[1:]):
        a, b = ops.s3_to_nchw(a), ops.s3_to_nchw(b)
        assert (a - b).abs().max().item() <= 1e-5 * max(b.abs().max().item(), 1.0)


def _scaled_case(case, g, lo, hi):
    """X6_CASES operands with every input channel of every source scaled by 2^-s_c,
    s_c uniform in [lo, hi] (activations far below fp16's comfortable range)."""
    xs, ws, bias, res, _, _ = _fp64_case(case, g)
    bias = bias * 2.0 ** -6        # on the scale of the small products (sum |w x| ~ 2^-5)
    B, srcs, cout, ks, pad, relu, use_res = case
    exps = [torch.randint(lo, hi + 1, (x.shape[1],), generator=g) for x in xs]
    xt = [x * torch.pow(2.0, -e.double()).float()[None, :, None, None] for x, e in zip(xs, exps)]
    ref, absd = None, None
    for x, w, (c, h, wd, s, u) in zip(xt, ws, srcs):
        xx = F.interpolate(x, scale_factor=2, mode="nearest") if u else x
        y = F.conv2d(xx.double(), w.double(), stride=s, padding=pad)
        a = F.conv2d(xx.double().abs(), w.double().abs(), stride=s, padding=pad)
        ref = y if ref is None else ref + y
        absd = a if absd is None else absd + a
    # the bound's denominator is the sum of the magnitudes of every added term: sum |w x|
    # plus |bias| (+ |residual|) — no constant slack
    ref = ref + bias.double()[None, :, None, None]
    absd = absd + bias.double().abs()[None, :, None, None]
    if res is not None:
        ref = ref + res.double()
        absd = absd + res.double().abs()
    if relu:
        ref = ref.clamp_min(0)
    return xs, xt, exps, ws, bias, res, ref, absd


def _rel_err(out, ref, absd, eout=None):
    got = ops.s3_to_nchw(out).cpu().double()
    if eout is not None:
        got = got * torch.pow(2.0, -eout.double())[None, :, None, None]
    return ((got - ref).abs() / absd.clamp_min(1e-300)).max().item()


@pytest.mark.parametrize("tile", [-1] + list(range(38)))
@pytest.mark.parametrize("case", X6_CASES)
def test_conv2d_f16x3_small_activations_relative(cuda, case, tile):
    """Activations scaled per channel by 2^-4 ... 2^-12: stored raw in S2 their low parts
    fall into fp16's subnormal range (an absolute 2^-25 floor per element, far above the
    fp32 band relative to sum |w x|); stored with the plans' per-channel exponents
    (models.act_exponents: x * 2^e in S2, the weights times 2^-e, the output times 2^e_out)
    every tile meets X6_TOL * (sum |w x| + |bias| (+ |res|)) with no absolute slack."""
    from tcam_wsol_video_amd import _lib
    B, srcs, cout, ks, pad, relu, use_res = case
    if srcs[0][0] == 8 and ks == 7:
        pytest.skip("the stem reads the image (O(1), exponent 0)")
    g = torch.Generator().manual_seed(hash(str(case)) % 1000 + 7)
    xs, xt, exps, ws, bias, res, ref, absd = _scaled_case(case, g, 4, 12)
    Ho, Wo = ref.shape[2:]
    eout = torch.randint(0, 4, (cout,), generator=g)
    fo = torch.pow(2.0, eout.double())
    w_eff = [(w.double() * fo[:, None, None, None] *
              torch.pow(2.0, -e.double())[None, :, None, None]).float() for w, e in zip(ws, exps)]
    wt, wscale = ops.pack_conv_weight_f16([w.to(cuda) for w in w_eff])
    s2 = [ConvSrc(_s2(x, cuda), s, bool(u)) for x, (c, h, w, s, u) in zip(xs, srcs)]
    res_s = (res.double() * fo[None, :, None, None]).float() if res is not None else None
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    try:
        out = ops.conv2d_x6(s2, wt, (bias.double() * fo).float().to(cuda), cout, Ho, Wo, ks,
                            pad, relu, residual=_s2(res_s, cuda) if res is not None else None,
                            wscale=wscale)
    finally:
        lib.tcam_conv_x6_force_tile(-1)
    ops.check_f16_overflow(cuda)
    err = _rel_err(out, ref, absd, eout)
    assert err <= X6_TOL, f"max |err| / sum|wx| = {err:.3g}"
    if tile == -1 and not use_res:
        # control (the test has teeth): activations at 2^-11 ... 2^-13 stored WITHOUT
        # exponents miss the bound
        _, xt2, _, ws2, bias2, _, ref2, absd2 = _scaled_case(case, g, 11, 13)
        wt0, ws0 = ops.pack_conv_weight_f16([w.to(cuda) for w in ws2])
        raw = ops.conv2d_x6([ConvSrc(_s2(x, cuda), s, bool(u))
                             for x, (c, h, w, s, u) in zip(xt2, srcs)], wt0, bias2.to(cuda),
                            cout, Ho, Wo, ks, pad, relu, wscale=ws0)
        assert _rel_err(raw, ref2, absd2) > X6_TOL


def test_r50_small_range_layers_keep_fp32_accuracy(cuda, monkeypatch):
    """A ResNet50-TCAM whose layer2 BatchNorms (gamma, beta) are 2^-10 of their usual size
    (small-range trained channels): with the plans' activation exponents the f16x3 features
    and CAM stay within the fp32 band of the x6 path's; with them turned off
    (TCAM_F16_ACT_SCALE=0) layer2's S2 tensors lose bits."""
    from tcam_wsol_video_amd.models import _ResNetPlanX6, build_r50_tcam
    model = build_r50_tcam(seed=6)
    with torch.no_grad():
        for m in model.encoder.layer2.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.mul_(2.0 ** -10)
                m.bias.mul_(2.0 ** -10)
    model = model.to(cuda).eval()
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(2)).to(cuda)
    with torch.no_grad():
        ref = _ResNetPlanX6(model.encoder, cuda, "x6").forward(x)
        plan = _ResNetPlanX6(model.encoder, cuda, "f16x3")
        assert plan.out_exps[3] is not None and int(plan.out_exps[3].min()) >= 8
        assert plan.out_exps[2] is None and plan.out_exps[4] is None
        got = plan.forward(x)
        monkeypatch.setenv("TCAM_F16_ACT_SCALE", "0")
        raw = _ResNetPlanX6(model.encoder, cuda, "f16x3").forward(x)
    ops.check_f16_overflow(cuda)

    def rel(a, b, e=None):
        a = ops.s3_to_nchw(a).double()
        if e is not None:
            a = a * torch.pow(2.0, -e.double()).to(cuda)[None, :, None, None]
        b = ops.s3_to_nchw(b).double()
        return ((a - b).abs().max() / b.abs().max()).item()
    errs = [rel(a, b, e) for a, b, e in zip(got[1:], ref[1:], plan.out_exps[1:])]
    errs_raw = [rel(a, b) for a, b in zip(raw[1:], ref[1:])]
    assert max(errs) <= 2e-6, errs
    assert errs_raw[2] > 10 * errs[2], (errs_raw, errs)
    # the model-level forward (encoder + decoder + seg head + CAM) against x6
    monkeypatch.delenv("TCAM_F16_ACT_SCALE")
    with torch.no_grad():
        model.conv_precision = "x6"
        lo6, fc6, _ = model(x)
        cam6 = model.cam.clone()
        model.conv_precision = "f16x3"
        lo3, fc3, _ = model(x)
        cam3 = model.cam.clone()
    assert (lo3 - lo6).abs().max().item() <= 1e-5 * max(lo6.abs().max().item(), 1e-3)
    assert (fc3 - fc6).abs().max().item() <= 1e-5 * max(fc6.abs().max().item(), 1.0)
    assert (cam3 - cam6).abs().max().item() <= 1e-5


@pytest.mark.parametrize("fp_tile,base_tile", [(35, 30), (36, 26)])
@pytest.mark.parametrize("case", [
    # (B, srcs [(C, H, W, stride, up2)], Cout, k, pad, relu, residual)
    (2, [(256, 14, 14, 1, 0), (128, 14, 14, 1, 0)], 256, 3, 1, True, False),   # d0.c1-like, 2 srcs
    (2, [(512, 14, 14, 1, 0)], 512, 3, 1, True, False),                        # l4.c2-like
    (2, [(512, 14, 14, 1, 0)], 512, 1, 0, True, True),                         # 1x1 + residual
    (1, [(64, 9, 7, 1, 0)], 128, 3, 1, False, False),                          # K = 18 steps
    (1, [(32, 5, 5, 1, 0)], 256, 1, 0, True, False),                           # K = 1 step
    (1, [(64, 5, 5, 1, 0)], 256, 1, 0, True, False),                           # K = 2 steps
    (1, [(96, 5, 5, 1, 0)], 256, 1, 0, True, True),                            # K = 3 steps
])
def test_fragment_prefetch_tiles_bit_identical(cuda, case, fp_tile, base_tile):
    """Tiles 35 / 36 (the fragment-prefetch ring: next step's LDS fragments read under this
    step's MFMAs, two LDS-DMA steps in flight) run the same MFMAs on the same operands in
    the same order as tiles 30 / 26: bit-identical outputs, every K-step count parity
    (1, 2, 3, even, odd: the unrolled pair, the peeled last step)."""
    from tcam_wsol_video_amd import _lib
    B, srcs, cout, ks, pad, relu, use_res = case
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(B, c, h, w, generator=g) for c, h, w, s, u in srcs]
    ws = [torch.randn(cout, c, ks, ks, generator=g) / np.sqrt(c * ks * ks)
          for c, *_ in srcs]
    bias = torch.randn(cout, generator=g)
    H, W = srcs[0][1], srcs[0][2]
    res = torch.randn(B, cout, H, W, generator=g) if use_res else None
    wt, wscale = ops.pack_conv_weight_f16([w.to(cuda) for w in ws])
    s2 = [ConvSrc(_s2(x, cuda), s, bool(u)) for x, (c, h, w, s, u) in zip(xs, srcs)]
    lib = _lib.load()
    outs = []
    for t in (base_tile, fp_tile):
        lib.tcam_conv_x6_force_tile(t)
        try:
            outs.append(ops.conv2d_x6(s2, wt, bias.to(cuda), cout, H, W, ks, pad, relu,
                                      residual=_s2(res, cuda) if res is not None else None,
                                      wscale=wscale))
        finally:
            lib.tcam_conv_x6_force_tile(-1)
    ops.check_f16_overflow(cuda)
    assert torch.equal(outs[0], outs[1])
