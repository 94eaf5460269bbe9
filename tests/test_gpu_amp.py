"""GPU checks of the AMP path (the reference's ``--amp True``: train_wsol.py:1077, 1155-1184,
``autocast`` + ``GradScaler``): S1 (fp16) activations, tcam_conv2d_f16 (one fp16 MFMA
product per MAC, fp32 accumulation, fp16 output), the S1 training kernels, and the
device-side GradScaler — against fp64 restatements fed the same fp16-rounded operands
(oracle/train_ref.py ``amp=True``)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import train_ref as T
from tcam_wsol_video_amd import _lib, ops
from tcam_wsol_video_amd.models import build_r50_tcam
from tcam_wsol_video_amd.ops import ConvSrc
from tcam_wsol_video_amd.training import DecoderTrainer

pytestmark = pytest.mark.gpu

U16 = 2.0 ** -11          # fp16 unit roundoff (one rounding of the output)


def _r16(x):
    return x.to(torch.float16).to(x.dtype)


def _s1(x, cuda, cpad=None):
    return ops.s3_from_nchw(x.to(cuda).float().contiguous(), cpad, "amp")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_s1_layout_round_trip(cuda):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 20, 7, 9, generator=g) * 3
    x[0, 0, 0, 0] = 1e6          # beyond fp16: inf, as autocast's cast
    t = _s1(x, cuda, 24)
    assert ops.is_s1(t) and tuple(t.shape) == (2, 7, 9, 3, 1, 8)
    back = ops.s3_to_nchw(t).cpu()
    assert torch.equal(back[:, :20], x.half().float())
    assert (back[:, 20:] == 0).all()


CONV_CASES = [
    # (sources [(C, H, W, up2, stride)], cout, k, pad, relu, residual)
    ([(8, 33, 35, 0, 2)], 64, 7, 3, True, False),             # stem-like 7x7 / 2
    ([(64, 14, 14, 0, 1)], 256, 1, 0, True, True),            # 1x1 + residual
    ([(64, 9, 9, 1, 1), (32, 18, 18, 0, 1)], 64, 3, 1, True, False),   # up2 + skip concat
    ([(32, 20, 20, 0, 1)], 16, 3, 1, True, False),            # thin 3x3 (Cout 16)
    ([(16, 24, 24, 0, 1)], 16, 3, 1, False, False),           # thin 3x3, Ctot 16
    ([(256, 12, 12, 0, 1)], 512, 3, 1, True, False),          # deep 3x3 (LDS-DMA tiles)
    ([(40, 11, 13, 0, 2)], 72, 3, 1, True, False),            # unaligned, strided
]


@pytest.mark.parametrize("case", range(len(CONV_CASES)))
@pytest.mark.parametrize("tile", [-1, 2, 3, 6, 15, 17, 18, 20, 26, 30, 31, 32, 38, 39, 40, 41])
def test_conv2d_f16_matches_fp64(cuda, case, tile):
    srcs, cout, k, pad, relu, has_res = CONV_CASES[case]
    g = torch.Generator().manual_seed(100 * case + tile)
    B = 2
    xs = [torch.randn(B, c, h, w, generator=g) for (c, h, w, u, s) in srcs]
    full = [F.interpolate(x, scale_factor=2, mode="nearest") if u else x
            for x, (c, h, w, u, s) in zip(xs, srcs)]
    xin = _r16(torch.cat(full, 1).double())
    stride = srcs[0][4]
    W = torch.randn(cout, xin.shape[1], k, k, generator=g) * (2.0 / (xin.shape[1] * k * k)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    y = F.conv2d(xin, _r16(W.double()), bias.double(), stride=stride, padding=pad)
    mag = F.conv2d(xin.abs(), _r16(W.double()).abs(), stride=stride, padding=pad)
    Ho, Wo = y.shape[2:]
    res = None
    if has_res:
        res = torch.randn(B, cout, Ho, Wo, generator=g)
        y = y + _r16(res.double())
        mag = mag + res.double().abs()
    if relu:
        y = torch.relu(y)
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(tile)
    try:
        wt = ops.pack_conv_weight_h1([W.to(cuda)])
        assert wt.shape[2] == 1 and ops.weight_fmt(wt) == "amp"
        out = ops.conv2d_x6([ConvSrc(_s1(x, cuda), s, up2=bool(u))
                             for x, (c, h, w, u, s) in zip(xs, srcs)], wt, bias.to(cuda), cout,
                            Ho, Wo, k, pad, relu,
                            residual=None if res is None else _s1(res, cuda))
        torch.cuda.synchronize()
    finally:
        lib.tcam_conv_x6_force_tile(-1)
    assert ops.is_s1(out)
    dev = ops.s3_to_nchw(out).cpu().double()
    # one fp16 rounding of the output + fp32 accumulation of exact fp16 x fp16 products
    bound = U16 * y.abs() + 2e-6 * (mag + 1)
    err = (dev - y).abs()
    assert (err <= bound).all(), (err / (bound)).max().item()


@pytest.mark.parametrize("srcs,cout", [([(24, 9, 11, 0)], 40),
                                       ([(32, 7, 20, 1), (16, 14, 40, 0)], 16),
                                       ([(64, 9, 9, 1), (32, 18, 18, 0)], 72),
                                       ([(64, 14, 14, 1), (64, 28, 28, 0)], 64)])
def test_wgrad_s1_matches_fp64(cuda, srcs, cout):
    """tcam_conv_wgrad_s1 (one fp16 product on v_mfma_f32_32x32x16_f16 for 3x3 / stride 1,
    the generic fp32-MFMA kernel otherwise) vs fp64 on the same fp16 operands; dW rounded
    to fp16 as an autocast conv's weight gradient."""
    g = torch.Generator().manual_seed(cout)
    B = 3
    xs = [_r16(torch.randn(B, c, h, w, generator=g)) for (c, h, w, u) in srcs]
    full = [F.interpolate(x, scale_factor=2, mode="nearest") if u else x
            for x, (c, h, w, u) in zip(xs, srcs)]
    xin = torch.cat(full, 1).double()
    Ho, Wo = xin.shape[2:]
    dy = _r16(torch.randn(B, cout, Ho, Wo, generator=g, dtype=torch.float64))
    Wd = torch.zeros(cout, xin.shape[1], 3, 3, dtype=torch.float64, requires_grad=True)
    (F.conv2d(xin, Wd, padding=1) * dy).sum().backward()
    mag = torch.nn.grad.conv2d_weight(xin.abs(), Wd.shape, dy.abs(), padding=1)
    lib = _lib.load()
    arr = (_lib.tcam_conv_src * len(srcs))()
    keep = []
    for i, (x, (c, h, w, u)) in enumerate(zip(xs, srcs)):
        t = _s1(x, cuda)
        keep.append(t)
        arr[i] = _lib.tcam_conv_src(t.data_ptr(), c, h, w, 1, u)
    dys = _s1(dy, cuda)
    nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, len(srcs), B, cout, Ho, Wo, 3, 3))
    ws = torch.empty(nb, dtype=torch.uint8, device=cuda)
    dw = torch.empty(cout, xin.shape[1], 3, 3, device=cuda)
    _lib.check(lib.tcam_conv_wgrad_s1(arr, len(srcs), B, dys.data_ptr(), cout, Ho, Wo, 3, 3,
                                      1, 1, cout, dw.data_ptr(), ws.data_ptr(), nb, _stream()),
               "wgrad s1")
    torch.cuda.synchronize()
    dev = dw.cpu().double()
    assert torch.equal(dev, _r16(dev))            # an fp16 gradient
    err = (dev - Wd.grad).abs()
    assert (err <= U16 * Wd.grad.abs() + 2e-6 * (mag + 1e-3)).all()


def test_bn_relu_and_bwd_s1(cuda):
    """The BatchNorm-ReLU forward / backward on S1 (fp16 in / out, fp32 inside)."""
    C, B, H, W = 64, 2, 20, 20
    g = torch.Generator().manual_seed(5)
    y = _r16(torch.randn(B, C, H, W, generator=g, dtype=torch.float64))
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    dout = _r16(torch.randn(B, C, H, W, generator=g, dtype=torch.float64))
    yd = y.clone().requires_grad_(True)
    gd, bd = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    mu = yd.mean((0, 2, 3), keepdim=True)
    var = yd.var((0, 2, 3), unbiased=False, keepdim=True)
    o = torch.relu((yd - mu) / torch.sqrt(var + 1e-5) * gd[None, :, None, None] +
                   bd[None, :, None, None])
    (o * dout).sum().backward()
    lib = _lib.load()
    P = B * H * W
    ys = _s1(y, cuda)
    ws = torch.empty(int(lib.tcam_bn_ws_bytes(P, C)), dtype=torch.uint8, device=cuda)
    mean, invstd = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    gam, bet = gamma.float().to(cuda), beta.float().to(cuda)
    _lib.check(lib.tcam_bn_stats_s1(ys.data_ptr(), P, C, 1e-5, 0.1, mean.data_ptr(),
                                    invstd.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                                    ws.data_ptr(), _stream()), "bn stats s1")
    out = torch.empty_like(ys)
    _lib.check(lib.tcam_bn_relu_s1(ys.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                   gam.data_ptr(), bet.data_ptr(), out.data_ptr(), P, C,
                                   _stream()), "bn relu s1")
    o_dev = ops.s3_to_nchw(out).cpu().double()
    assert ((o_dev - o.detach()).abs() <= U16 * o.detach().abs() + 1e-6).all()
    dy = torch.empty_like(ys)
    dgamma, dbeta = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    douts = _s1(dout, cuda)
    _lib.check(lib.tcam_bn_relu_bwd_s1(douts.data_ptr(), out.data_ptr(), ys.data_ptr(),
                                       mean.data_ptr(), invstd.data_ptr(), gam.data_ptr(),
                                       dy.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), P, C,
                                       ws.data_ptr(), _stream()), "bn bwd s1")
    torch.cuda.synchronize()
    ref = yd.grad
    d_dev = ops.s3_to_nchw(dy).cpu().double()
    assert ((d_dev - ref).abs() <= U16 * ref.abs() + 1e-4 * ref.abs().max()).all()
    assert (dbeta.cpu().double() - bd.grad).abs().max() <= 1e-5 * bd.grad.abs().max()
    assert (dgamma.cpu().double() - gd.grad).abs().max() <= 1e-4 * gd.grad.abs().max()


def _batch(n, size, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, size, size, generator=g)
    raw = (torch.rand(n, 3, size, size, generator=g) * 255).round()
    seeds = torch.randint(-1, 2, (n, size, size), generator=g)
    seeds[seeds < 0] = -255
    return x, raw, seeds


def _rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _amp_masks_and_feats(tr, x):
    saved = tr.bn_flat.clone()
    from tcam_wsol_video_amd.models import _encoder_plan_x6
    enc = _encoder_plan_x6(tr.model.encoder, x.device, "amp")   # the trainer's plan, rebuilt
    feats = [x.cpu()] + [ops.s3_to_nchw(f).cpu() for f in enc.forward(x)[1:]]
    _, _, st = tr.forward(x)
    masks = {}
    for i, blk in enumerate(st["blocks"]):
        masks[f"decoder.blocks.{i}.conv1"] = (ops.s3_to_nchw(blk["a1"]) > 0).cpu()
        masks[f"decoder.blocks.{i}.conv2"] = (ops.s3_to_nchw(blk["a2"]) > 0).cpu()
    tr.set_bn_flat(saved)
    torch.cuda.synchronize()
    return masks, feats


# measured on MI355X (round 3, profiles/round3_amp_oracle_errors.txt): worst per-parameter
# gradient error 2.4e-3 / 2.5e-3 of the parameter's max |grad| (seeds (21,5), (22,7)):
# single fp16 ulps (4.9e-4 relative) of the device's fp32-then-fp16 roundings against the
# oracle's fp64-then-fp16 ones, carried through the backward
AMP_GRAD_TOL = 1e-2


@pytest.mark.parametrize("mseed,bseed", [(21, 5), (22, 7)])
def test_amp_train_step_matches_fp64_oracle(cuda, mseed, bseed):
    """One --amp step (ResNet50-TCAM, 2 frames 64x64) vs oracle/train_ref.train_step(amp=True)
    fed the device's autocast encoder features and ReLU branches: losses, BN statistics,
    every decoder / seg-head gradient (unscaled), the SGD update."""
    model = build_r50_tcam(seed=mseed)
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(cuda)
    x, raw, seeds = _batch(2, 64, seed=bseed)
    tr = DecoderTrainer(model, amp=True)
    masks, feats = _amp_masks_and_feats(tr, x.to(cuda))
    losses_ref, grads, new, bufs = T.train_step(sd_cpu, x, raw, seeds, masks=masks, amp=True,
                                                scale=float(tr.scale.item()), feats=feats)
    losses = tr.step(x.to(cuda), raw.to(cuda), seeds.to(cuda)).cpu().numpy()
    torch.cuda.synchronize()
    assert (tr.applied_steps, tr.skipped_steps) == (1, 0)
    for i, k in enumerate(("total", "sl", "crf", "size")):
        assert abs(losses[i] - losses_ref[k]) <= 2e-3 * max(abs(losses_ref[k]), 1e-3), k
    sd = model.state_dict()
    for k, v in bufs.items():
        assert _rel(sd[k], v) < 2e-3, k
    named = dict(model.named_parameters())
    errs = {k: _rel(tr.g(named[k]), gref) for k, gref in grads.items()}
    worst = max(errs, key=errs.get)
    print(f"amp seeds ({mseed},{bseed}): worst {worst} {errs[worst]:.2e}")
    assert errs[worst] <= AMP_GRAD_TOL, (worst, errs[worst])
    for k, v in new.items():
        d = (sd[k].cpu().double() - v).abs().max().item()
        # (lr 0.01, nesterov's first step moves p by 1.9 lr d)
        assert d <= 1e-7 + 2 * 0.01 * AMP_GRAD_TOL * grads[k].abs().max().item() + \
            1e-5 * v.abs().max().item(), k


def test_amp_step_close_to_fp32_step(cuda):
    """Sanity: the AMP step's gradients against the fp32-accurate (x6) step's on the same
    batch.  Not a parity bound (the oracle test above is): fp16 operands through the frozen
    50-layer encoder and ReLU branch flips move the random-init gradient by ~6 % (measured
    0.059 of its norm on MI355X)."""
    x, raw, seeds = _batch(2, 64, seed=3)
    ta = DecoderTrainer(build_r50_tcam(seed=8).to(cuda), amp=True)
    tf = DecoderTrainer(build_r50_tcam(seed=8).to(cuda))
    la = ta.step(x.to(cuda), raw.to(cuda), seeds.to(cuda)).cpu()
    lf = tf.step(x.to(cuda), raw.to(cuda), seeds.to(cuda)).cpu()
    torch.cuda.synchronize()
    assert abs(float(la[0]) - float(lf[0])) <= 1e-2 * abs(float(lf[0]))
    num = (ta.grad - tf.grad).norm().item()
    assert num <= 0.15 * tf.grad.norm().item(), num / tf.grad.norm().item()


def test_amp_grad_scaler_semantics(cuda):
    """GradScaler on the device (torch.cuda.amp.GradScaler semantics, train_wsol.py:1180-1183):
    a non-finite loss skips the step and leaves the scale alone (the reference never calls
    the scaler then); an fp16 overflow of the scaled gradients skips the step and halves the
    scale; growth_interval clean steps double it."""
    x, raw, seeds = _batch(2, 64, seed=12)
    xd, rd, sdd = x.to(cuda), raw.to(cuda), seeds.to(cuda)
    # (1) NaN loss
    bad = xd.clone()
    bad[1, :, 5:9, 7:11] = float("nan")
    tr = DecoderTrainer(build_r50_tcam(seed=3).to(cuda), amp=True, growth_interval=2)
    w0 = tr.flat.clone()
    tr.step(bad, rd, sdd)
    torch.cuda.synchronize()
    assert torch.equal(tr.flat, w0) and float(tr.scale.item()) == 2.0 ** 16
    assert (tr.applied_steps, tr.skipped_steps) == (0, 1)
    # (2) growth: two clean steps -> scale x2
    tr.step(xd, rd, sdd)
    tr.step(xd, rd, sdd)
    torch.cuda.synchronize()
    assert (tr.applied_steps, tr.skipped_steps) == (2, 1)
    assert float(tr.scale.item()) == 2.0 ** 17 and int(tr.growth_tracker.item()) == 0
    # (3) overflow: a scale far beyond fp16's range makes the scaled gradients inf
    tr2 = DecoderTrainer(build_r50_tcam(seed=3).to(cuda), amp=True, init_scale=2.0 ** 60)
    w1, m1 = tr2.flat.clone(), tr2.mom.clone()
    tr2.step(xd, rd, sdd)
    torch.cuda.synchronize()
    assert float(tr2.found_inf.item()) != 0.0
    assert torch.equal(tr2.flat, w1) and torch.equal(tr2.mom, m1)
    assert float(tr2.scale.item()) == 2.0 ** 59 and (tr2.applied_steps, tr2.skipped_steps) == (0, 1)
    # backs off until the step fits fp16 again
    for _ in range(60):
        tr2.step(xd, rd, sdd)
        if tr2.applied_steps:
            break
    torch.cuda.synchronize()
    assert tr2.applied_steps == 1 and float(tr2.scale.item()) <= 2.0 ** 40


def test_amp_eval_plan_close_to_fp32(cuda):
    """conv_precision='amp' (--amp_eval) on the eval plans: fp16 convolutions, CAMs within
    fp16 error of the fp32-accurate path."""
    model = build_r50_tcam(seed=1).to(cuda).eval()
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(2)).to(cuda)
    with torch.no_grad():
        model.conv_precision = "x6"
        lo_f, fc_f, _ = model(x)
        model.conv_precision = "amp"
        lo_a, fc_a, _ = model(x)
    torch.cuda.synchronize()
    assert _rel(lo_a, lo_f) < 5e-2
    assert _rel(fc_a, fc_f) < 5e-2
