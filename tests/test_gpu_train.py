"""GPU parity of the TCAM training step (tcam_wsol_video_amd.training) against the CPU
autograd restatement of the reference step (oracle/train_ref.py: train-mode decoder BN,
SelfLearning + CRF + ELB-size losses, torch.optim.SGD nesterov), and of its kernels."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import train_ref as T
from tcam_wsol_video_amd import _lib, ops
from tcam_wsol_video_amd.models import build_r50_tcam, build_vgg16_tcam
from tcam_wsol_video_amd.ops import ConvSrc
from tcam_wsol_video_amd.training import DecoderTrainer

pytestmark = pytest.mark.gpu


def _s3(x, cuda, cpad=None):
    return ops.s3_from_nchw(x.to(cuda).contiguous(), cpad)


def _rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("srcs,cout,stride", [([(24, 9, 11, 0)], 40, 1),
                                              ([(16, 5, 6, 1), (8, 10, 12, 0)], 32, 1),
                                              ([(32, 12, 12, 0)], 16, 2),
                                              # 3x3/s1 patch path: up2 + skip, M 1 and 2 subtiles
                                              ([(32, 7, 20, 1), (16, 14, 40, 0)], 16, 1),
                                              ([(64, 9, 9, 1), (32, 18, 18, 0)], 72, 1),
                                              ([(16, 37, 35, 0)], 8, 1),
                                              # several patches per block and split
                                              ([(64, 14, 14, 1), (64, 28, 28, 0)], 64, 1)])
@pytest.mark.parametrize("fp32", [0, 1])   # 3x3/s1: x6 (default) and the fp32-MFMA kernel
def test_wgrad_matches_fp64(cuda, srcs, cout, stride, fp32):
    g = torch.Generator().manual_seed(cout + stride)
    B = 3
    xs = [torch.randn(B, c, h, w, generator=g) for (c, h, w, u) in srcs]
    full = [F.interpolate(x, scale_factor=2, mode="nearest") if u else x
            for x, (c, h, w, u) in zip(xs, srcs)]
    xin = torch.cat(full, 1).double().requires_grad_(True)
    W = torch.randn(cout, xin.shape[1], 3, 3, generator=g, dtype=torch.float64)
    y = F.conv2d(xin, W.requires_grad_(True), stride=stride, padding=1)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (y * dy).sum().backward()
    Ho, Wo = y.shape[2:]
    lib = _lib.load()
    arr = (_lib.tcam_conv_src * len(srcs))()
    keep = []
    for i, (x, (c, h, w, u)) in enumerate(zip(xs, srcs)):
        t = _s3(x, cuda)
        keep.append(t)
        arr[i] = _lib.tcam_conv_src(t.data_ptr(), c, h, w, stride, u)
    dys = _s3(dy.float(), cuda)
    nb = int(lib.tcam_conv_wgrad_ws_bytes(arr, len(srcs), B, cout, Ho, Wo, 3, 3))
    ws = torch.empty(nb, dtype=torch.uint8, device=cuda)
    dw = torch.empty(cout, xin.shape[1], 3, 3, device=cuda)
    lib.tcam_wgrad_force_fp32(fp32)
    try:
        _lib.check(lib.tcam_conv_wgrad_s3(arr, len(srcs), B, dys.data_ptr(), cout, Ho, Wo, 3, 3,
                                          1, 1, cout, dw.data_ptr(), ws.data_ptr(), nb,
                                          torch.cuda.current_stream().cuda_stream), "wgrad")
        torch.cuda.synchronize()
    finally:
        lib.tcam_wgrad_force_fp32(0)
    assert _rel(dw, W.grad) < 2e-5


def test_up2_resize_bwd_is_adjoint(cuda):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 16, 14, 14, generator=g, dtype=torch.float64, requires_grad=True)
    up = F.interpolate(F.interpolate(x, scale_factor=2, mode="nearest"), size=(13, 13),
                       mode="bilinear", align_corners=True)
    gout = torch.randn(up.shape, generator=g, dtype=torch.float64)
    (up * gout).sum().backward()
    gx = ops.s3_empty(2, 14, 14, 16, cuda)
    lib = _lib.load()
    _lib.check(lib.tcam_up2_resize_bwd_s3(_s3(gout.float(), cuda).data_ptr(), gx.data_ptr(), 2,
                                          16, 14, 14, 13, 13,
                                          torch.cuda.current_stream().cuda_stream), "bwd")
    assert _rel(ops.s3_to_nchw(gx), x.grad) < 1e-5


def _batch(n, size, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, size, size, generator=g)
    raw = (torch.rand(n, 3, size, size, generator=g) * 255).round()
    seeds = torch.randint(-1, 2, (n, size, size), generator=g)
    seeds[seeds < 0] = -255
    return x, raw, seeds


# (model seed, batch seed) triples of the parity check.  A ReLU whose pre-activation
# sits within fp32 rounding of 0 takes the other branch under any fp32 forward
# (torch's own fp32 step included: at seeds (21, 6) it is 1.2e-2 from fp64), which
# moves that pixel's gradient discontinuously; at 64^2 with batch 2 roughly one seed
# in three has such a pixel somewhere in the decoder for a given summation order.
# The check therefore asks every seed to stay clear of a gross error and a majority
# of seeds to meet the fp32 bound (a systematic kernel error fails all of them).
# VGG16's un-normalised 13-conv chain flips kinks on most seeds (measured: 9.5e-3,
# 2.8e-2, 4.9e-2 against torch fp32's 6.7e-3, 3.9e-3, 1.7e-3): one seed within the
# fp32 bound, every seed under a 1e-1 guard.
TRAIN_SEEDS = [(21, 5), (22, 7), (24, 9)]


@pytest.mark.parametrize("build,size,need,gross", [(build_r50_tcam, 64, 2, 5e-2),
                                                   (build_vgg16_tcam, 64, 1, 1e-1)])
def test_train_step_matches_autograd_oracle(cuda, build, size, need, gross):
    within, report = 0, []
    for mseed, bseed in TRAIN_SEEDS:
        model = build(seed=mseed)
        sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()}
        model = model.to(cuda)
        x, raw, seeds = _batch(2, size, seed=bseed)
        losses_ref, grads, new, bufs = T.train_step(sd_cpu, x, raw, seeds)
        tr = DecoderTrainer(model)
        losses = tr.step(x.to(cuda), raw.to(cuda), seeds.to(cuda)).cpu().numpy()
        torch.cuda.synchronize()
        # the forward (losses, BN running statistics) is continuous: every seed
        for i, k in enumerate(("total", "sl", "crf", "size")):
            assert abs(losses[i] - losses_ref[k]) <= 1e-4 * max(abs(losses_ref[k]), 1e-3), k
        sd = model.state_dict()
        for k, v in bufs.items():
            assert _rel(sd[k], v) < 1e-4, k
        named = dict(model.named_parameters())
        errs = {k: _rel(tr.g(named[k]), gref) for k, gref in grads.items()}
        # The reference's own fp32 step (torch CPU autograd) against the same fp64 oracle
        # bounds the conditioning: ReLU kinks in deep chains (the un-normalised VGG16
        # features) move fp32 gradients by up to ~7e-3 there, ~1e-5 for ResNet50.
        _, g32, _, _ = T.train_step(sd_cpu, x, raw, seeds, dtype=torch.float32)
        cond = max(_rel(g32[k], grads[k]) for k in errs)   # the model's fp32 conditioning
        # our step and torch's fp32 step are two independent fp32 roundings of the same
        # chain; where it is ill-conditioned (VGG16: cond ~7e-3) each lands ~cond from
        # fp64 in its own direction, so allow 4x that spread (ResNet50: 1e-3 floor)
        tol = max(1e-3, 4.0 * cond)
        worst = max(errs, key=errs.get)
        report.append(f"seeds ({mseed},{bseed}): worst {worst} {errs[worst]:.1e} / tol "
                      f"{tol:.1e} (torch fp32 {cond:.1e})")
        assert errs[worst] <= max(gross, 4.0 * cond), report   # gross-error guard
        if errs[worst] <= tol:
            within += 1
            # SGD update (lr * grad) on a seed whose gradient met the bound
            for k, v in new.items():
                assert (sd[k].cpu() - v).abs().max().item() <= \
                    1e-6 + 1e-4 * v.abs().max().item(), k
    print("\n".join(report))
    assert within >= need, report


def test_train_steps_reduce_loss(cuda):
    model = build_r50_tcam(seed=4).to(cuda)
    x, raw, seeds = _batch(4, 64, seed=9)
    tr = DecoderTrainer(model, lr=0.01)
    first = None
    for _ in range(5):
        l = tr.step(x.to(cuda), raw.to(cuda), seeds.to(cuda))
        first = float(l[1]) if first is None else first
    assert float(l[1]) < first   # self-learning CE decreases on a fixed batch
    # the trained model still runs the inference path (plans re-folded)
    model.eval()
    with torch.no_grad():
        lo, fc, _ = model(x.to(cuda))
    assert torch.isfinite(fc).all()


@pytest.mark.parametrize("C,B,H,W", [(16, 3, 40, 37), (24, 2, 9, 11), (64, 2, 20, 20),
                                     (256, 4, 28, 28)])
def test_bn_relu_bwd_matches_fp64(cuda, C, B, H, W):
    """tcam_bn_relu_bwd_s3 (coalesced partials when 256 % (C/8) == 0, else the per-group
    kernel) against fp64 autograd of relu(BN_train(y))."""
    g = torch.Generator().manual_seed(C + H)
    y = torch.randn(B, C, H, W, generator=g)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    dout = torch.randn(B, C, H, W, generator=g)
    yd = y.double().requires_grad_(True)
    gd, bd = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    mu = yd.mean((0, 2, 3), keepdim=True)
    var = yd.var((0, 2, 3), unbiased=False, keepdim=True)
    o = torch.relu((yd - mu) / torch.sqrt(var + 1e-5) * gd[None, :, None, None] + bd[None, :, None, None])
    (o * dout.double()).sum().backward()
    mean = mu.flatten().float()
    invstd = (1.0 / torch.sqrt(var.flatten() + 1e-5)).float()
    lib = _lib.load()
    P = B * H * W
    ys, outs, douts = _s3(y, cuda), _s3(o.detach().float(), cuda), _s3(dout, cuda)
    ws = torch.empty(int(lib.tcam_bn_ws_bytes(P, C)), dtype=torch.uint8, device=cuda)
    dy = torch.empty_like(ys)
    dgamma, dbeta = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    mean_d, invstd_d, gamma_d = mean.to(cuda), invstd.to(cuda), gamma.to(cuda)  # kept alive
    _lib.check(lib.tcam_bn_relu_bwd_s3(douts.data_ptr(), outs.data_ptr(), ys.data_ptr(),
                                       mean_d.data_ptr(), invstd_d.data_ptr(),
                                       gamma_d.data_ptr(), dy.data_ptr(),
                                       dgamma.data_ptr(), dbeta.data_ptr(), P, C, ws.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), "bn bwd")
    assert _rel(dbeta, bd.grad) < 1e-5
    assert _rel(dgamma, gd.grad) < 1e-4
    assert _rel(ops.s3_to_nchw(dy), yd.grad) < 1e-4
