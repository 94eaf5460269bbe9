"""GPU parity of the stage-1 (STD_CL) training step — the encoder backward
(tcam_wsol_video_amd.cl_training, csrc/enc_train.hip) — against fp64 references: its kernels
one by one against torch fp64 on the same operands, and one whole step (forward, ClLoss,
backward, both SGD groups, BN statistics) against the fp64 autograd oracle
(oracle/train_ref.stdcl_step, pinned to the reference's own STDClassifier / ClLoss /
get_optimizer goldens by tests/test_train_oracle.py), mask-exact: the oracle's ReLUs take
the branches the device forward took."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import train_ref as T
from tcam_wsol_video_amd import _lib, ops
from tcam_wsol_video_amd.cl_training import ClassifierTrainer
from tcam_wsol_video_amd.models import build_r50_stdcl

pytestmark = pytest.mark.gpu


def _st():
    return torch.cuda.current_stream().cuda_stream


def _act(x, cuda, fmt, cpad=None):
    return ops.s3_from_nchw(x.to(cuda).float().contiguous(), cpad, fmt)


def _nchw(t):
    return ops.s3_to_nchw(t).double().cpu()


def _dy_scaled(dy):
    """dy's per-channel scaled S2 copy (tcam_dy_scaled_s2 with the channel maxima given:
    its own max pass needs C / 8 to divide 256, which every ResNet50 width does)."""
    lib = _lib.load()
    B, H, W, C = ops.s3_dims(dy)
    amax = ops.s3_to_nchw(dy).abs().amax(dim=(0, 2, 3)).contiguous().view(torch.int32)
    scale = torch.empty(C, device=dy.device, dtype=torch.float32)
    dy2 = ops.s2_empty(B, H, W, C, dy.device)
    assert lib.tcam_dy_scaled_s2(dy.data_ptr(), B * H * W, C, amax.data_ptr(), 0,
                                 scale.data_ptr(), dy2.data_ptr(), _st()) == 0
    return dy2, scale


def _wgrad11(x, stride, dy, amp=False):
    lib = _lib.load()
    B, Hin, Win, Cin = ops.s3_dims(x)
    _, Ho, Wo, Cout = ops.s3_dims(dy)
    nb = lib.tcam_wgrad11_ws_bytes(B, Cin, Hin, Win, stride, Cout, Ho, Wo)
    assert nb > 0
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    dw = torch.full((Cout, Cin), float("nan"), device=x.device)
    if amp:
        rc = lib.tcam_wgrad11_s1(x.data_ptr(), B, Cin, Hin, Win, stride, dy.data_ptr(), Cout, Ho,
                                 Wo, dw.data_ptr(), ws.data_ptr(), nb, _st())
    else:
        dy2, sc = _dy_scaled(dy)
        rc = lib.tcam_wgrad11_s2_f16x3(x.data_ptr(), B, Cin, Hin, Win, stride, dy2.data_ptr(),
                                       sc.data_ptr(), Cout, Ho, Wo, dw.data_ptr(),
                                       ws.data_ptr(), nb, _st())
    assert rc == 0
    return dw.cpu().double()


@pytest.mark.parametrize("B,cin,cout,H,W,stride", [
    (2, 64, 256, 14, 14, 1), (2, 256, 64, 14, 14, 1), (3, 256, 512, 16, 16, 2),
    (1, 1024, 2048, 7, 7, 1), (2, 8, 8, 5, 7, 1), (2, 72, 136, 9, 11, 1), (2, 64, 64, 9, 9, 2),
    (4, 512, 128, 28, 28, 1)])
@pytest.mark.parametrize("dmag", [1.0, 1e-7])
def test_wgrad11_f16x3_matches_fp64(cuda, B, cin, cout, H, W, stride, dmag):
    """dW = sum_p dy[p] x[s p]: the f16x3 GEMM on S2 x and the per-channel scaled S2 copy of
    an S3 dy (gradients ~1e-7 included) within fp32 accuracy of the fp64 sum."""
    g = torch.Generator().manual_seed(cin + cout + H + stride)
    x = torch.randn(B, cin, H, W, generator=g)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = torch.randn(B, cout, Ho, Wo, generator=g) * dmag * \
        torch.logspace(-2, 2, cout)[None, :, None, None]
    xs, dys = _act(x, cuda, "f16x3"), _act(dy, cuda, "x6")
    x64, dy64 = _nchw(xs), _nchw(dys)
    xsub = x64[:, :, ::stride, ::stride][:, :, :Ho, :Wo]
    ref = torch.einsum("bmhw,bnhw->mn", dy64, xsub)
    mag = torch.einsum("bmhw,bnhw->mn", dy64.abs(), xsub.abs())
    got = _wgrad11(xs, stride, dys)
    err = (got - ref).abs()
    assert torch.isfinite(got).all()
    assert (err <= 1e-6 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())


@pytest.mark.parametrize("B,cin,cout,H,W,stride", [(2, 64, 256, 14, 14, 1),
                                                   (3, 256, 512, 16, 16, 2),
                                                   (2, 72, 136, 9, 11, 1)])
def test_wgrad11_amp_matches_fp64(cuda, B, cin, cout, H, W, stride):
    """The AMP (S1) 1x1 weight gradient: one fp16 product per MAC, fp32 sums, dW rounded to
    fp16 (autocast's weight gradient)."""
    g = torch.Generator().manual_seed(cin * 3 + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = torch.randn(B, cout, Ho, Wo, generator=g)
    xs, dys = _act(x, cuda, "amp"), _act(dy, cuda, "amp")
    x64, dy64 = _nchw(xs), _nchw(dys)
    xsub = x64[:, :, ::stride, ::stride][:, :, :Ho, :Wo]
    ref = torch.einsum("bmhw,bnhw->mn", dy64, xsub)
    mag = torch.einsum("bmhw,bnhw->mn", dy64.abs(), xsub.abs())
    got = _wgrad11(xs, stride, dys, amp=True)
    assert ((got - ref).abs() <= 2.0 ** -11 * ref.abs() + 1e-6 * mag).all()


@pytest.mark.parametrize("H,W", [(14, 14), (13, 11), (112, 112)])
def test_maxpool_bwd_matches_torch(cuda, H, W):
    """MaxPool2d(3, 2, 1) backward (S3 gradient, S2 forward input) == torch's autograd on the
    same values, including ties (values on a 0.5 grid, ReLU zeros): the first maximum in
    (kh, kw) scan order takes the gradient."""
    g = torch.Generator().manual_seed(H * W)
    B, C = 2, 16
    x = (torch.randn(B, C, H, W, generator=g) * 2).round() / 2
    x = x.clamp(min=0)
    xs = _act(x, cuda, "f16x3")
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    gout = torch.randn(B, C, Ho, Wo, generator=g)
    gs = _act(gout, cuda, "x6")
    lib = _lib.load()
    ws = torch.empty(lib.tcam_maxpool_bwd_ws_bytes(B, C, Ho, Wo), dtype=torch.uint8,
                     device=cuda)
    gin = ops.s3_empty(B, H, W, C, cuda)
    assert lib.tcam_maxpool3x3s2_bwd_s3s2(gs.data_ptr(), xs.data_ptr(), gin.data_ptr(),
                                          ws.data_ptr(), B, C, H, W, Ho, Wo, _st()) == 0
    xr = _nchw(xs).requires_grad_(True)
    F.max_pool2d(xr, 3, 2, 1).backward(_nchw(gs))
    got = _nchw(gin)
    assert torch.allclose(got, xr.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
@pytest.mark.parametrize("proj", [False, True])
@pytest.mark.parametrize("C,H,W", [(64, 9, 7), (24, 9, 7), (512, 28, 30)])
def test_bn_add_relu_matches_torch(cuda, fmt, proj, C, H, W):
    """relu(bn3(y) + (bn_ds(yd) | x)) on given batch statistics (autocast's fp16 BN outputs and
    sum on the AMP path); C / 8 dividing 256 takes the fixed-grid kernel (several elements per
    thread at 512 x 28 x 30), 24 channels the one-element-per-thread one."""
    g = torch.Generator().manual_seed(7 + proj + C)
    B = 2
    y, r = torch.randn(B, C, H, W, generator=g), torch.randn(B, C, H, W, generator=g)
    st = [torch.randn(C, generator=g) * 0.1 for _ in range(2)] + \
        [torch.rand(C, generator=g) + 0.5 for _ in range(2)]
    st2 = [torch.randn(C, generator=g) * 0.1 for _ in range(2)] + \
        [torch.rand(C, generator=g) + 0.5 for _ in range(2)]
    ys, rs = _act(y, cuda, fmt), _act(r, cuda, fmt)
    y64, r64 = _nchw(ys), _nchw(rs)
    q = (lambda t: t.half().double()) if fmt == "amp" else (lambda t: t)

    def bn(v, s):
        mean, beta, invstd, gamma = [t.double()[None, :, None, None] for t in s]
        return gamma * ((v - mean) * invstd) + beta
    ref = F.relu(q(q(bn(y64, st)) + (q(bn(r64, st2)) if proj else r64)))
    dev = [t.to(cuda) for t in st]
    dev2 = [t.to(cuda) for t in st2]
    out = torch.empty_like(ys)
    lay = ops.FMT_LAYOUT[fmt]
    fn = getattr(_lib.load(), f"tcam_bn_add_relu_{lay}")
    args2 = ([rs.data_ptr(), dev2[0].data_ptr(), dev2[2].data_ptr(), dev2[3].data_ptr(),
              dev2[1].data_ptr(), None] if proj else [None] * 5 + [rs.data_ptr()])
    assert fn(ys.data_ptr(), dev[0].data_ptr(), dev[2].data_ptr(), dev[3].data_ptr(),
              dev[1].data_ptr(), *args2, out.data_ptr(), B * H * W, C, _st()) == 0
    got = _nchw(out)
    tol = 2 ** -10 if fmt == "amp" else 1e-6
    err = float(((got - ref).abs() - tol * ref.abs()).max())
    assert err <= 2 * tol, err


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
@pytest.mark.parametrize("C,H,W,k,stride,pad", [(8, 13, 11, 7, 2, 3), (16, 9, 10, 3, 1, 1),
                                                (8, 224, 224, 7, 2, 3)])
def test_im2col_exact(cuda, fmt, C, H, W, k, stride, pad):
    """im2col in 8-channel groups == torch's unfold with the (tap, channel) order, zero
    padding included (the stem's weight-gradient operand)."""
    g = torch.Generator().manual_seed(C + H + k)
    B = 2
    xs = _act(torch.randn(B, C, H, W, generator=g), cuda, fmt)
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    col = ops.act_empty(xs, B, Ho, Wo, k * k * C)
    gb = 32 if fmt == "f16x3" else 16
    assert _lib.load().tcam_im2col(xs.data_ptr(), col.data_ptr(), gb, B, C, H, W, k, k, stride,
                                   pad, Ho, Wo, _st()) == 0
    u = F.unfold(_nchw(xs), k, padding=pad, stride=stride).view(B, C, k * k, Ho, Wo)
    ref = u.permute(0, 2, 1, 3, 4).reshape(B, k * k * C, Ho, Wo)
    assert torch.equal(_nchw(col), ref)


def test_grad_add_mask_and_zero_up2_exact(cuda):
    g = torch.Generator().manual_seed(3)
    B, C, H, W = 2, 24, 10, 12
    a, d = torch.randn(B, C, H, W, generator=g), torch.randn(B, C, H, W, generator=g)
    o = torch.randn(B, C, H, W, generator=g).clamp(min=0)
    as_, ds, os_ = _act(a, cuda, "x6"), _act(d, cuda, "x6"), _act(o, cuda, "f16x3")
    r = torch.empty_like(as_)
    lib = _lib.load()
    assert lib.tcam_grad_add_mask_s3s2(as_.data_ptr(), ds.data_ptr(), os_.data_ptr(),
                                       r.data_ptr(), B * H * W, C, _st()) == 0
    ref = (a + torch.where(_nchw(os_).float() > 0, d, torch.zeros_like(d))).double()
    assert torch.equal(_nchw(r), ref)
    for fmt, gb in (("f16x3", 32), ("amp", 16), ("x6", 48)):
        src = _act(torch.randn(B, C, 5, 6, generator=g), cuda, fmt)
        out = ops.act_empty(src, B, H, W, C)
        assert lib.tcam_zero_up2(src.data_ptr(), out.data_ptr(), gb, B, C, H, W, 5, 6,
                                 _st()) == 0
        ref = torch.zeros(B, C, H, W, dtype=torch.float64)
        ref[:, :, ::2, ::2] = _nchw(src)
        assert torch.equal(_nchw(out), ref)


@pytest.mark.parametrize("fmt", ["f16x3", "amp"])
def test_cls_head_fwd_bwd_matches_torch(cuda, fmt):
    """WGAP (avgpool + fc), nn.CrossEntropyLoss and their backward (fp16 points on AMP)."""
    g = torch.Generator().manual_seed(11)
    B, C, H, W, K = 6, 2048, 7, 5, 10
    x = torch.randn(B, C, H, W, generator=g).clamp(min=0)
    w = torch.randn(K, C, generator=g) * 0.02
    b = torch.randn(K, generator=g) * 0.1
    y = torch.tensor([3, 0, 9, 3, 5, 1], dtype=torch.int32)
    xs = _act(x, cuda, fmt)
    lib = _lib.load()
    lay = ops.FMT_LAYOUT[fmt]
    pooled = torch.empty((B, C), device=cuda)
    logits = torch.empty((B, K), device=cuda)
    ws = torch.empty(lib.tcam_cls_pool_ws_bytes(B, C), dtype=torch.uint8, device=cuda)
    wd, bd = w.to(cuda), b.to(cuda)
    assert getattr(lib, f"tcam_cls_fwd_{lay}")(xs.data_ptr(), B, H * W, C, wd.data_ptr(),
                                               bd.data_ptr(), K, pooled.data_ptr(),
                                               logits.data_ptr(), ws.data_ptr(), _st()) == 0
    loss = torch.empty(1, device=cuda)
    dl = torch.empty((B, K), device=cuda)
    yd = y.to(cuda)
    assert lib.tcam_ce_loss(logits.data_ptr(), yd.data_ptr(), B, K, 1.0, None, loss.data_ptr(),
                            dl.data_ptr(), _st()) == 0
    amp = fmt == "amp"
    gw, gb, dp = torch.empty_like(wd), torch.empty_like(bd), torch.empty((B, C), device=cuda)
    assert lib.tcam_cls_bwd(dl.data_ptr(), pooled.data_ptr(), wd.data_ptr(), B, K, C,
                            1 if amp else 0, gw.data_ptr(), gb.data_ptr(), dp.data_ptr(),
                            _st()) == 0
    gl = "s1" if amp else "s3"
    dout = ops.lay_empty(gl, B, H, W, C, cuda)
    assert getattr(lib, f"tcam_pool_bwd_{gl}")(dp.data_ptr(), B, H * W, C, dout.data_ptr(),
                                               _st()) == 0
    q = T.r16 if amp else (lambda t: t)
    x64 = _nchw(xs).requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    p64 = q(F.adaptive_avg_pool2d(x64, 1).flatten(1))
    z64 = q(F.linear(p64, q(w64), q(b64)))
    l64 = F.cross_entropy(z64, y.long())
    l64.backward()
    tol = 2e-3 if amp else 1e-5
    assert abs(float(loss) - float(l64.detach())) <= tol * abs(float(l64.detach()))
    for got, ref in ((logits, z64.detach()), (gw, w64.grad), (gb, b64.grad),
                     (dout, x64.grad)):
        got = _nchw(got) if got.dim() == 6 else got.cpu().double()
        err = float((got - ref).norm() / ref.norm())
        assert err <= tol, err


@pytest.mark.parametrize("case", ["stem", "conv2s2"])
def test_generic_wgrad_s3s2_matches_fp64(cuda, case):
    """The stem's 7x7/2 (8-channel padded image) and layer2.0's 3x3/2 weight gradients:
    dy S3, x S2, fp32 MFMA."""
    g = torch.Generator().manual_seed(5)
    if case == "stem":
        B, cin, cout, H, W, k, s, pad, cpad = 2, 3, 64, 40, 36, 7, 2, 3, 8
    else:
        B, cin, cout, H, W, k, s, pad, cpad = 2, 32, 48, 14, 15, 3, 2, 1, 32
    x = torch.randn(B, cin, H, W, generator=g)
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    dy = torch.randn(B, cout, Ho, Wo, generator=g)
    xs, dys = _act(x, cuda, "f16x3", cpad), _act(dy, cuda, "x6")
    lib = _lib.load()
    arr = (_lib.tcam_conv_src * 1)()
    arr[0] = _lib.tcam_conv_src(xs.data_ptr(), cpad, H, W, s, 0)
    nb = lib.tcam_conv_wgrad_generic_ws_bytes(arr, 1, B, cout, Ho, Wo, k, k)
    ws = torch.empty(nb, dtype=torch.uint8, device=cuda)
    dw = torch.empty((cout, cpad, k, k), device=cuda)
    assert lib.tcam_conv_wgrad_s3s2(arr, 1, B, dys.data_ptr(), cout, Ho, Wo, k, k, pad, pad,
                                    cout, dw.data_ptr(), ws.data_ptr(), nb, _st()) == 0
    x64 = _nchw(xs)[:, :cin]
    w64 = torch.zeros(cout, cin, k, k, dtype=torch.float64, requires_grad=True)
    F.conv2d(x64, w64, stride=s, padding=pad).backward(_nchw(dys))
    got = dw.cpu().double()[:, :cin]
    assert torch.allclose(got, w64.grad, rtol=1e-5, atol=1e-5 * w64.grad.abs().max())
    assert torch.equal(dw[:, cin:].cpu(), torch.zeros_like(dw[:, cin:].cpu()))


# ------------------------------------------------------------------ the whole step
def _frames(B, size, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, 3, size, size, generator=g)
    mean = torch.tensor([0.485, .456, .406])[None, :, None, None]
    std = torch.tensor([.229, .224, .225])[None, :, None, None]
    return ((x - mean) / std).contiguous()


def _masks(tr, st):
    """The device forward's ReLU branches, keyed as oracle/train_ref.resnet50_train_features."""
    m = {"encoder.relu": _nchw(st["stem"][1]) > 0}
    blocks = [f"encoder.layer{li + 1}.{bi}" for li, layer in enumerate(tr.layers)
              for bi in range(len(layer))]
    for name, s in zip(blocks, st["blocks"]):
        m[name + ".relu1"] = _nchw(s["a1"]) > 0
        m[name + ".relu2"] = _nchw(s["a2"]) > 0
        m[name + ".relu3"] = _nchw(s["out"]) > 0
    return m


def _norm_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("B,size", [(2, 64), (8, 224)])
def test_stdcl_step_matches_fp64_oracle(cuda, B, size):
    """One stage-1 SGD step (f16x3, fp32-accurate) vs the fp64 oracle with the device's ReLU
    branches: loss, logits, EVERY parameter gradient norm-relative <= 1e-4, both SGD groups'
    updated weights, the BN running statistics."""
    torch.manual_seed(0)
    model = build_r50_stdcl(seed=21).to(cuda)
    sd0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    tr = ClassifierTrainer(model, lr=0.01)
    x = _frames(B, size, 3)
    y = torch.tensor([(7 * i + 3) % 10 for i in range(B)], dtype=torch.int32)
    xd = x.to(cuda)
    logits, st = tr.forward(xd)
    loss, dl = tr.loss_and_grad(logits, y.to(cuda))
    tr.loss_gate.copy_(loss)
    tr.backward(dl, st)
    masks = _masks(tr, st)
    names = [n for n, _ in model.named_parameters()]
    gdev = {n: tr.g(p).detach().cpu().clone() for n, p in model.named_parameters()}
    tr.all_reduce_and_step()
    torch.cuda.synchronize()
    ops.check_f16_overflow(cuda, all_ranks=False)
    new_dev = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    lo, lg, grads, new, bufs = T.stdcl_step(sd0, x, y, lr=0.01, masks=masks)
    assert abs(float(loss) - lo) <= 1e-5 * abs(lo)
    assert _norm_rel(logits, lg) <= 1e-5
    worst = max((_norm_rel(gdev[n], grads[n]), n) for n in names)
    assert worst[0] <= 1e-4, worst
    for n in names:   # SGD (both groups: layer4 + head at 10x lr), to fp32's resolution
        d_ref = new[n] - sd0[n].double()
        err = (new_dev[n].double() - new[n]).norm()
        assert err <= 1e-4 * d_ref.norm() + 2 ** -23 * new[n].norm(), n
    msd = model.state_dict()
    for k, v in bufs.items():
        assert torch.allclose(msd[k].cpu().double(), v, rtol=1e-5, atol=1e-6), k
    assert int(msd["encoder.bn1.num_batches_tracked"]) == 1


def test_stdcl_autograd_path_equals_trainer(cuda):
    """model.train(); loss = CrossEntropy(model(x), y); loss.backward() — the reference's loop
    (train_wsol.py:1162-1184) — gives the trainer's gradients (same kernels; the CE gradient
    comes from torch here)."""
    model = build_r50_stdcl(seed=5).to(cuda)
    ref = build_r50_stdcl(seed=5).to(cuda)
    x = _frames(4, 64, 9).to(cuda)
    y = torch.tensor([1, 2, 3, 4], device=cuda)
    tr = ClassifierTrainer(ref, lr=0.01)
    logits, st = tr.forward(x)
    _, dl = tr.loss_and_grad(logits, y)
    tr.backward(dl, st)
    model.train()
    out = model(x)
    assert torch.allclose(out, logits, rtol=0, atol=0)
    F.cross_entropy(out, y).backward()
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        # (torch's CE gradient vs the device kernel's: fp32 rounding, amplified by the
        # train-mode BatchNorm chain as in the oracle pin)
        assert _norm_rel(p.grad, tr.g(q)) <= 1e-4, n
    model.eval()


def test_stdcl_amp_step_matches_fp64_oracle(cuda):
    """--amp True: autocast's fp16 convolutions (S1) + the device GradScaler vs the fp64
    oracle with autocast's fp16 rounding points and the device's ReLU branches."""
    model = build_r50_stdcl(seed=21).to(cuda)
    sd0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    tr = ClassifierTrainer(model, lr=0.01, amp=True)
    B = 4
    x = _frames(B, 96, 4)
    y = torch.tensor([1, 5, 5, 8], dtype=torch.int32)
    logits, st = tr.forward(x.to(cuda))
    loss, dl = tr.loss_and_grad(logits, y.to(cuda))
    tr.backward(dl, st)
    masks = _masks(tr, st)
    gdev = {n: tr.g(p).detach().cpu() / float(tr.scale) for n, p in model.named_parameters()}
    lo, lg, grads, new, bufs = T.stdcl_step(sd0, x, y, lr=0.01, masks=masks, amp=True)
    assert abs(float(loss) - lo) <= 2e-3 * abs(lo)
    worst = max((_norm_rel(gdev[n], grads[n]), n) for n in grads)
    assert worst[0] <= 3e-2, worst


def test_stdcl_steps_reduce_loss_and_skip_nonfinite(cuda):
    """A few steps on a fixed batch lower the loss; a NaN frame skips the step on the device
    (the weights stay bit-unchanged, train_wsol.py:1181)."""
    model = build_r50_stdcl(seed=8).to(cuda)
    tr = ClassifierTrainer(model, lr=0.002)
    x = _frames(8, 64, 1).to(cuda)
    y = torch.arange(8, device=cuda) % 10
    losses = [float(tr.step(x, y)) for _ in range(4)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
    before = tr.flat.clone()
    xb = x.clone()
    xb[0, 0, 0, 0] = float("nan")
    tr.step(xb, y)
    torch.cuda.synchronize()
    assert torch.equal(before, tr.flat)
    assert tr.skipped_steps == 1 and tr.applied_steps == 4


@pytest.mark.parametrize("f16x3", [1, 0])
def test_batched_weight_packs_equal_per_item(cuda, f16x3):
    """tcam_pack_weights (one or two launches for a table of items) == the per-item
    tcam_pack_weight_f16x3 / _f16 calls bit for bit: forward items (incl. the stem's padded
    input channels), data-gradient items over a channel slice with and without kdiv; a second
    call with changed weights re-packs through the cached table."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(11)
    specs = [(64, 3, 7, 7, 0, 0, 0, 8), (256, 64, 1, 1, 0, 0, 0, 0), (64, 64, 3, 3, 0, 0, 0, 0),
             (128, 96, 3, 3, 1, 16, 64, 0), (40, 24, 1, 1, 1, 0, 24, 0)]
    items = (_lib.tcam_pack_item * len(specs))()
    refs, outs, keep = [], [], []
    for it, (co, ci, kh, kw, mode, c0, sel, cpad) in zip(items, specs):
        w = (torch.randn(co, ci, kh, kw, generator=g) * 0.1).to(cuda)
        kdiv = (2.0 ** torch.randint(-3, 4, (co,), generator=g).float()).to(cuda) \
            if (mode and f16x3 and c0) else None
        K, M = (kh * kw * max(ci, cpad), co) if mode == 0 else (kh * kw * co, sel)
        kp, mp = ops.conv_x6_weight_dims(K, M)
        shape = (kp // 32, 4, 2 if f16x3 else 1, mp, 8)
        ref, out = (torch.zeros(shape, dtype=torch.float16, device=cuda) for _ in range(2))
        rsc, osc = (torch.zeros(mp, device=cuda) for _ in range(2))
        if f16x3:
            assert lib.tcam_pack_weight_f16x3(w.data_ptr(), ref.data_ptr(), rsc.data_ptr(), mode,
                                              co, ci, kh, kw, c0, sel, cpad,
                                              kdiv.data_ptr() if kdiv is not None else None,
                                              _st()) == 0
        else:
            assert lib.tcam_pack_weight_f16(w.data_ptr(), ref.data_ptr(), mode, co, ci, kh, kw,
                                            c0, sel, cpad, _st()) == 0
        it.w, it.out, it.wscale = w.data_ptr(), out.data_ptr(), osc.data_ptr()
        it.kdiv = kdiv.data_ptr() if kdiv is not None else None
        it.mode, it.CoutW, it.CtotW, it.KH, it.KW = mode, co, ci, kh, kw
        it.c0, it.cout_sel, it.cin_pad = c0, sel, cpad
        refs.append((ref, rsc))
        outs.append((out, osc))
        keep.append((w, kdiv))
    table = torch.empty(int(lib.tcam_pack_table_bytes(len(specs))), dtype=torch.uint8, device=cuda)
    for rep in range(2):
        if rep:   # new weights, same table: the per-item packs again, then the batched call
            for (w, kdiv), it, (ref, rsc), (co, ci, kh, kw, mode, c0, sel, cpad) in zip(
                    keep, items, refs, specs):
                w.mul_(-1.5)
                if f16x3:
                    lib.tcam_pack_weight_f16x3(w.data_ptr(), ref.data_ptr(), rsc.data_ptr(), mode,
                                               co, ci, kh, kw, c0, sel, cpad,
                                               kdiv.data_ptr() if kdiv is not None else None,
                                               _st())
                else:
                    lib.tcam_pack_weight_f16(w.data_ptr(), ref.data_ptr(), mode, co, ci, kh, kw,
                                             c0, sel, cpad, _st())
        assert lib.tcam_pack_weights(items, len(specs), f16x3, table.data_ptr(), _st()) == 0
        torch.cuda.synchronize()
        for (ref, rsc), (out, osc) in zip(refs, outs):
            assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
            if f16x3:
                assert torch.equal(osc, rsc)
