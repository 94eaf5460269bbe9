"""Parity at the BASELINE configurations' real sizes (BASELINE.json configs[1]-[4]):

* ResNet50-TCAM, the bench's own 32-frame 224^2 clip and weights, through the bench's
  CAMComputer configuration (2 forward streams, 1000 taus): CAM <= 1e-4 and logits
  <= 1e-3 vs the oracle; BoxEvaluator counters bit-exact vs the oracle evaluator fed
  the same uint8 CAMs (inference_wsol.py:332-346, wsol_metrics.py:295-370);
* VGG16-TCAM on a 32-frame 224^2 clip vs the oracle, and the CRF bilateral filter of
  those 32 frames' softmaxed fcams bit-exact vs the reference filter compiled from its
  own sources (dense_crf_loss.py:42-66, bilateralfilter.cpp:42-55);
* InceptionV3-TCAM, an 8-frame 299^2 shard, vs the oracle;
* the > 2 GiB frame-chunked x6 convolution (taken by ResNet50's layer4 at the training
  batch of 256 frames) bit-exact vs per-chunk single launches, and the 256-frame
  training forward / seg-head gradient vs the oracle and torch.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import bbox_ref as BR
from oracle import crf_ref as CR
from oracle import model_ref as R
from tcam_wsol_video_amd import crf, ops
from tcam_wsol_video_amd.inference import CAMComputer
from tcam_wsol_video_amd.models import build_inceptionv3_tcam, build_r50_tcam, build_vgg16_tcam
from tcam_wsol_video_amd.ops import ConvSrc

pytestmark = pytest.mark.gpu
CAM_TOL = 1e-4      # north_star: CAMs within 1e-4 fp32 of the reference CPU path
LOGIT_TOL = 1e-3


def _clip(frames, seed, size):
    import bench
    return bench.make_clip(frames, seed=seed, size=size)


def _u8_close(u8, u8_ref):
    d = np.abs(u8.astype(int) - u8_ref.astype(int))
    assert d.max() <= 1 and np.mean(d != 0) < 1e-3


def _forward_vs_oracle(model, x, cuda, want_ref=False):
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        logits, fcams, _ = model(x.to(cuda))
    torch.cuda.synchronize()
    lo_ref, fc_ref, _ = R.tcam_forward(sd, x)
    cam_ref = R.segmentation_cam(fc_ref)
    assert (logits.cpu() - lo_ref).abs().max().item() < LOGIT_TOL
    assert (model.cam.cpu() - cam_ref).abs().max().item() < CAM_TOL
    _u8_close(model.cam_u8.cpu().numpy(), R.quantize_u8(cam_ref.double().numpy()))
    if want_ref:
        return logits, fcams, lo_ref, cam_ref
    return logits, fcams


def _oracle_own_evaluator(cam_ref, lo_ref, targets, gt, taus):
    """The reference's evaluation of its OWN CAMs, end to end: the oracle's fp32 CAM as the
    float64 scoremap t2n hands BoxEvaluator (inference_wsol.py:332-346: a same-size
    interpolate is the identity), its own logits' stable descending order
    (inference_wsol.py:368-369), then compute_bboxes_from_scoremaps' uint8 quantisation,
    threshold sweep and IoU counters (wsol_metrics.py:127-197, 295-370) in the oracle."""
    ref = BR.BoxEvaluatorRef(taus)
    for b in range(cam_ref.shape[0]):
        _, order = torch.sort(lo_ref[b], descending=True, stable=True)
        ref.accumulate(cam_ref[b].double().numpy(), gt[b].numpy(), int(targets[b]),
                       order.numpy())
    return ref


def _assert_counters_equal(dev, ref, what):
    """north_star: bbox IoU bit-identical on the same frames -> every (IoU threshold, tau)
    counter of the device evaluator equals the oracle evaluator's; on a mismatch the message
    lists the differing cells."""
    bad = []
    for thr in ref.iou_threshold_list:
        for name in ("num_correct", "num_correct_top1", "num_correct_top5"):
            a, b = getattr(dev, name)[thr], getattr(ref, name)[thr]
            for i in np.nonzero(a != b)[0][:20]:
                bad.append((name, thr, int(i), float(a[i]), float(b[i])))
    assert not bad, (what, bad)


def test_r50_tcam_bench_clip_vs_oracle(cuda):
    import bench
    x, targets, gt = _clip(32, 1000, 224)          # rank 0's bench clip
    model = build_r50_tcam(seed=0).to(cuda)         # the bench's weights
    comp = CAMComputer(model, cam_curve_interval=0.001, device=cuda, fwd_streams=2)
    u8 = comp.evaluate_batch(x.to(cuda), targets.to(cuda), gt.to(cuda))
    comp.synchronize()
    acc = comp.compute_and_evaluate()
    u8 = u8.cpu().numpy()
    logits, _, lo_ref, cam_ref = _forward_vs_oracle(model, x, cuda, want_ref=True)
    assert np.array_equal(model.cam_u8.cpu().numpy(), u8)   # pipelined == plain forward
    ref = BR.BoxEvaluatorRef(comp.cam_threshold_list)
    lo = logits.cpu()
    for b in range(32):
        sm = np.minimum((u8[b].astype(np.float64) + 0.5) / 255.0, 1.0)
        _, order = torch.sort(lo[b], descending=True, stable=True)
        ref.accumulate(sm, gt[b].numpy(), int(targets[b]), order.numpy())
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(comp.evaluator.num_correct[thr], ref.num_correct[thr])
        np.testing.assert_array_equal(comp.evaluator.num_correct_top1[thr],
                                      ref.num_correct_top1[thr])
        np.testing.assert_array_equal(comp.evaluator.num_correct_top5[thr],
                                      ref.num_correct_top5[thr])
    assert acc == ref.compute()
    # end to end: the oracle's own CAMs and logits (not the device's uint8 CAMs) through the
    # oracle evaluator give the same counters, BoxAcc, best tau and top-1/5 localisation
    own = _oracle_own_evaluator(cam_ref, lo_ref, targets, gt, comp.cam_threshold_list)
    _assert_counters_equal(comp.evaluator, own, "r50 bench clip, oracle's own CAMs")
    assert acc == own.compute()
    assert comp.evaluator.best_tau_list == own.best_tau_list
    assert comp.evaluator.top1 == own.top1 and comp.evaluator.top5 == own.top5
    assert bench.GFLOP_PER_FRAME == 55.29


def test_vgg16_tcam_clip_and_crf_vs_oracle(cuda):
    import bench
    x, targets, gt = _clip(32, 1001, 224)
    model = build_vgg16_tcam(seed=0).to(cuda)
    _, fcams, lo_ref, cam_ref = _forward_vs_oracle(model, x, cuda, want_ref=True)
    # end-to-end boxes: device CAM -> device sweep vs the oracle evaluator on its own CAMs
    comp = CAMComputer(model, cam_curve_interval=0.001, device=cuda)
    comp.evaluate_batch(x.to(cuda), targets.to(cuda), gt.to(cuda))
    acc = comp.compute_and_evaluate()
    own = _oracle_own_evaluator(cam_ref, lo_ref, targets, gt, comp.cam_threshold_list)
    _assert_counters_equal(comp.evaluator, own, "vgg16 clip, oracle's own CAMs")
    assert acc == own.compute() and comp.evaluator.best_tau_list == own.best_tau_list
    raw = ((x * torch.tensor(bench.IMNET_STD)[None, :, None, None] +
            torch.tensor(bench.IMNET_MEAN)[None, :, None, None]) * 255).clamp(0, 255).round()
    seg = torch.softmax(fcams, 1).contiguous()
    AS = crf.bilateral_filter(raw.to(cuda), seg, 15.0, 100.0, check_range=True).cpu().numpy()
    img_np, seg_np = raw.numpy().astype(np.float32), seg.cpu().numpy()
    ref = (CR.ref_bilateral(img_np, seg_np, 15.0, 100.0) if CR.ref_available("xy")
           else CR.port_bilateral(img_np, seg_np, 15.0, 100.0))
    assert np.array_equal(AS, ref)


def test_inceptionv3_tcam_shard_vs_oracle(cuda):
    x, targets, gt = _clip(8, 1002, 299)
    model = build_inceptionv3_tcam(seed=0).to(cuda)
    _, _, lo_ref, cam_ref = _forward_vs_oracle(model, x, cuda, want_ref=True)
    comp = CAMComputer(model, cam_curve_interval=0.001, device=cuda)
    u8 = comp.evaluate_batch(x.to(cuda), targets.to(cuda), gt.to(cuda)).cpu().numpy()
    acc = comp.compute_and_evaluate()
    own = _oracle_own_evaluator(cam_ref, lo_ref, targets, gt, comp.cam_threshold_list)
    _assert_counters_equal(comp.evaluator, own, "inceptionv3 299 shard, oracle's own CAMs")
    assert acc == own.compute() and comp.evaluator.best_tau_list == own.best_tau_list
    boxes, vmax = ops.bbox_levels(torch.from_numpy(u8).to(cuda))
    boxes, vmax = boxes.cpu().numpy(), vmax.cpu().numpy()
    for b in range(8):
        levels = np.arange(vmax[b])
        np.testing.assert_array_equal(boxes[b][levels], BR.boxes_for_levels(u8[b], levels))


def _chunk_frames(per_frame_bytes):
    lim = 0x80000000 - (1 << 20)      # csrc/conv_x6.hip: OOB - 1 MiB
    return max(1, lim // per_frame_bytes)


def test_frame_chunked_conv_bit_exact_vs_per_chunk_launches(cuda):
    """ResNet50 layer4 conv3 shape (512 -> 2048, 1x1, 28^2, residual + ReLU) at the training
    batch of 256 frames: 256 x 9.6 MB > 2 GiB, so tcam_conv2d_x6 runs it as frame-chunked
    launches; each chunk must equal a single launch over the same frames."""
    B, C, Co, H = 256, 512, 2048, 28
    fc = _chunk_frames(H * H * Co * 6)
    assert fc < B
    g = torch.Generator().manual_seed(0)
    x = ops.s3_from_nchw(torch.randn(B, C, H, H, generator=g).to(cuda))
    res = ops.s3_from_nchw(torch.randn(B, Co, H, H, generator=g).to(cuda))
    w = (torch.randn(Co, C, 1, 1, generator=g) / np.sqrt(C)).to(cuda)
    bias = torch.randn(Co, generator=g).to(cuda)
    wt = ops.pack_conv_weight_x6([w])
    full = ops.conv2d_x6([ConvSrc(x)], wt, bias, Co, H, H, 1, 0, True, residual=res)
    for b0 in range(0, B, fc):
        b1 = min(B, b0 + fc)
        part = ops.conv2d_x6([ConvSrc(x[b0:b1].contiguous())], wt, bias, Co, H, H, 1, 0, True,
                             residual=res[b0:b1].contiguous())
        assert torch.equal(full[b0:b1], part), (b0, b1)
    # and a few frames against fp64 (the x6 arithmetic bound, test_gpu_x6.py)
    for b in (0, fc - 1, fc, B - 1):
        xs = ops.s3_to_nchw(x[b:b + 1].contiguous()).double()
        rs = ops.s3_to_nchw(res[b:b + 1].contiguous()).double()
        ref = (F.conv2d(xs, w.double(), bias.double()) + rs).clamp_min(0)
        absd = F.conv2d(xs.abs(), w.double().abs()) + rs.abs() + bias.double().abs()[:, None, None]
        got = ops.s3_to_nchw(full[b:b + 1].contiguous()).double()
        assert bool(((got - ref).abs() <= 2e-6 * (absd + 1.0)).all()), b


def test_training_forward_at_256_frames(cuda):
    """configs[2] per-GPU batch (8 clips x 32 frames): the frozen encoder runs its layer4
    through the frame-chunked convs; logits of frames on both sides of the chunk boundary
    vs the oracle, the decoder's batch-statistics BN vs torch over all 256 frames, and the
    seg-head weight/bias gradients (12.8 M pixels) vs torch fp32."""
    from tcam_wsol_video_amd.training import DecoderTrainer
    x, _, _ = _clip(256, 1003, 224)
    model = build_r50_tcam(seed=5).to(cuda)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    tr = DecoderTrainer(model)
    xd = x.to(cuda)
    cl_logits, fcams, st = tr.forward(xd)
    torch.cuda.synchronize()
    fc = _chunk_frames(28 * 28 * 2048 * 6)
    pick = [0, fc - 1, fc, 255]
    lo_ref, _, _ = R.tcam_forward(sd, x[pick])
    assert (cl_logits[pick].cpu() - lo_ref).abs().max().item() < LOGIT_TOL
    # batch-statistics BN of the first decoder conv over all 256 frames
    blk = st["blocks"][0]
    y = ops.s3_to_nchw(blk["y1"]).double()
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3), unbiased=False)
    eps = model.decoder.blocks[0].conv1[1].eps
    assert torch.allclose(blk["m1"].double(), mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(blk["i1"].double(), 1.0 / torch.sqrt(var + eps), rtol=1e-5)
    del y
    # seg-head gradients from a dF over all 256 x 224^2 pixels
    g = torch.Generator(device=cuda).manual_seed(1)
    dF = torch.randn(fcams.shape, device=cuda, generator=g) * 1e-3
    tr.grad.zero_()
    tr.backward(dF, st)
    torch.cuda.synchronize()
    x16 = ops.s3_to_nchw(st["dec_out"])
    wref = torch.nn.grad.conv2d_weight(x16, tr.seg.weight.shape, dF, padding=1)
    gw = tr.g(tr.seg.weight)
    rel = ((gw - wref).norm() / wref.norm()).item()
    assert rel < 1e-4, rel
    gb = tr.g(tr.seg.bias).double()
    assert torch.allclose(gb, dF.double().sum(dim=(0, 2, 3)), rtol=1e-5, atol=1e-7)
    assert torch.isfinite(tr.grad).all()
    # every trainable decoder gradient against the same backward with its parameter
    # reductions in fp64: torch fp32 autograd over the same frozen-encoder features
    # (oracle/train_ref.decoder_train on the device, the device forward's ReLU branches)
    # supplies each layer's input and output gradient, and the up-to-12.8 M-pixel sums that
    # form the conv-weight / BN-gamma / BN-beta / bias gradients are redone in fp64 (an fp32
    # sum of that length is itself only ~1e-4 accurate): norm-relative <= 1e-4 per parameter.
    # (The BN-beta sums cancel heavily — measured up to 6.7e-5 norm-relative — and the
    # per-element dy of a BN backward is itself a cancelling difference, so neither a 2e-5
    # norm bound nor an element bound by the sum of |terms| is met by two fp32 chains that
    # differ only in rounding.)
    from oracle import train_ref as T
    from tcam_wsol_video_amd.models import _encoder_plan_x6
    from tcam_wsol_video_amd.models import _precision
    prec = _precision(model)   # the trainer's frozen-encoder precision
    enc = model._plan_get("enc_" + prec, lambda: _encoder_plan_x6(model.encoder, cuda, prec),
                          model.encoder)
    with torch.no_grad():
        feats = [None] + [ops.s3_to_nchw(f) for f in enc.forward(xd)[1:]]
    masks = {}
    for i, b in enumerate(st["blocks"]):
        masks[f"decoder.blocks.{i}.conv1"] = ops.s3_to_nchw(b["a1"]) > 0
        masks[f"decoder.blocks.{i}.conv2"] = ops.s3_to_nchw(b["a2"]) > 0
    named = dict(model.named_parameters())
    keys = [k for k in named if k.startswith(("decoder.", "segmentation_head."))]
    p = {k: named[k].detach().clone().requires_grad_(True) for k in keys}
    bufs = {k: v.detach().clone() for k, v in model.state_dict().items()
            if k.startswith("decoder.") and k.endswith(("running_mean", "running_var"))}
    convs, bns = {}, {}
    name_of = {id(v): k for k, v in p.items()}
    conv0, bn0 = F.conv2d, T._bn_train

    def conv_rec(x, w, b=None, *a, **kw):
        y = conv0(x, w, b, *a, **kw)
        if id(w) in name_of:
            y.retain_grad()
            convs[name_of[id(w)]] = (x, y, kw.get("padding", a[1] if len(a) > 1 else 0))
        return y

    def bn_rec(y, w, b, rm, rv, eps=1e-5, momentum=0.1):
        z = bn0(y, w, b, rm, rv, eps, momentum)
        z.retain_grad()
        bns[name_of[id(w)]] = (y, z, eps)
        return z

    F.conv2d, T._bn_train = conv_rec, bn_rec
    try:
        d = T.decoder_train(p, bufs, feats, n_blocks=5, center=False, masks=masks)
        fc_ref = F.conv2d(d, p["segmentation_head.0.weight"], p["segmentation_head.0.bias"],
                          padding=1)
    finally:
        F.conv2d, T._bn_train = conv0, bn0
    assert (fc_ref - fcams).abs().max().item() <= 1e-4 * fc_ref.abs().max().item()
    (fc_ref * dF).sum().backward()
    ref64 = {}
    for wname, (x, y, pad) in convs.items():
        gy = y.grad.double()
        kh, kw = p[wname].shape[2:]
        xp = F.pad(x.detach().double(), (pad, pad, pad, pad))
        H, W = y.shape[2:]
        g = torch.empty(p[wname].shape, dtype=torch.float64, device=cuda)
        for i in range(kh):
            for j in range(kw):
                g[:, :, i, j] = torch.einsum("bchw,bohw->oc", xp[:, :, i:i + H, j:j + W], gy)
        ref64[wname] = g
        if wname.replace("weight", "bias") in p:
            ref64[wname.replace("weight", "bias")] = gy.sum(dim=(0, 2, 3))
        del xp, gy
    for wname, (y, z, eps) in bns.items():
        yd = y.detach().double()
        mean = yd.mean(dim=(0, 2, 3), keepdim=True)
        inv = 1.0 / torch.sqrt(yd.var(dim=(0, 2, 3), unbiased=False, keepdim=True) + eps)
        gz = z.grad.double()
        ref64[wname] = (gz * (yd - mean) * inv).sum(dim=(0, 2, 3))
        ref64[wname.replace("weight", "bias")] = gz.sum(dim=(0, 2, 3))
        del yd, gz
    assert sorted(ref64) == sorted(keys), sorted(set(keys) ^ set(ref64))
    errs = {k: ((tr.g(named[k]).double() - ref64[k]).norm() / ref64[k].norm()).item()
            for k in keys}
    worst = max(errs, key=errs.get)
    assert errs[worst] <= 1e-4, (worst, errs[worst])
