"""GPU parity of every C-ABI op against a CPU reference (PyTorch fp32 for the
floating-point kernels, the oracle for the integer bbox path)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from scipy import ndimage

from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.ops import ConvSrc

pytestmark = pytest.mark.gpu


def _rel_close(out, ref, tol=2e-5):
    out = out.detach().cpu().double()
    ref = ref.detach().cpu().double()
    scale = ref.abs().max().item() + 1e-12
    err = (out - ref).abs().max().item()
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


CONV_CASES = [
    # (B, [(C, H, W, stride, up2)], Cout, KS, pad, relu, residual)
    (2, [(3, 37, 41, 2, 0)], 64, 7, 3, True, False),          # stem-like, odd sizes
    (2, [(64, 14, 14, 1, 0)], 64, 1, 0, True, False),
    (2, [(64, 14, 14, 1, 0)], 256, 1, 0, False, True),        # conv3 + identity
    (3, [(32, 15, 15, 2, 0)], 32, 3, 1, True, False),         # strided 3x3
    (2, [(128, 7, 7, 1, 0)], 128, 3, 1, True, False),
    (2, [(128, 7, 7, 1, 0), (96, 14, 14, 2, 0)], 512, 1, 0, True, False),  # conv3+downsample
    (2, [(48, 7, 9, 1, 1), (40, 14, 18, 1, 0)], 64, 3, 1, True, False),    # decoder up2+skip
    (2, [(32, 9, 9, 1, 1)], 16, 3, 1, True, False),           # last decoder block
    (1, [(200, 5, 6, 1, 0)], 132, 3, 1, True, False),         # ragged M, K tails
    (2, [(64, 28, 28, 1, 1), (32, 56, 56, 1, 0)], 64, 3, 1, True, False),  # fast path, up2
    (4, [(256, 14, 14, 1, 0)], 512, 3, 1, True, False),       # fast path, multi-wave
    (2, [(64, 16, 16, 1, 0), (64, 32, 32, 2, 0)], 256, 1, 0, True, False),  # fast ds fusion
    (3, [(96, 9, 11, 1, 0)], 40, 3, 1, False, True),          # BM=32/64 tiles, residual
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_matches_torch(cuda, case):
    B, srcs, cout, ks, pad, relu, use_res = case
    g = torch.Generator().manual_seed(hash(str(case)) % 1000)
    xs = [torch.randn(B, c, h, w, generator=g) for (c, h, w, s, u) in srcs]
    ws = [torch.randn(cout, c, ks, ks, generator=g) / np.sqrt(c * ks * ks)
          for (c, h, w, s, u) in srcs]
    bias = torch.randn(cout, generator=g)
    ref = None
    for x, w, (c, h, wd, s, u) in zip(xs, ws, srcs):
        xx = F.interpolate(x, scale_factor=2, mode="nearest") if u else x
        y = F.conv2d(xx.double(), w.double(), stride=s, padding=pad)
        ref = y if ref is None else ref + y
    ref = ref + bias.double()[None, :, None, None]
    Ho, Wo = ref.shape[2:]
    res = torch.randn(B, cout, Ho, Wo, generator=g) if use_res else None
    if res is not None:
        ref = ref + res.double()
    if relu:
        ref = ref.clamp_min(0)
    wt = ops.pack_conv_weight([w.to(cuda) for w in ws])
    out = ops.conv2d([ConvSrc(x.to(cuda), s, u) for x, (c, h, wd, s, u) in zip(xs, srcs)],
                     wt, bias.to(cuda), cout, Ho, Wo, ks, pad, relu,
                     residual=None if res is None else res.to(cuda))
    torch.cuda.synchronize()
    _rel_close(out, ref)


def test_maxpool(cuda):
    x = torch.randn(2, 5, 17, 22)
    out = ops.maxpool3x3s2(x.to(cuda))
    assert torch.equal(out.cpu(), F.max_pool2d(x, 3, 2, 1))


@pytest.mark.parametrize("hw,size", [((28, 28), (28, 28)), ((7, 5), (11, 9)), ((4, 4), (8, 8))])
def test_up2_resize(cuda, hw, size):
    x = torch.randn(2, 3, *hw)
    ref = F.interpolate(F.interpolate(x, scale_factor=2, mode="nearest"), size=size,
                        mode="bilinear", align_corners=True)
    out = ops.up2_resize(x.to(cuda), size)
    assert (out.cpu() - ref).abs().max().item() < 1e-5


def test_wgap(cuda):
    x = torch.randn(3, 2048, 28, 28)
    w = torch.randn(10, 2048) * 0.02
    b = torch.randn(10)
    ref = F.linear(F.adaptive_avg_pool2d(x, 1).flatten(1), w, b)
    out = ops.wgap(x.to(cuda), w.to(cuda), b.to(cuda))
    assert (out.cpu() - ref).abs().max().item() < 1e-4


def test_seghead_cam(cuda):
    x = torch.randn(2, 16, 33, 40)
    w = torch.randn(2, 16, 3, 3) * 0.2
    b = torch.randn(2)
    fc_ref = F.conv2d(x, w, b, padding=1)
    cam_ref = torch.softmax(fc_ref, 1)[:, 1]
    fc, cam, u8 = ops.seghead_cam(x.to(cuda), w.to(cuda), b.to(cuda))
    assert (fc.cpu() - fc_ref).abs().max().item() < 1e-4
    assert (cam.cpu() - cam_ref).abs().max().item() < 1e-5
    # u8 is exactly uint8(double(cam) * 255) of the kernel's own cam
    exp = (cam.cpu().double().numpy() * 255).astype(np.uint8)
    np.testing.assert_array_equal(u8.cpu().numpy(), exp)
    _, cam_a, _ = ops.seghead_cam(x.to(cuda), w.to(cuda), b.to(cuda), argmax=True)
    assert torch.equal(cam_a.cpu(), torch.argmax(fc_ref, 1).float())


def test_std_cam(cuda):
    from oracle import model_ref as R
    A = torch.relu(torch.randn(2, 64, 7, 7))
    fcw = torch.randn(5, 64)
    cls = torch.tensor([1, 3])
    low, cam, u8 = ops.std_cam(A.to(cuda), fcw.to(cuda), cls.to(cuda), (28, 28))
    sd = {"classification_head.fc.weight": fcw}
    for i in range(2):
        lo_ref, cam_ref = R.std_cam(sd, A[i], int(cls[i]), (28, 28))
        assert (low[i].cpu() - lo_ref).abs().max().item() < 1e-5
        assert np.abs(cam[i].cpu().double().numpy() - cam_ref).max() < 1e-5


@pytest.mark.parametrize("t", [0.0, 3.0])
def test_temporal_max(cuda, t):
    from oracle import model_ref as R
    cams = torch.rand(6, 28, 28)
    idx = torch.tensor([[0, 1, -1], [2, 3, 4], [5, -1, -1]])
    out = ops.temporal_max(cams.to(cuda), idx.to(cuda), t=t)
    for i in range(3):
        ref = R.temporal_max([cams[j] for j in idx[i].tolist() if j >= 0], t=t)
        assert (out[i].cpu() - ref).abs().max().item() < 1e-6


def test_topk_flags(cuda):
    logits = torch.tensor([[0.1, 0.5, 0.5, 0.2, 0.0, -1.0, 0.3],
                           [1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0]])
    target = torch.tensor([2, 5])
    t1, t5 = ops.topk_flags(logits.to(cuda), target.to(cuda))
    for b in range(2):
        _, order = torch.sort(logits[b], descending=True, stable=True)
        assert t1[b].item() == int(order[0].item() == target[b].item())
        assert t5[b].item() == int(target[b].item() in order[:5].tolist())


def _cams(kind, B, H, W, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(B):
        if kind == "smooth":
            f = ndimage.gaussian_filter(rng.random((H, W)), 6)
            f = (f - f.min()) / (f.max() - f.min() + 1e-12)
            out.append((f * rng.uniform(0.3, 1.0) * 255).astype(np.uint8))
        elif kind == "noise":
            out.append(rng.integers(0, 256, (H, W)).astype(np.uint8))
        elif kind == "binary":
            out.append(((rng.random((H, W)) < 0.6) * 255).astype(np.uint8))
        elif kind == "rings":
            # concentric rings around a random centre (levels of a few to hundreds of new
            # pixels, so runs of small levels on one wave alternate with block levels), a
            # plateau and a few isolated spikes
            yy, xx = np.mgrid[0:H, 0:W]
            cy, cx = rng.uniform(0, H), rng.uniform(0, W)
            d = np.hypot(yy - cy, xx - cx)
            f = 255 * (1 - d / (d.max() + 1e-9)) ** rng.uniform(0.5, 3.0)
            f[(yy // 7 + xx // 5) % 11 == 0] = 90
            f[rng.random((H, W)) < 0.002] = 250
            out.append(f.astype(np.uint8))
        elif kind == "blobs":
            f = ndimage.gaussian_filter(rng.random((H, W)), 2)
            out.append((255 * (f > np.median(f))).astype(np.uint8) // 2 +
                       (rng.integers(0, 2, (H, W)) * 100).astype(np.uint8))
        else:
            out.append(np.zeros((H, W), np.uint8))
    return np.stack(out)


@pytest.mark.parametrize("kind,H,W", [("smooth", 224, 224), ("noise", 224, 224),
                                      ("binary", 64, 80), ("blobs", 97, 131),
                                      ("zeros", 32, 32), ("smooth", 5, 3), ("rings", 160, 224),
                                      # > 256: the psi-only-LDS fill + large level kernel
                                      ("smooth", 299, 299), ("blobs", 300, 257),
                                      ("binary", 261, 320)])
def test_bbox_levels_bit_exact_vs_oracle(cuda, kind, H, W):
    from oracle import bbox_ref as BR
    u8 = _cams(kind, 3, H, W, seed=H * W)
    boxes, vmax = ops.bbox_levels(torch.from_numpy(u8).to(cuda))
    boxes, vmax = boxes.cpu().numpy(), vmax.cpu().numpy()
    for b in range(u8.shape[0]):
        assert vmax[b] == u8[b].max()
        levels = np.arange(vmax[b])
        if len(levels) == 0:
            continue
        ref = BR.boxes_for_levels(u8[b], levels)
        np.testing.assert_array_equal(boxes[b][levels], ref)


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("kind,H,W", [("smooth", 224, 224), ("noise", 224, 224),
                                      ("binary", 64, 80), ("blobs", 97, 131),
                                      ("smooth", 5, 3), ("blobs", 224, 200), ("zeros", 8, 8),
                                      ("binary", 224, 224), ("blobs", 1, 224), ("noise", 224, 1),
                                      ("rings", 224, 224), ("rings", 61, 97), ("rings", 224, 3)])
def test_bbox_incremental_levels_match_per_level_ccl(cuda, kind, H, W, variant):
    """The level sweeps for frames <= 224^2 — the sorted-list sweep (0, default) and the
    incremental sweep (2) — give exactly the boxes of the per-level CCL kernel on every level
    (which the test above pins to the oracle)."""
    from tcam_wsol_video_amd import _lib
    lib = _lib.load()
    u8 = torch.from_numpy(_cams(kind, 6, H, W, seed=H + W + 7)).to(cuda)
    try:
        lib.tcam_bbox_level_variant(1)
        b1, v1 = ops.bbox_levels(u8)
        lib.tcam_bbox_level_variant(variant)
        b0, v0 = ops.bbox_levels(u8)
    finally:
        lib.tcam_bbox_level_variant(0)
    assert torch.equal(v0, v1)
    valid = torch.arange(256, device=cuda)[None, :] < v0[:, None]
    assert torch.equal(b0 * valid[..., None], b1 * valid[..., None])


@pytest.mark.parametrize("kind,H,W", [("smooth", 224, 224), ("noise", 224, 224),
                                      ("blobs", 97, 131), ("smooth", 5, 3), ("binary", 256, 250),
                                      ("noise", 1, 200), ("blobs", 224, 1)])
def test_bbox_fill_variants_agree(cuda, kind, H, W):
    """The clamp-scan fill (default), the LDS-sweep fill and the register-line fill give the
    same psi, hence the same boxes on every level."""
    from tcam_wsol_video_amd import _lib
    lib = _lib.load()
    u8 = torch.from_numpy(_cams(kind, 5, H, W, seed=H * 3 + W)).to(cuda)
    outs = []
    try:
        for v in (0, 1, 2):
            lib.tcam_bbox_fill_variant(v)
            outs.append(ops.bbox_levels(u8))
    finally:
        lib.tcam_bbox_fill_variant(0)
    (b0, v0) = outs[0]
    valid = (torch.arange(256, device=cuda)[None, :] < v0[:, None])[..., None]
    for bx, vx in outs[1:]:
        assert torch.equal(vx, v0)
        assert torch.equal(bx * valid, b0 * valid)


def test_bbox_incremental_winner_key_drop(cuda):
    """The incremental sweep takes the winner over the roots touched at a level; when the
    previous winner's first-pixel key drops with no area gain (a new pixel joins it
    diagonally, before its first pixel in raster order) an untouched root of equal area
    takes over, which only the full fallback pass sees."""
    from oracle import bbox_ref as BR
    from tcam_wsol_video_amd import _lib
    u8 = np.zeros((2, 8, 12), np.uint8)
    u8[:, 2:4, 2:4] = 200    # A: first pixel 26, wins the tie at levels 150..199
    u8[:, 1:3, 8:10] = 200   # B: first pixel 20, same area
    u8[0, 1, 1] = 150        # joins A at level 149 with no area: A's key 26 -> 13
    lib = _lib.load()
    t = torch.from_numpy(u8).to(cuda)
    b0, v0 = ops.bbox_levels(t)
    try:
        lib.tcam_bbox_level_variant(1)
        b1, _ = ops.bbox_levels(t)
    finally:
        lib.tcam_bbox_level_variant(0)
    b0 = b0.cpu().numpy()
    for b in range(2):
        levels = np.arange(int(v0[b]))
        np.testing.assert_array_equal(b0[b][levels], BR.boxes_for_levels(u8[b], levels))
        np.testing.assert_array_equal(b0[b][levels], b1.cpu().numpy()[b][levels])
    assert tuple(b0[0][149]) == (8, 1, 10, 3)   # B (x0, y0, x0 + w, y0 + h)
    assert tuple(b0[0][150]) == (2, 2, 4, 4)    # A


def test_box_accumulate_matches_reference_evaluator(cuda):
    from oracle import bbox_ref as BR
    u8 = _cams("smooth", 4, 64, 64, seed=3)
    taus = list(np.arange(0, 1, 0.01))
    rng = np.random.default_rng(0)
    gts, targets, preds = [], [], []
    for b in range(4):
        x0, y0 = rng.integers(0, 30, 2)
        gts.append([[int(x0), int(y0), int(x0) + 20, int(y0) + 25], [5, 5, 60, 60]])
        targets.append(int(rng.integers(0, 10)))
        preds.append(rng.permutation(10))
    ref = BR.BoxEvaluatorRef(taus)
    for b in range(4):
        sm = np.minimum((u8[b].astype(np.float64) + 0.5) / 255.0, 1.0)
        ref.accumulate(sm, gts[b], targets[b], preds[b])
    from tcam_wsol_video_amd.metrics import BoxEvaluator
    ev = BoxEvaluator(taus, device=cuda)
    logits = torch.zeros(4, 10)
    for b in range(4):  # logits whose stable descending order is preds[b]
        logits[b, torch.from_numpy(preds[b])] = torch.arange(10, 0, -1).float()
    t1, t5 = ops.topk_flags(logits.to(cuda), torch.tensor(targets).to(cuda))
    ev.accumulate_batch(torch.from_numpy(u8).to(cuda),
                        torch.tensor(gts, dtype=torch.int32).to(cuda),
                        torch.full((4,), 2, dtype=torch.int32).to(cuda), t1, t5)
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(ev.num_correct[thr], ref.num_correct[thr])
        np.testing.assert_array_equal(ev.num_correct_top1[thr], ref.num_correct_top1[thr])
        np.testing.assert_array_equal(ev.num_correct_top5[thr], ref.num_correct_top5[thr])
    assert ev.compute() == ref.compute()


def test_compute_bboxes_from_scoremaps_api(cuda):
    from oracle import bbox_ref as BR
    from tcam_wsol_video_amd.metrics import compute_bboxes_from_scoremaps
    sm = ndimage.gaussian_filter(np.random.default_rng(5).random((224, 224)), 8)
    sm = (sm - sm.min()) / (sm.max() - sm.min())
    taus = list(np.arange(0, 1, 0.004))
    a, na = compute_bboxes_from_scoremaps(sm, taus, device=cuda)
    b, nb = BR.compute_bboxes_from_scoremaps(sm, taus)
    assert na == nb
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_box_evaluator_reference_signature_with_metadata(cuda, tmp_path):
    """B3: BoxEvaluator built from a split's metadata (GT boxes resized to 224 by
    resize_bbox, wsol_metrics.py:266-293) and fed one float64 scoremap per frame through
    the reference signature accumulate(scoremap, image_id, target, preds_ordered, bbox,
    bbox_status) (wsol_metrics.py:295-370) — counters and compute() equal the oracle's."""
    from oracle import bbox_ref as BR
    from tcam_wsol_video_amd.metrics import BoxEvaluator
    rng = np.random.default_rng(2)
    ids = [f"dog/data/0001/shots/00{k}/frame0001.jpg" for k in range(4)]
    sizes = [(480, 360), (450, 360), (500, 333), (224, 224)]
    boxes = {}
    with open(tmp_path / "image_ids.txt", "w") as f:
        f.write("\n".join(ids) + "\n")
    with open(tmp_path / "image_sizes.txt", "w") as f:
        f.write("\n".join(f"{i},{w},{h}" for i, (w, h) in zip(ids, sizes)) + "\n")
    with open(tmp_path / "localization.txt", "w") as f:
        for i, (w, h) in zip(ids, sizes):
            nb = 1 + int(rng.integers(0, 2))
            boxes[i] = []
            for _ in range(nb):
                x0, y0 = rng.uniform(0, w / 2), rng.uniform(0, h / 2)
                b = (x0, y0, x0 + rng.uniform(10, w / 2 - 1), y0 + rng.uniform(10, h / 2 - 1))
                boxes[i].append(b)
                f.write(f"{i},{b[0]},{b[1]},{b[2]},{b[3]}\n")
    taus = list(np.arange(0, 1, 0.004))
    ev = BoxEvaluator(taus, (30, 50, 70), metadata=str(tmp_path), device=cuda)
    ref = BR.BoxEvaluatorRef(taus)
    u8 = _cams("smooth", 4, 224, 224, seed=11)
    for k, i in enumerate(ids):
        sm = np.minimum((u8[k].astype(np.float64) + 0.5) / 255.0, 1.0)
        preds = rng.permutation(10)
        target = int(preds[k % 3 * 3])
        ev.accumulate(sm, i, target, preds, None, None)
        w, h = sizes[k]
        # utils/tools.py:231-250 resize_bbox (int() truncation) restated for the oracle
        gt = [(int(b[0] * 224 / w), int(b[1] * 224 / h), int(b[2] * 224 / w), int(b[3] * 224 / h))
              for b in boxes[i]]
        assert [tuple(g) for g in ev.gt_bboxes[i]] == gt
        ref.accumulate(sm, np.asarray(gt), target, preds)
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(ev.num_correct[thr], ref.num_correct[thr])
        np.testing.assert_array_equal(ev.num_correct_top1[thr], ref.num_correct_top1[thr])
        np.testing.assert_array_equal(ev.num_correct_top5[thr], ref.num_correct_top5[thr])
    assert ev.cnt == 4 and ev.compute() == ref.compute()
    with pytest.raises(ValueError):   # check_scoremap_validity (utils/wsol.py:63-78)
        ev.accumulate(np.full((224, 224), 1.5), ids[0], 0, np.arange(10), None, None)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 64, 200, 224, 255, 256])
def test_bbox_scan_line_matches_serial_sweep(cuda, n):
    """The wave-parallel clamp scan of one line equals the serial sweep
    x_i = max(u_i, min(psi_i, x_{i-1})), x_{-1} = -1 (forward, then backward)."""
    from tcam_wsol_video_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(n)
    for trial in range(20):
        u = rng.integers(0, 256, n)
        p = np.maximum(u, rng.integers(0, 256, n)) if trial % 2 else np.full(n, 255)
        for mode in (1, 0):
            x, ref = -1, p.copy()
            for i in range(n):
                x = max(u[i], min(ref[i], x))
                ref[i] = x
            if mode == 0:
                x = -1
                for i in range(n - 1, -1, -1):
                    x = max(u[i], min(ref[i], x))
                    ref[i] = x
            pt = torch.from_numpy(p.astype(np.uint8)).to(cuda)
            ut = torch.from_numpy(u.astype(np.uint8)).to(cuda)
            out = torch.zeros(n, dtype=torch.uint8, device=cuda)
            assert lib.tcam_bbox_scan_line(pt.data_ptr(), ut.data_ptr(), out.data_ptr(), n, mode,
                                           None) == 0
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"mode {mode}")


def test_bbox_levels_chunks_bit_identical(cuda):
    """The level sweep on 1..4 level ranges per frame (tcam_bbox_set_chunks: the evaluator's
    drain of its last clip runs on 4) gives the same boxes."""
    g = torch.Generator().manual_seed(11)
    base = torch.rand(6, 1, 28, 28, generator=g)
    cam = torch.nn.functional.interpolate(base, size=(224, 224), mode="bilinear",
                                          align_corners=False)[:, 0]
    cam = cam + 0.05 * torch.rand(6, 224, 224, generator=g)
    u8 = (cam / cam.amax(dim=(1, 2), keepdim=True) * 255).to(torch.uint8).to(cuda)
    ref, vref = ops.bbox_levels(u8)
    for c in (1, 2, 3, 4):
        b, v = ops.bbox_levels(u8, chunks=c)
        assert torch.equal(v, vref), c
        for f in range(u8.shape[0]):   # rows >= vmax are not written
            n = int(vref[f])
            assert torch.equal(b[f, :n], ref[f, :n]), (c, f)


def test_cam_computer_held_back_clip_counted(cuda):
    """CAMComputer holds each clip's sweep back until the next call; a counter read (the
    evaluator's flush hook), synchronize() and compute_and_evaluate() all launch it, so the
    pipelined counters equal the unpipelined ones."""
    from tcam_wsol_video_amd.inference import CAMComputer
    from tcam_wsol_video_amd.models import build_r50_tcam
    model = build_r50_tcam(seed=3).to(cuda)
    g = torch.Generator().manual_seed(5)
    clips = [torch.randn(4, 3, 64, 64, generator=g).to(cuda) for _ in range(3)]
    tg = torch.tensor([0, 1, 2, 3], device=cuda)
    gt = torch.tensor([[[5, 6, 40, 50]]] * 4, dtype=torch.int32, device=cuda)
    ref = CAMComputer(model, cam_curve_interval=0.01, device=cuda, overlap=False)
    for x in clips:
        ref.evaluate_batch(x, tg, gt)
    want = ref.compute_and_evaluate()
    comp = CAMComputer(model, cam_curve_interval=0.01, device=cuda, fwd_streams=2)
    for x in clips:
        comp.evaluate_batch(x, tg, gt)
    # a direct counter read flushes the held-back clip
    assert comp.evaluator.num_correct[50].tolist() == ref.evaluator.num_correct[50].tolist()
    assert comp.compute_and_evaluate() == want and comp.evaluator.cnt == 12
