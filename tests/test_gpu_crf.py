"""GPU parity of the permutohedral bilateral filter (csrc/bilateral.hip) against the
REFERENCE filter compiled from its own sources (oracle/_ref) and the reference's
golden vectors: bit-exact outputs, plus the DenseCRFLoss forward/backward."""
import os

import numpy as np
import pytest
import torch

from oracle import crf_ref as R
from tcam_wsol_video_amd import crf

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden", "crf_bilateral.npz")


def _smooth_img(rng, n, h, w, noise=6.0):
    yy, xx = np.mgrid[0:h, 0:w]
    base = 128 + 100 * np.sin(xx / 17.0 + rng.random()) * np.cos(yy / 23.0)
    img = np.stack([base, 0.7 * base + 30, 255 - base], 0)[None].repeat(n, 0)
    return (img + rng.normal(0, noise, img.shape)).clip(0, 255).astype(np.float32)


def _oracle(img, seg, sr, sx, dim=0):
    if R.ref_available("xy" if dim == 0 else "color"):
        return R.ref_colorbilateral(img, seg, sr, dim) if dim else R.ref_bilateral(img, seg, sr, sx)
    return R.port_bilateral(img, seg, sr, sx, dim=dim)


def test_golden_bitexact(cuda):
    d = np.load(G)
    names = sorted({k.split("_")[0] for k in d.files})
    for nm in names:
        n, k, h, w, sr, sx = d[f"{nm}_meta"]
        kind = str(d[f"{nm}_kind"])
        img = torch.from_numpy(d[f"{nm}_img"]).to(cuda)
        seg = torch.from_numpy(d[f"{nm}_seg"]).to(cuda)
        if kind == "xy":
            out = crf.bilateral_filter(img, seg, sr, sx, check_range=True)
        else:
            out = crf.color_bilateral_filter(img, seg, sr, int(kind[-1]), check_range=True)
        assert np.array_equal(out.cpu().numpy(), d[f"{nm}_out"]), nm


@pytest.mark.parametrize("n,k,h,w,sr,sx", [
    (1, 2, 224, 224, 15.0, 100.0),     # the TCAM configuration (README.md:327-331)
    (4, 2, 224, 224, 15.0, 100.0),
    (3, 1, 57, 43, 15.0, 100.0),       # H*W % 4 != 0
    (2, 5, 64, 80, 8.0, 12.0),
    (1, 8, 33, 31, 30.0, 7.0),
    (2, 2, 96, 96, 2.0, 3.0),          # fine lattice: many vertices
    (1, 2, 1, 1, 15.0, 100.0),
])
def test_bilateral_bitexact_vs_reference(cuda, n, k, h, w, sr, sx):
    rng = np.random.default_rng(n * 1000 + h)
    img = _smooth_img(rng, n, h, w)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    ref = _oracle(img, seg, sr, sx)
    out = crf.bilateral_filter(torch.from_numpy(img).to(cuda), torch.from_numpy(seg).to(cuda),
                               sr, sx, check_range=True).cpu().numpy()
    assert np.array_equal(out, ref), float(np.abs(out - ref).max())


def test_bilateral_merge_fallback_mixed_batch(cuda):
    """One call over a flat frame (few vertices: one LDS merge per image part) and a
    noise frame at a fine colour scale (far more vertices than the merge table holds: its
    parts split into hash sub-parts) — both bit-identical to the reference."""
    rng = np.random.default_rng(123)
    n, k, h, w = 2, 2, 128, 128
    img = _smooth_img(rng, n, h, w)
    img[0] = img[0].mean()                  # a flat frame: a handful of vertices
    img[1] = (rng.random((3, h, w)) * 255).astype(np.float32)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    ref = _oracle(img, seg, 4.0, 100.0)
    out = crf.bilateral_filter(torch.from_numpy(img).to(cuda), torch.from_numpy(seg).to(cuda),
                               4.0, 100.0, check_range=True).cpu().numpy()
    assert np.array_equal(out, ref), float(np.abs(out - ref).max())
    hdr = crf._workspace(torch.device(cuda), n, k, h, w, 5)[:16].view(torch.int32).cpu()
    assert 1 <= int(hdr[2]) <= 8   # only parts of the noise frame split


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_colorbilateral_bitexact_vs_reference(cuda, dim):
    rng = np.random.default_rng(dim)
    n, k, h, w = 2, 2, 61, 47
    img = (rng.random((n, 3, h, w)) * 255).astype(np.float32)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    ref = _oracle(img, seg, 15.0, 0.0, dim=dim)
    out = crf.color_bilateral_filter(torch.from_numpy(img).to(cuda),
                                     torch.from_numpy(seg).to(cuda), 15.0, dim,
                                     check_range=True).cpu().numpy()
    assert np.array_equal(out, ref)


def test_uniform_image_long_segments(cuda):
    # every pixel in a few simplices: per-vertex segments of thousands of entries
    n, k, h, w = 1, 2, 128, 128
    img = np.full((n, 3, h, w), 77.0, np.float32)
    seg = np.random.default_rng(5).random((n, k, h, w)).astype(np.float32)
    ref = _oracle(img, seg, 15.0, 1000.0)
    out = crf.bilateral_filter(torch.from_numpy(img).to(cuda), torch.from_numpy(seg).to(cuda),
                               15.0, 1000.0).cpu().numpy()
    assert np.array_equal(out, ref)


def test_deterministic_and_linear(cuda):
    rng = np.random.default_rng(11)
    img = torch.from_numpy(_smooth_img(rng, 3, 80, 72)).to(cuda)
    seg = torch.rand(3, 2, 80, 72, device=cuda)
    a = crf.bilateral_filter(img, seg, 15.0, 100.0)
    b = crf.bilateral_filter(img, seg, 15.0, 100.0)
    assert torch.equal(a, b)
    # per-image independence: filtering frame 1 alone gives the same result
    c = crf.bilateral_filter(img[1:2], seg[1:2].contiguous(), 15.0, 100.0)
    assert torch.equal(a[1:2], c)


def test_host_compat_symbol(cuda):
    rng = np.random.default_rng(2)
    n, k, h, w = 2, 2, 30, 26
    img = _smooth_img(rng, n, h, w)
    seg = rng.random((n, k, h, w)).astype(np.float32)
    outs = np.zeros(n * k * h * w, np.float32)
    crf.bilateralfilter_batch(img.reshape(-1), seg.reshape(-1), outs, n, k, h, w, 15.0, 100.0)
    assert np.array_equal(outs.reshape(n, k, h, w), _oracle(img, seg, 15.0, 100.0))
    outs2 = np.zeros_like(outs)
    crf.colorbilateralfilter_batch(img.reshape(-1), seg.reshape(-1), outs2, n, k, h, w, 15.0, 3)
    assert np.array_equal(outs2.reshape(n, k, h, w), _oracle(img, seg, 15.0, 0.0, dim=3))


def test_dense_crf_loss_forward_backward(cuda):
    """DenseCRFLoss (crf/dense_crf_loss.py:33-133): loss = w * -sum(S*AS)/N,
    grad_S = w * -2 AS / N; checked in fp64 against the reference filter's AS."""
    rng = np.random.default_rng(7)
    n, h, w = 3, 64, 64
    img = _smooth_img(rng, n, h, w)
    logits = torch.randn(n, 2, h, w, device=cuda, requires_grad=True)
    S = torch.softmax(logits, 1)
    weight = 2e-9 * 1e6
    loss_mod = crf.DenseCRFLoss(weight=weight, sigma_rgb=15.0, sigma_xy=100.0, scale_factor=1.0)
    loss = loss_mod(torch.from_numpy(img), S)
    loss.backward()
    S_np = S.detach().cpu().numpy()
    AS = _oracle(img, S_np, 15.0, 100.0).astype(np.float64)
    exp = weight * -(S_np.astype(np.float64) * AS).sum() / n
    assert abs(float(loss.detach()) - exp) <= 1e-5 * abs(exp)
    # d loss / d logits through softmax with grad_S = weight * -2 AS / N
    S64 = torch.from_numpy(S_np.astype(np.float64))
    gS = torch.from_numpy(weight * -2.0 * AS / n)
    g_exp = S64 * (gS - (gS * S64).sum(1, keepdim=True))
    np.testing.assert_allclose(logits.grad.cpu().double().numpy(), g_exp.numpy(),
                               rtol=1e-4, atol=2e-5 * float(g_exp.abs().max()))


def test_color_dense_crf_loss(cuda):
    rng = np.random.default_rng(8)
    n, h, w = 2, 40, 50
    img = (rng.random((n, 3, h, w)) * 255).astype(np.float32)
    S = torch.softmax(torch.randn(n, 2, h, w, device=cuda), 1).requires_grad_(True)
    loss = crf.ColorDenseCRFLoss(weight=1.0, sigma_rgb=15.0, scale_factor=1.0)(
        torch.from_numpy(img), S)
    loss.backward()
    AS = _oracle(img, S.detach().cpu().numpy(), 15.0, 0.0, dim=3).astype(np.float64)
    exp = -(S.detach().cpu().double().numpy() * AS).sum() / n
    assert abs(float(loss.detach()) - exp) <= 1e-5 * abs(exp)
    np.testing.assert_allclose(S.grad.cpu().double().numpy(), -2.0 * AS / n, rtol=1e-6, atol=0)


def test_concurrent_streams_use_separate_workspaces(cuda):
    """Two streams filtering at the same time (pipelined clips) get the same bits as one
    stream: each stream has its own lattice workspace."""
    g = torch.Generator().manual_seed(11)
    imgs = [(torch.rand(4, 3, 96, 80, generator=g) * 255).round().to(cuda) for _ in range(2)]
    segs = [torch.rand(4, 2, 96, 80, generator=g).to(cuda) for _ in range(2)]
    ref = [crf.bilateral_filter(i, s, 15.0, 100.0) for i, s in zip(imgs, segs)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    outs = [[], []]
    for _ in range(3):
        for j, st in enumerate(streams):
            with torch.cuda.stream(st):
                outs[j].append(crf.bilateral_filter(imgs[j], segs[j], 15.0, 100.0))
    torch.cuda.synchronize()
    for j in range(2):
        for o in outs[j]:
            assert torch.equal(o, ref[j])


def test_prepared_lattice_on_a_side_stream_is_bitexact(cuda):
    """tcam_bilateral_prepare on a side stream + tcam_bilateral_apply on the current one
    == tcam_bilateral_batch, over consecutive prepares from the workspace pool (the
    trainer builds the next lattice while the previous one is still to be applied)."""
    rng = np.random.default_rng(17)
    n, k, h, w = 3, 2, 72, 88
    side = torch.cuda.Stream()
    lats, refs, segs = [], [], []
    for i in range(3):
        img = torch.from_numpy(_smooth_img(rng, n, h, w)).to(cuda)
        seg = torch.rand(n, k, h, w, device=cuda)
        refs.append(crf.bilateral_filter(img, seg, 15.0, 100.0))
        lats.append(crf.PreparedLattice(img, k, 15.0, 100.0, stream=side))
        segs.append(seg)
    for lat, seg, ref in zip(lats, segs, refs):
        assert torch.equal(lat.apply(seg, check_range=True), ref)
    with pytest.raises(RuntimeError, match="already applied"):
        lats[0].apply(segs[0])
    # a pooled workspace is reused after its apply: same bits again
    img = torch.from_numpy(_smooth_img(np.random.default_rng(5), n, h, w)).to(cuda)
    seg = torch.rand(n, k, h, w, device=cuda)
    assert torch.equal(crf.PreparedLattice(img, k, 15.0, 100.0, stream=side).apply(seg),
                       crf.bilateral_filter(img, seg, 15.0, 100.0))
