"""GPU parity of the heterogeneous grouped convolution launch (tcam_conv2d_group,
csrc/conv_x6.hip conv_x6_group_kernel): up to four independent convolutions — own source,
weights, taps, pads and output slice each — in one grid.  Every member must equal, bit for
bit, the same convolution launched alone on the same tile (tcam_conv_x6_force_tile), must
match fp64 within the x6 bound, and must leave the channels outside its slice untouched.
The members are the Inception blocks' stages (wsol_backbones/inceptionv3.py:80-158)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_x6 import X6_TOL
from tcam_wsol_video_amd import _lib, ops
from tcam_wsol_video_amd.ops import ConvMember, ConvSrc

pytestmark = pytest.mark.gpu

# (cin, cout, (kh, kw), (ph, pw), out slice): out slice (wide C, coff) or None (own tensor)
STAGES = {
    # InceptionA stage 2: branch5x5_2 (48 -> 64, 5x5) | branch3x3dbl_2 | branch_pool 1x1
    "a": [(48, 64, (5, 5), (2, 2), (160, 0)), (64, 96, (3, 3), (1, 1), None),
          (288, 32, (1, 1), (0, 0), (160, 128))],
    # InceptionC stage 2: 1x7 | 7x1 | branch_pool (aligned: the LDS-DMA tiles apply)
    "c": [(128, 128, (1, 7), (0, 3), None), (160, 160, (7, 1), (3, 0), None),
          (256, 192, (1, 1), (0, 0), (256, 64))],
    # InceptionB: branch3x3 (wide Cout) | branch3x3dbl_1, then a lone member
    "b": [(96, 384, (3, 3), (1, 1), (480, 0)), (96, 64, (1, 1), (0, 0), None)],
    "one": [(64, 40, (3, 3), (1, 1), None)],
    # four members (GROUP_MAX), ragged couts
    "four": [(32, 24, (1, 1), (0, 0), None), (64, 56, (3, 3), (1, 1), None),
             (32, 136, (1, 7), (0, 3), None), (96, 8, (7, 1), (3, 0), (64, 48))],
}
ALIGNED = {"c": True, "b": True, "one": True, "four": True, "a": False}


def _case(stage, B, H, W, g):
    specs = STAGES[stage]
    xs = [torch.randn(B, cin, H, W, generator=g) for cin, *_ in specs]
    ws = [torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
          for cin, cout, (kh, kw), *_ in specs]
    bs = [torch.randn(cout, generator=g) * 0.1 for _, cout, *_ in specs]
    return specs, xs, ws, bs


def _members(specs, xs, ws, bs, fmt, cuda, sentinel=7.0):
    f16 = fmt == "f16x3"
    wides, members, packs = {}, [], []
    B, _, H, W = xs[0].shape
    for (cin, cout, k, p, sl), x, w, b in zip(specs, xs, ws, bs):
        src = ops.s3_from_nchw(x.to(cuda), fmt=fmt)
        if f16:
            wt, wsc = ops.pack_conv_weight_f16([w.to(cuda)])
        else:
            wt, wsc = ops.pack_conv_weight_x6([w.to(cuda)]), None
        out, coff = None, 0
        if sl is not None:
            wc, coff = sl
            if wc not in wides:
                wides[wc] = ops.s3_from_nchw(torch.full((B, wc, H, W), sentinel).to(cuda),
                                             fmt=fmt)
            out = wides[wc]
        members.append(ConvMember(ConvSrc(src, 1), wt, b.to(cuda), cout, H, W, k, p, True,
                                  wscale=wsc, out=out, out_coff=coff))
        packs.append((wt, wsc))
    return members, wides


def _alone(m):
    return ops.conv2d_x6([m.src], m.wt, m.bias, m.cout, m.hout, m.wout, m.ksize, m.pad,
                         m.relu, stream_k=False, wscale=m.wscale)


def _slice(t, coff, c):
    return ops.s3_to_nchw(t)[:, coff:coff + c]


@pytest.mark.parametrize("fmt", ["f16x3", "x6"])
@pytest.mark.parametrize("tile", [-1, 15, 26, 17, 18, 20])
@pytest.mark.parametrize("stage", list(STAGES))
def test_group_members_equal_lone_launches(cuda, stage, tile, fmt):
    if tile in (15, 26) and not ALIGNED[stage]:
        pytest.skip("LDS-DMA tiles need C % 32 == 0 (the launch falls back to 18)")
    g = torch.Generator().manual_seed(len(stage) * 31 + tile)
    B, H, W = 2, 13, 11
    specs, xs, ws, bs = _case(stage, B, H, W, g)
    members, wides = _members(specs, xs, ws, bs, fmt, cuda)
    lib = _lib.load()
    outs = ops.conv2d_group(members, tile)
    used = tile if tile >= 0 else ((26 if any(k != (1, 1) for _, _, k, *_ in specs) else 15)
                                  if ALIGNED[stage] else 18)
    lib.tcam_conv_x6_force_tile(used)
    try:
        alone = [_alone(m) for m in members]
    finally:
        lib.tcam_conv_x6_force_tile(-1)
    if fmt == "f16x3":
        ops.check_f16_overflow(cuda)
    for (cin, cout, k, p, sl), m, o, a, x, w, b in zip(specs, members, outs, alone, xs, ws, bs):
        got = _slice(o, m.out_coff, cout)
        assert torch.equal(got, ops.s3_to_nchw(a)), (stage, cout, k)
        ref = (F.conv2d(x.double(), w.double(), padding=p) +
               b.double()[None, :, None, None]).clamp_min(0)
        absd = F.conv2d(x.double().abs(), w.double().abs(), padding=p)
        err = (got.cpu().double() - ref).abs()
        assert bool((err <= X6_TOL * (absd + 1.0)).all()), float(err.max())
    # channels of the wide outputs no member writes keep the sentinel
    for wc, t in wides.items():
        full = ops.s3_to_nchw(t).cpu()
        written = torch.zeros(wc, dtype=torch.bool)
        for (cin, cout, k, p, sl), m in zip(specs, members):
            if sl is not None and sl[0] == wc:
                written[sl[1]:sl[1] + cout] = True
        assert bool((full[:, ~written] == 7.0).all())


def test_group_frame_count_and_large_shard(cuda):
    """The InceptionC stage at the benchmark's shard geometry (8 x 37 x 37, 344 tiles over
    three members): members equal their lone launches."""
    g = torch.Generator().manual_seed(5)
    specs, xs, ws, bs = _case("c", 8, 37, 37, g)
    members, _ = _members(specs, xs, ws, bs, "f16x3", cuda)
    outs = ops.conv2d_group(members)
    lib = _lib.load()
    lib.tcam_conv_x6_force_tile(26)
    try:
        alone = [_alone(m) for m in members]
    finally:
        lib.tcam_conv_x6_force_tile(-1)
    ops.check_f16_overflow(cuda)
    for (cin, cout, *_), m, o, a in zip(specs, members, outs, alone):
        assert torch.equal(_slice(o, m.out_coff, cout), ops.s3_to_nchw(a))


def test_group_rejects_bad_arguments(cuda):
    g = torch.Generator().manual_seed(1)
    specs, xs, ws, bs = _case("four", 1, 5, 5, g)
    members, _ = _members(specs, xs, ws, bs, "f16x3", cuda)
    with pytest.raises(AssertionError):
        ops.conv2d_group(members + members[:1])
    with pytest.raises(RuntimeError):
        ops.conv2d_group(members, tile=23)     # not a group tile
    m16 = _members(specs[:1], xs[:1], ws[:1], bs[:1], "x6", cuda)[0]
    with pytest.raises(AssertionError):       # precisions do not mix
        ops.conv2d_group(members[:1] + m16)


def test_inception_stages_match_separate_launches(cuda, monkeypatch):
    """The InceptionV3 encoder with staged (grouped) launches against the same encoder with
    one launch per branch conv, f16x3 and x6, 2 frames at 299^2: within fp32 rounding of
    each other: the members run the group's tile instead of their own choice, so sums split
    differently — ~2e-6 of the feature range after 11 blocks; a member writing the wrong
    slice or reading the wrong source would be off by O(1))."""
    from tcam_wsol_video_amd import backbones
    from tcam_wsol_video_amd.models import build_inceptionv3_tcam
    torch.manual_seed(0)
    model = build_inceptionv3_tcam(seed=3).to(cuda).eval()
    x = torch.randn(2, 3, 299, 299).to(cuda)
    res = {}
    for staged in (True, False):
        monkeypatch.setattr(backbones._InceptionPlanX6, "STAGES", staged)
        for prec in ("f16x3", "x6"):
            plan = backbones._InceptionPlanX6(model.encoder, cuda, prec)
            with torch.no_grad():
                res[staged, prec] = [ops.s3_to_nchw(f).cpu() for f in plan.forward(x)[1:]]
    for prec in ("f16x3", "x6"):
        for a, b in zip(res[True, prec], res[False, prec]):
            scale = b.abs().max().item() + 1
            assert (a - b).abs().max().item() <= 1e-5 * scale
