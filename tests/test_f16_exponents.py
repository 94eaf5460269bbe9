"""Host logic of the f16x3 plans' per-channel activation exponents (models.act_exponents,
FoldedConv's exact weight / bias folding, the consumers' unscaling).  CPU only: the packing
kernel is replaced by a capture of the folded fp32 weights."""
import pytest
import torch
import torch.nn as nn

from tcam_wsol_video_amd import models as M


def test_act_exponents_rule(monkeypatch):
    e = M.act_exponents(torch.tensor([1.0, 0.3, 0.2, 2.0 ** -10, 0.0, 2.0 ** -30, 0.2499]))
    assert e.tolist() == [0, 0, 3, 10, 0, 16, 3]
    # 2^e * mag lands in [1, 2) for every scaled channel
    mag = torch.tensor([0.2, 2.0 ** -10 * 1.7, 0.01])
    e = M.act_exponents(mag)
    assert bool(((mag * 2.0 ** e.double() >= 1) & (mag * 2.0 ** e.double() < 2)).all())
    assert M.act_exponents(torch.tensor([0.5, 3.0])) is None
    monkeypatch.setenv("TCAM_F16_ACT_SCALE", "0")
    assert M.act_exponents(torch.tensor([2.0 ** -10])) is None


def test_bn_magnitude_and_seeded_models_are_unscaled():
    """The seeded (random-init) models of the goldens and the bench are O(1): no exponent,
    so their f16x3 arithmetic is unchanged."""
    model = M.build_r50_tcam(seed=0)
    for mod in model.modules():
        if isinstance(mod, nn.BatchNorm2d):
            assert M.act_exponents(M.bn_magnitude(mod)) is None
    bn = nn.BatchNorm2d(3)
    with torch.no_grad():
        bn.weight.copy_(torch.tensor([1.0, -0.01, 0.0]))
        bn.bias.copy_(torch.tensor([0.0, 0.02, -0.5]))
    assert torch.allclose(M.bn_magnitude(bn), torch.tensor([3.0, 0.05, 0.5], dtype=torch.float64))


def test_folded_conv_absorbs_exponents_exactly(monkeypatch):
    captured = {}

    def fake_pack(ws):
        captured["ws"] = [w.clone() for w in ws]
        return None, None
    monkeypatch.setattr(M.ops, "pack_conv_weight_f16", fake_pack)
    g = torch.Generator().manual_seed(0)
    c1, c2 = nn.Conv2d(5, 4, 3, bias=False), nn.Conv2d(3, 4, 1, bias=False)
    b1, b2 = nn.BatchNorm2d(4), nn.BatchNorm2d(4)
    for m in (c1, c2, b1, b2):
        for p in m.parameters():
            with torch.no_grad():
                p.copy_(torch.randn(p.shape, generator=g))
    for b in (b1, b2):
        b.running_mean.copy_(torch.randn(4, generator=g))
        b.running_var.copy_(torch.rand(4, generator=g) + 0.5)
    b1.eval(), b2.eval()
    e_in1 = torch.tensor([0, 3, 7, 0, 12])
    e_in2 = torch.tensor([5, 0, 1])
    e_out = torch.tensor([0, 2, 9, 4])
    fc = M.FoldedConv([(c1, b1), (c2, b2)], torch.device("cpu"), "f16x3", ein=[e_in1, e_in2],
                      eout=e_out)
    fc_ws = captured["ws"]
    ref = M.FoldedConv([(c1, b1), (c2, b2)], torch.device("cpu"), "f16x3")
    ref_ws = captured["ws"]
    # fold(W) * 2^(e_out - e_in) and bias * 2^e_out, bit for bit (powers of two)
    for w, w0, e_in in zip(fc_ws, ref_ws, (e_in1, e_in2)):
        f = torch.pow(2.0, (e_out[:, None] - e_in[None, :]).double()).float()
        assert torch.equal(w, w0 * f[:, :, None, None])
    assert torch.equal(fc.bias, ref.bias * torch.pow(2.0, e_out.double()).float())


def test_unscale_and_signature_helpers():
    w = torch.randn(2, 5, 3, 3)
    e = torch.tensor([0, 1, 2, 3, 4])
    u = M.unscale_in(w, e)
    assert torch.equal(u * torch.pow(2.0, e.float())[None, :, None, None], w)
    assert M.unscale_in(w, None) is w
    fc = torch.randn(10, 5)
    assert torch.equal(M.unscale_in(fc, e) * torch.pow(2.0, e.float())[None, :], fc)
    assert M.exps_signature([None, None]) == ""
    assert M.exps_signature([None, torch.tensor([1, 0])]) == ":|1,0"
    assert M.cat_exponents([(None, 2), (None, 3)]) is None
    assert M.cat_exponents([(None, 2), (torch.tensor([4, 5]), 2)]).tolist() == [0, 0, 4, 5]
