"""CPU: the C-ABI library loads and exports every symbol include/tcam_hip.h
declares (no compute calls), host-side weight folding, and the
no-CPU-fallback contract."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from tcam_wsol_video_amd import _lib
from tcam_wsol_video_amd.models import FoldedConv, build_r50_tcam, fold_conv_bn
from tcam_wsol_video_amd.utils.seeding import seeded_state_dict, synthetic_clip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "tcam_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:[\w\*\s]+?)\b(\w+)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "sizeof")))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _header_symbols()
    assert "tcam_conv2d" in syms and "bilateralfilter_batch" in syms
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} missing from ctypes SIGNATURES"
    assert lib.tcam_abi_version() == 2
    assert lib.tcam_arch() == b"gfx950"


def test_group_launch_validates_before_touching_the_device():
    """tcam_conv2d_group's argument checks run on the host (no HIP call before them): member
    count 1..4, fmt 0 / 1, group tiles only, the f16x3 scale pointer, a member's geometry."""
    lib = _lib.load()
    probs = (_lib.tcam_conv_prob * 5)()
    assert lib.tcam_conv2d_group(None, 1, 1, 0, -1, None, None) == -1
    assert lib.tcam_conv2d_group(probs, 0, 1, 0, -1, None, None) == -1
    assert lib.tcam_conv2d_group(probs, 5, 1, 0, -1, None, None) == -1
    assert lib.tcam_conv2d_group(probs, 1, 1, 2, -1, None, None) == -1   # fmt
    assert lib.tcam_conv2d_group(probs, 1, 1, 0, 23, None, None) == -1   # not a group tile
    # an all-zero member: f16x3 without wscale, and x6 with a null source / zero Cout
    assert lib.tcam_conv2d_group(probs, 1, 1, 1, -1, None, None) == -1
    assert lib.tcam_conv2d_group(probs, 1, 1, 0, -1, None, None) == -1


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_fold_conv_bn_matches_eval_bn():
    torch.manual_seed(0)
    conv = nn.Conv2d(8, 6, 3, padding=1, bias=True)
    bn = nn.BatchNorm2d(6).eval()
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-1, 1)
    x = torch.randn(2, 8, 9, 9)
    ref = bn(conv(x))
    w, b = fold_conv_bn(conv, bn)
    out = F.conv2d(x.double(), w.reshape(6, 8, 3, 3), b, padding=1)
    assert (out.float() - ref).abs().max() < 1e-5


def test_folded_conv_k_concat_layout():
    c3, b3 = nn.Conv2d(4, 8, 1, bias=False), nn.BatchNorm2d(8).eval()
    cd, bd = nn.Conv2d(6, 8, 1, bias=False), nn.BatchNorm2d(8).eval()
    fc = FoldedConv([(c3, b3), (cd, bd)], torch.device("cpu"))
    assert fc.wt.shape == (32, 128)  # (roundup(K, 32), roundup(Cout, 128)), zero padded
    w3, bb3 = fold_conv_bn(c3, b3)
    wd, bbd = fold_conv_bn(cd, bd)
    assert torch.allclose(fc.wt[:4, :8].double(), w3.t(), atol=1e-6)
    assert torch.allclose(fc.wt[4:10, :8].double(), wd.t(), atol=1e-6)
    assert fc.wt[10:].abs().sum() == 0 and fc.wt[:, 8:].abs().sum() == 0
    assert torch.allclose(fc.bias.double(), bb3 + bbd)


def test_pack_conv_weight_tap_major():
    from tcam_wsol_video_amd.ops import pack_conv_weight
    w1 = torch.arange(2 * 3 * 9, dtype=torch.float32).reshape(2, 3, 3, 3)
    w2 = -torch.arange(2 * 1 * 9, dtype=torch.float32).reshape(2, 1, 3, 3)
    wt = pack_conv_weight([w1, w2])
    # k = (kh * 3 + kw) * Ctot + c with c over [w1 channels, w2 channels]
    for kh in range(3):
        for kw in range(3):
            for c in range(4):
                k = (kh * 3 + kw) * 4 + c
                ref = w1[:, c, kh, kw] if c < 3 else w2[:, 0, kh, kw]
                assert torch.equal(wt[k, :2], ref)


def test_model_refuses_cpu_inputs():
    m = build_r50_tcam()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 3, 64, 64))


def test_seeding_is_deterministic_and_reference_named():
    m = build_r50_tcam()
    a = seeded_state_dict(m, 3)
    b = seeded_state_dict(m, 3)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert not torch.equal(a["encoder.conv1.weight"], seeded_state_dict(m, 4)["encoder.conv1.weight"])


def test_synthetic_clip_shape():
    c = synthetic_clip(3, seed=0)
    assert c.shape == (3, 360, 480, 3) and c.dtype == np.uint8


def test_prepared_lattice_refuses_host_images():
    """crf.PreparedLattice has no CPU fallback either (the refusal comes before any device
    call); the training step's lattice must be applied exactly once."""
    from tcam_wsol_video_amd import crf
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        crf.PreparedLattice(torch.zeros(1, 3, 8, 8), 2, 15.0, 100.0)
    syms = _header_symbols()
    assert "tcam_bilateral_prepare" in syms and "tcam_bilateral_apply" in syms
