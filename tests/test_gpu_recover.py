"""f16x3 overflow recovery in the batched evaluation (inference.CAMComputer): a clip whose
f16x3 activations leave the S2 range (|x| > 65504) is not an error any more — its counts are
gated off on the device, and compute_and_evaluate re-evaluates it on the exact x6 path (fp32
range), so the pass's counters equal those of evaluating that clip in x6 and the others in
f16x3, with no raise and no per-clip host synchronisation."""
import os

import pytest
import torch

import bench
from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd.inference import CAMComputer
from tcam_wsol_video_amd.models import build_r50_stdcl, build_r50_tcam

pytestmark = pytest.mark.gpu

SCALE = 2.0e4    # an input this large drives the seeded networks' activations past 65504


def _clips(cuda, n=3, frames=8):
    out = []
    for k in range(n):
        x, t, g = bench.make_clip(frames, seed=500 + k)
        out.append([x.to(cuda), t.to(cuda), g.to(cuda)])
    return out


def _counters(comp):
    ev = comp.evaluator
    return ev.counters.clone(), ev.cls_correct.clone(), ev.cnt


@pytest.mark.parametrize("fwd_streams,overlap", [(2, True), (1, False)])
@pytest.mark.parametrize("arch", ["tcam", "stdcl"])
def test_overflowed_clip_is_reevaluated_in_x6(cuda, fwd_streams, overlap, arch):
    build = build_r50_tcam if arch == "tcam" else build_r50_stdcl
    model = build(seed=3).to(cuda)
    model.conv_precision = "f16x3"
    clips = _clips(cuda)
    clips[1][0] = clips[1][0] * SCALE
    ops.check_f16_overflow(cuda)   # start clean
    comp = CAMComputer(model, cam_curve_interval=0.01, device=cuda, fwd_streams=fwd_streams,
                       overlap=overlap)
    for x, t, g in clips:
        comp.evaluate_batch(x, t, g)
    acc = comp.compute_and_evaluate()          # no raise
    assert comp.recovered_clips == 1
    got = _counters(comp)
    # the reference: the same pass with that clip on x6 from the start
    ref = CAMComputer(model, cam_curve_interval=0.01, device=cuda, fwd_streams=fwd_streams,
                      overlap=overlap)
    for k, (x, t, g) in enumerate(clips):
        model.conv_precision = "x6" if k == 1 else "f16x3"
        ref.evaluate_batch(x, t, g)
        ref.synchronize()
    model.conv_precision = "f16x3"
    acc_ref = ref.compute_and_evaluate()
    exp = _counters(ref)
    assert torch.equal(got[0], exp[0]) and torch.equal(got[1], exp[1]) and got[2] == exp[2]
    assert acc == acc_ref and got[2] == 3 * 8


def test_recovery_off_raises(cuda, monkeypatch):
    monkeypatch.setenv("TCAM_F16_RECOVER", "0")
    model = build_r50_tcam(seed=3).to(cuda)
    model.conv_precision = "f16x3"
    clips = _clips(cuda, n=2)
    clips[0][0] = clips[0][0] * SCALE
    ops.check_f16_overflow(cuda)
    comp = CAMComputer(model, cam_curve_interval=0.01, device=cuda, fwd_streams=2)
    for x, t, g in clips:
        comp.evaluate_batch(x, t, g)
    with pytest.raises(FloatingPointError):
        comp.compute_and_evaluate()
    assert os.environ["TCAM_F16_RECOVER"] == "0"
