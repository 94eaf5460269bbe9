"""Pins the training-loss oracle (oracle/train_ref.py::tcam_losses) to goldens produced by
the REFERENCE loss modules (tests/golden/make_train_golden.py: MasterLoss over
ConRanFieldTcams + MaxSizePositiveTcams(ELB) + SelfLearningTcams, losses/tcam.py:48-278,
elb.py:119-137, dense_crf_loss.py:32-123, the CRF filter compiled from its own sources)."""
import os

import numpy as np
import pytest
import torch

from oracle import crf_ref
from oracle import train_ref as T

G = os.path.join(os.path.dirname(__file__), "golden", "tcam_losses.npz")
CASES = ("a", "b", "c")


def _case(d, c):
    return {k[len(c) + 1:]: d[k] for k in d.files if k.startswith(c + "_")}


@pytest.mark.parametrize("case", CASES)
def test_loss_oracle_matches_reference_goldens(case):
    d = _case(np.load(G), case)
    f = torch.from_numpy(d["fcams"]).clone().requires_grad_(True)
    raw = torch.from_numpy(d["raw"])
    seeds = torch.from_numpy(d["seeds"])
    total, sl, crf, size = T.tcam_losses(f, raw, seeds, elb_t=float(d["elb_t"]))
    total.backward()
    for name, v in (("total", total), ("sl", sl), ("crf", crf), ("size", size)):
        ref = float(d[name])
        assert abs(float(v) - ref) <= 1e-6 * max(1.0, abs(ref)), (name, float(v), ref)
    g = f.grad.numpy()
    assert np.abs(g - d["grad"]).max() <= 1e-6 * np.abs(d["grad"]).max()


def test_golden_exercises_both_elb_branches():
    """case b has an all-background frame: its channel-1 size -bl is > -1/t^2 (the linear
    branch of elb.py:130-135) while the other frames take the log branch."""
    d = _case(np.load(G), "b")
    S = torch.softmax(torch.from_numpy(d["fcams"]), 1)
    bl = S[:, 1].reshape(S.shape[0], -1).sum(-1)
    ct = -1.0 / float(d["elb_t"]) ** 2
    assert (-bl > ct).any() and (-bl <= ct).any()


def test_crf_term_uses_compiled_reference():
    assert crf_ref.ref_available("xy"), "oracle/_ref not built (make -C oracle)"


RGB = os.path.join(os.path.dirname(__file__), "golden", "rgb_joint_crf.npz")


@pytest.mark.parametrize("case", ("a", "b", "c", "d"))
def test_rgb_joint_oracle_matches_reference_goldens(case):
    """oracle/train_ref.rgb_joint_crf vs the REFERENCE RgbJointConRanFieldTcams (MasterLoss
    over it alone, losses/tcam.py:158-232, the colour filter compiled from its sources)."""
    d = _case(np.load(RGB), case)
    f = torch.from_numpy(d["fcams"]).clone().requires_grad_(True)
    raw = torch.from_numpy(d["raw"].astype(np.float32))
    loss = T.rgb_joint_crf(f, raw, torch.from_numpy(d["seq"]), torch.from_numpy(d["frm"]),
                           float(d["lam"]), float(d["sigma_rgb"]))
    loss.backward()
    ref = float(d["total"])
    assert abs(float(loss) - ref) <= 1e-6 * abs(ref), (float(loss), ref)
    assert np.abs(f.grad.numpy() - d["grad"]).max() <= 1e-6 * np.abs(d["grad"]).max()


def test_group_ordered_frames_matches_oracle():
    """The product's host grouping (losses.group_ordered_frames) == the restatement of
    losses/tcam.py:32-45 on the golden batches and on ties / unsorted ids."""
    from tcam_wsol_video_amd.losses import group_ordered_frames
    d = np.load(RGB)
    cases = [(d[c + "_seq"], d[c + "_frm"]) for c in "abcd"]
    cases.append(([2.0, 0.0, 2.0, 0.0, 1.0, 2.0], [1.0, 1.0, 0.0, 1.0, 0.0, 1.0]))
    for seq, frm in cases:
        assert group_ordered_frames(seq, frm) == T.group_ordered_frames(
            torch.as_tensor(seq), torch.as_tensor(frm))
    assert group_ordered_frames([3, 3, 3, 7, 7, 3, 3, 3], [0, 1, 2, 0, 1, 0, 1, 2]) == \
        [[0, 5, 1, 6, 2, 7], [3, 4]]


STD = os.path.join(os.path.dirname(__file__), "golden", "stdcl_train.npz")


@pytest.mark.parametrize("case", ("a", "b"))
def test_stdcl_step_oracle_matches_reference_goldens(case):
    """oracle/train_ref.stdcl_step (fp64) vs the REFERENCE stage-1 step
    (tests/golden/make_stdcl_golden.py: STDClassifier in train mode, MasterLoss + ClLoss,
    instantiators.get_optimizer's two SGD groups): logits, loss, every parameter's gradient
    norm, full gradients / updated values / running statistics of the stored tensors.
    Run in fp32 — the reference's CPU arithmetic — the restatement reproduces it to fp32
    rounding (its ReLUs take the same branches); the device tests use it in fp64 with the
    device's ReLU branches (a fp32 / fp64 branch flip at a pre-activation within rounding
    of 0 moves a gradient discontinuously: ~2e-3 on these gradient norms)."""
    from tcam_wsol_video_amd.models import build_r50_stdcl
    d = np.load(STD)
    g = {k[len(case) + 1:]: d[k] for k in d.files if k.startswith(case + ":")}
    sd = build_r50_stdcl(seed=int(d["seed"])).state_dict()
    lr, mom, damp, wd, nest, ratio = [float(v) for v in d["opt"]]
    # the goldens were made with 8 intra-op threads: torch's single-threaded fp32 CPU conv
    # rounds differently, and this step amplifies fp32 rounding to ~1e-3 (branch flips)
    nt = torch.get_num_threads()
    torch.set_num_threads(8)
    try:
        loss, logits, grads, new, bufs = T.stdcl_step(
            sd, torch.from_numpy(g["x"]), torch.from_numpy(g["labels"]), lr=lr,
            lr_classifier_ratio=ratio, momentum=mom, dampening=damp, weight_decay=wd,
            nesterov=bool(nest), dtype=torch.float32)
    finally:
        torch.set_num_threads(nt)
    assert abs(loss - float(g["loss"])) <= 2e-6 * abs(float(g["loss"]))
    assert np.abs(logits.numpy() - g["logits"]).max() <= 2e-5 * np.abs(g["logits"]).max()
    names = list(g["names"])
    assert names == [k for k in grads], "parameter order / names differ from the reference"
    gsq = np.array([float((grads[k] ** 2).sum()) for k in names])
    np.testing.assert_allclose(gsq, g["gsq"], rtol=1e-5)
    for k in [n[5:] for n in g if n.startswith("grad/")]:
        ref = g["grad/" + k]
        assert np.abs(grads[k].numpy() - ref).max() <= 1e-5 * np.abs(ref).max(), k
        refn = g["new/" + k]
        assert np.abs(new[k].numpy() - refn).max() <= 1e-5 * max(np.abs(refn).max(), 1e-3), k
    for k in [n[3:] for n in g if n.startswith("rm/")]:
        np.testing.assert_allclose(bufs[k + ".running_mean"].numpy(), g["rm/" + k], atol=2e-6)
        np.testing.assert_allclose(bufs[k + ".running_var"].numpy(), g["rv/" + k], rtol=2e-5)
    feat, cls = T.stdcl_param_groups(names)
    assert [len(feat), len(cls)] == list(g["group_sizes"])
