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
