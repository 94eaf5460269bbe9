"""CPU: reference-format checkpoint files (train_wsol.py:1681-1726,
utils_checkpoints.py:112-213, instantiators.py:598-698) round trip through our
reference-named modules."""
import os

import torch

from tcam_wsol_video_amd import checkpoints as CK
from tcam_wsol_video_amd.models import build_r50_stdcl, build_r50_tcam


def _eq(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    return all(torch.equal(sa[k], sb[k]) for k in sa)


def test_best_model_round_trip(tmp_path):
    src = build_r50_tcam(seed=1)
    dst = build_r50_tcam(seed=2)
    assert not _eq(src, dst)
    CK.save_best_model(src, "TCAM", str(tmp_path), 40)
    CK.save_best_model(dst, "TCAM", str(tmp_path), 7)        # older: ignored
    cpt = torch.load(str(tmp_path / "40_best_model.pth"), weights_only=True)
    assert set(cpt) == {"encoder", "decoder", "classification_head", "segmentation_head"}
    assert "layer4.2.conv3.weight" in cpt["encoder"]
    assert CK.load_best_model(dst, "TCAM", str(tmp_path)) == 40
    assert _eq(src, dst)


def test_corrupted_newest_checkpoint_is_skipped(tmp_path):
    src = build_r50_stdcl(seed=3)
    CK.save_best_model(src, "STD_CL", str(tmp_path), 5)
    (tmp_path / "9_best_model.pth").write_bytes(b"not a checkpoint")
    it, cpt = CK.find_last_checkpoint(str(tmp_path), CK.CHP_BEST_M)
    assert it == 5 and cpt["decoder"] is None
    # stage-1 classifier into a TCAM model (instantiators.py:598-625)
    tcam = build_r50_tcam(seed=4)
    assert CK.load_pretrained_classifier(tcam, str(tmp_path)) == 5
    for k, v in src.encoder.state_dict().items():
        assert torch.equal(tcam.encoder.state_dict()[k], v)
    assert torch.equal(tcam.classification_head.fc.weight, src.classification_head.fc.weight)


def test_missing_checkpoint_defaults(tmp_path):
    it, cpt = CK.find_last_checkpoint(str(tmp_path), CK.CHP_CP)
    assert it == 0 and cpt["model"] is None and cpt["iter"] == 0
