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


def _reference_sgd(model, lr=0.01, ratio=10.):
    """The reference's optimizer (instantiators.py:742-841): torch SGD over two groups of
    ALL named parameters."""
    g0, g1 = CK.reference_param_groups(model)
    named = dict(model.named_parameters())
    return torch.optim.SGD([{"params": [named[n] for n in g0], "lr": lr},
                            {"params": [named[n] for n in g1], "lr": lr * ratio}],
                           lr=lr, momentum=0.9, dampening=0., weight_decay=1e-4, nesterov=True)


def test_reference_param_groups_resnet_and_vgg():
    from tcam_wsol_video_amd.models import build_vgg16_tcam
    r = build_r50_tcam(seed=1)
    g0, g1 = CK.reference_param_groups(r)
    assert all(n.startswith(("encoder.layer4.", "classification_head.")) for n in g1)
    assert "decoder.blocks.0.conv1.0.weight" in g0 and len(g0) + len(g1) == \
        len(list(r.named_parameters()))
    v = build_vgg16_tcam(seed=1)
    g0, g1 = CK.reference_param_groups(v)
    assert all(n.startswith("encoder.features.") for n in g0)
    assert "decoder.center.0.0.weight" in g1


def test_reference_optimizer_state_maps_to_trainable_params():
    """The two-group layout (the reference's non-TCAM tasks; TCAM's single group is
    tests/test_api.py): a reference-layout SGD state_dict (momentum only on the trained decoder + seg head,
    global indices across both groups) maps onto the right parameters, and the layout we
    write loads into the reference's optimizer and maps back."""
    model = build_r50_tcam(seed=1)
    train = CK.trainable_names(model)
    named = dict(model.named_parameters())
    opt = _reference_sgd(model)
    g = torch.Generator().manual_seed(0)
    for n in train:            # one step with gradients on the trainable params only
        named[n].grad = torch.randn(named[n].shape, generator=g)
    opt.step()
    sd = opt.state_dict()
    mom = CK.momentum_from_state_dict(model, sd)
    assert sorted(mom) == sorted(train)
    for n in train:
        assert torch.equal(mom[n], opt.state[named[n]]["momentum_buffer"]), n
    ours = CK.optimizer_state_dict(model, {"lr": 0.01, "momentum": 0.9, "dampening": 0.,
                                           "weight_decay": 1e-4, "nesterov": True}, mom,
                                   task="STD_CL")
    opt2 = _reference_sgd(build_r50_tcam(seed=2))
    opt2.load_state_dict(ours)                     # the reference optimizer accepts it
    assert [g["lr"] for g in opt2.param_groups] == [0.01, 0.1]
    back = CK.momentum_from_state_dict(model, opt2.state_dict())
    assert all(torch.equal(back[n], mom[n]) for n in train)


def test_loss_t_layout():
    t = CK._loss_t(1.5)
    assert CK._t_from(t) == 1.5 and CK._t_from(torch.tensor([2.0])) == 2.0


def test_tracker_round_trip_restores_model_selection(tmp_path):
    """train_wsol.py:1280-1316: the validation meters survive a resume, so the first
    evaluation after it is compared against the earlier epochs (not taken as the best)."""
    d = str(tmp_path)
    assert CK.load_tracker(d) == {}
    CK.save_tracker(d, 3, {"best_loc": [10.0, 42.5], "best_cl": [50.0, 40.0]})
    CK.save_tracker(d, 6, {"best_loc": [10.0, 42.5, 30.0], "best_cl": [50.0, 40.0, 60.0]})
    got = CK.load_tracker(d)
    assert got == {"best_loc": [10.0, 42.5, 30.0], "best_cl": [50.0, 40.0, 60.0]}
    it, cpt = CK.find_last_checkpoint(d, CK.CHP_TR)
    m = cpt[CK.CHP_TR]["val"]["localization"]
    assert it == 6 and m["best_value"] == 42.5 and m["best_epoch"] == 1
    assert CK.keep_last_n_checkpoints(d, 1, key=CK.CHP_TR) == [6]
