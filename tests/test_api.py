"""CPU: the host-side API pieces of the training loop against goldens made by the
reference's own code (tests/golden/make_api_golden.py):

* the model report the reference's ``get_model`` logs right after ``create_model``
  (process/instantiators.py:462-568: ``"{}".format(model)``, ``count_nb_params``,
  ``get_info_nbr_params``), run here over the drop-in ``create_model``;
* ``DecayTemp`` (dlib/cams/decay_temp.py) and the loader's heating gate;
* ``MyStepLR`` (learning/lr_scheduler.py) through ``training.lr_schedule``;
* ``_fill_minibatch`` (learning/train_wsol.py:1006-1023);
* the TCAM optimizer layout of the checkpoints (instantiators.py:746-754).
"""
import json
import os

import pytest
import torch

from tcam_wsol_video_amd import checkpoints as CK
from tcam_wsol_video_amd.decay_temp import DecayTemp, heat_t
from tcam_wsol_video_amd.models import create_model

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "api_golden.json")))


def _get_model(task, encoder_name):
    """The reference's get_model (instantiators.py:462-568) over the drop-in create_model,
    with what it logs."""
    from tcam_wsol_video_amd.backbones import encoder_depth_channels
    depth, dec = encoder_depth_channels(encoder_name)
    aux = dict(pooling_head="WGAP", classes=10, support_background=False)
    if task == "TCAM":
        model = create_model(task=task, arch="UnetTCAM", encoder_name=encoder_name,
                             encoder_weights=None, encoder_depth=depth, decoder_channels=dec,
                             in_channels=3, seg_h_out_channels=2, scale_in=1.,
                             aux_params=aux, freeze_cl=True, im_rec=False, img_range="tanh")
    else:
        model = create_model(task=task, arch="STDClassifier", encoder_name=encoder_name,
                             encoder_weights=None, in_channels=3, encoder_depth=depth,
                             scale_in=1., aux_params=aux)
    count = sum(p.numel() for p in model.parameters())      # tools.count_nb_params
    return model, "{}".format(model), count, model.get_info_nbr_params()


@pytest.mark.parametrize("key", sorted(GOLD["models"]))
def test_get_model_report_matches_reference(key):
    task, name = key.split("/")
    _, s, count, info = _get_model(task, name)
    g = GOLD["models"][key]
    assert s == g["str"]
    assert count == g["count"]
    assert info == g["info"]


@pytest.mark.parametrize("case", range(len(GOLD["decay_temp"])))
def test_decay_temp_matches_reference(case):
    c = GOLD["decay_temp"][case]
    t, tmin, k, mode, sw, tech = c["args"]
    m = DecayTemp(sl_tc_knn_t=t, sl_tc_min_t=tmin, sl_tc_knn=k, sl_tc_knn_mode=mode,
                  sl_tc_knn_epoch_switch_uniform=sw, sl_tc_seed_tech=tech)
    assert str(m) == c["str"]
    for e, tt, st, status in c["epochs"]:
        m.set_epoch(e)
        assert m.sl_tc_knn_t == tt and m.sl_tc_seed_tech == st, e
        assert m.get_current_status() == status
        # the loader heats only with sl_tc_knn > 0 (wsol_loader.py:571, 594)
        assert m.heat_t == (tt if (k > 0 and tt > 0) else 0.0)


def test_heat_gate():
    assert heat_t(0, 0.7) == 0.0 and heat_t(1, 0.7) == 0.7 and heat_t(2, 0.0) == 0.0


@pytest.mark.parametrize("case", range(len(GOLD["lr"])))
def test_lr_schedule_matches_reference(case):
    from tcam_wsol_video_amd.training import lr_schedule
    c = GOLD["lr"][case]

    class _T:
        lr = 0.01
    tr = _T()
    sch = lr_schedule(tr, c["step_size"], c["gamma"], c["min_lr"])
    got = []
    for _ in range(len(c["lr"])):
        got.append(tr.lr)
        sch.step()
    assert got == c["lr"]
    # resume: a fresh schedule loaded from the state_dict continues the sequence
    tr2 = _T()
    s2 = lr_schedule(tr2, c["step_size"], c["gamma"], c["min_lr"])
    sd = sch.state_dict()
    import io
    buf = io.BytesIO()
    torch.save(sd, buf)           # checkpointable (utils_checkpoints.py:203-212)
    s2.load_state_dict(torch.load(io.BytesIO(buf.getvalue()), weights_only=True))
    assert tr2.lr == tr.lr


def test_fill_minibatch_repeats_short_batch():
    from tcam_wsol_video_amd.training import fill_minibatch
    x = torch.arange(7 * 3).view(7, 3)
    y = fill_minibatch(x, 32)
    assert y.shape == (32, 3)
    # torch.cat(ceil(32 / 7) * [x])[:32] (train_wsol.py:1016-1021)
    for i in range(32):
        assert torch.equal(y[i], x[i % 7])
    assert fill_minibatch(x, 7) is x and fill_minibatch(None, 4) is None
    with pytest.raises(AssertionError):
        fill_minibatch(x, 5)


def _hp():
    return {"lr": 0.01, "momentum": 0.9, "dampening": 0., "weight_decay": 1e-4,
            "nesterov": True}


def _reference_tcam_sgd(model, lr=0.01):
    """get_optimizer for task TCAM (instantiators.py:751-754, 811-841): torch SGD over
    ONE group, model.parameters() at lr."""
    return torch.optim.SGD([{"params": model.parameters(), "lr": lr}], lr=lr, momentum=0.9,
                           dampening=0., weight_decay=1e-4, nesterov=True)


def test_tcam_checkpoint_optimizer_is_one_group():
    from tcam_wsol_video_amd.models import build_r50_tcam, build_vgg16_tcam
    for build in (build_r50_tcam, build_vgg16_tcam):
        model = build(seed=1)
        train = CK.trainable_names(model)
        named = dict(model.named_parameters())
        opt = _reference_tcam_sgd(model)
        g = torch.Generator().manual_seed(0)
        for n in train:
            named[n].grad = torch.randn(named[n].shape, generator=g)
        opt.step()
        sd = opt.state_dict()
        # a real reference TCAM checkpoint: one group covering every parameter
        mom = CK.momentum_from_state_dict(model, sd)
        assert sorted(mom) == sorted(train)
        for n in train:
            assert torch.equal(mom[n], opt.state[named[n]]["momentum_buffer"]), n
        ours = CK.optimizer_state_dict(model, _hp(), mom)
        assert len(ours["param_groups"]) == 1 and ours["param_groups"][0]["lr"] == 0.01
        opt2 = _reference_tcam_sgd(build(seed=2))
        opt2.load_state_dict(ours)                 # main.py:54-55 accepts it
        back = CK.momentum_from_state_dict(model, opt2.state_dict())
        assert all(torch.equal(back[n], mom[n]) for n in train)


def test_stdcl_optimizer_keeps_two_groups():
    from tcam_wsol_video_amd.models import build_r50_stdcl
    model = build_r50_stdcl(seed=1)
    sd = CK.optimizer_state_dict(model, _hp(), {}, task="STD_CL")
    assert len(sd["param_groups"]) == 2


def test_loss_t_lists_enabled_losses_in_reference_order():
    assert [n for n, _ in CK._loss_t(2.0)] == ["con_ran_field_tcams",
                                                "max_size_positive_tcams",
                                                "self_learning_tcams"]
    assert CK._loss_t(2.0, use=(True, False, True)) == [["max_size_positive_tcams", 2.0],
                                                        ["self_learning_tcams", 0.0]]
    assert CK._t_from(CK._loss_t(1.5, use=(False, True, True))) == 1.5


def test_keep_last_n_checkpoints(tmp_path):
    for it in (3, 10, 7, 12):
        torch.save({"iter": it}, str(tmp_path / f"{it}_checkpoint.pth"))
    (tmp_path / "11_checkpoint.pth").write_bytes(b"broken")
    kept = CK.keep_last_n_checkpoints(str(tmp_path), 3)
    assert kept == [12, 10]           # 11 is unloadable: deleted; 7 and 3 beyond n
    assert sorted(os.listdir(tmp_path)) == ["10_checkpoint.pth", "12_checkpoint.pth"]
