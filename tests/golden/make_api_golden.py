"""Generate tests/golden/api_golden.json from the REFERENCE's host-side API.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_api_golden.py

Imported from the reference (read-only, not copied), through the same stubs as
make_golden.py:

* dlib/unet/model.py ``UnetTCAM`` and dlib/stdcl/classifier.py ``STDClassifier``: the
  strings process/instantiators.py:568 logs right after ``create_model`` —
  ``"{}".format(model)``, ``count_nb_params(model)`` (utils/tools.py:87-98) and
  ``model.get_info_nbr_params()`` (base/model.py:36-50, 229-256) — for the three
  backbones;
* dlib/cams/decay_temp.py ``DecayTemp`` (skimage, imported there but unused by the class,
  is stubbed): ``sl_tc_knn_t`` and ``sl_tc_seed_tech`` per epoch for a grid of
  (t, min_t, switch) settings;
* dlib/learning/lr_scheduler.py ``MyStepLR``: the learning rate over 60 epochs for the
  README's (step 15, gamma 0.9) and the config defaults (step 40, gamma 0.1).
"""
from __future__ import annotations

import importlib
import json
import os
import sys
sys.dont_write_bytecode = True  # nothing may be written under /root/reference
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402


def model_strings(unet, stdcl, const):
    tools = importlib.import_module("dlib.utils.tools")
    out = {}
    for name in ("resnet50", "vgg16", "inceptionv3"):
        m = make_golden.build_ref_family_tcam(unet, const, name)
        out[f"TCAM/{name}"] = {"str": "{}".format(m), "count": tools.count_nb_params(m),
                               "info": m.get_info_nbr_params()}
        depth = 3 if name == "vgg16" else 5
        s = stdcl.STDClassifier(task=const.STD_CL, encoder_name=name, encoder_depth=depth,
                                encoder_weights=None, in_channels=3, scale_in=1.,
                                aux_params=dict(pooling_head="WGAP", classes=10,
                                                support_background=False))
        out[f"STD_CL/{name}"] = {"str": "{}".format(s), "count": tools.count_nb_params(s),
                                 "info": s.get_info_nbr_params()}
    return out


def decay_temp_cases():
    sk = types.ModuleType("skimage")
    skf = types.ModuleType("skimage.filters")
    skf.threshold_otsu = None
    sk.filters = skf
    sys.modules.setdefault("skimage", sk)
    sys.modules.setdefault("skimage.filters", skf)
    dt = importlib.import_module("dlib.cams.decay_temp")
    cases = []
    for t, tmin, sw, k, mode, tech in ((10., 1., 10, 1, "before", "seed_weighted"),
                                       (0., 0., -1, 1, "before", "seed_weighted"),
                                       (2.5, 0.5, 4, 2, "before-after", "seed_weighted"),
                                       (3., 3., 5, 1, "after", "seed_uniform"),
                                       (4., 1., 0, 1, "before", "seed_weighted"),
                                       (1.5, 0., -1, 0, "instant", "seed_weighted")):
        m = dt.DecayTemp(sl_tc_knn_t=t, sl_tc_min_t=tmin, sl_tc_knn=k, sl_tc_knn_mode=mode,
                         sl_tc_knn_epoch_switch_uniform=sw, sl_tc_seed_tech=tech)
        rows = []
        for e in range(0, 16):
            m.set_epoch(e)
            rows.append([e, m.sl_tc_knn_t, m.sl_tc_seed_tech, m.get_current_status()])
        cases.append({"args": [t, tmin, k, mode, sw, tech], "str": str(m), "epochs": rows})
    return cases


def lr_cases():
    lrs = importlib.import_module("dlib.learning.lr_scheduler")
    out = []
    for step, gamma, min_lr in ((15, 0.9, 1e-7), (40, 0.1, 1e-7), (2, 0.01, 1e-5)):
        p = torch.zeros(1, requires_grad=True)
        opt = torch.optim.SGD([p], lr=0.01)
        sch = lrs.MyStepLR(opt, step_size=step, gamma=gamma, last_epoch=-1, min_lr=min_lr)
        seq = []
        for _ in range(60):
            seq.append(opt.param_groups[0]["lr"])
            sch.step()
        out.append({"step_size": step, "gamma": gamma, "min_lr": min_lr, "lr": seq})
    return out


def main():
    unet, stdcl, const = make_golden.reference_models()
    out = {"models": model_strings(unet, stdcl, const), "decay_temp": decay_temp_cases(),
           "lr": lr_cases()}
    with open(os.path.join(HERE, "api_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote api_golden.json")


if __name__ == "__main__":
    main()
