"""Checkpoint interop with the reference's files.

Formats (reference paths relative to sbelharbi/tcam-wsol-video):

* best model ``<dir>/<step>_best_model.pth`` = ``{'encoder', 'decoder',
  'classification_head', 'segmentation_head'[, 'reconstruction_head']}`` state
  dicts for TCAM / F_CL, ``{'encoder', 'classification_head'}`` for STD_CL
  (learning/train_wsol.py:1681-1726, saved from a CPU copy of the model);
* training checkpoint ``<dir>/<step>_checkpoint.pth`` = ``{'model', 'optimizer',
  'lr_scheduler', 't', 'iter'}`` (utils/utils_checkpoints.py:193-213);
* the newest loadable ``*_<key>.pth`` wins (utils_checkpoints.py:112-150).

Loading restores the reference's strict ``load_state_dict`` calls
(process/instantiators.py:598-698); our modules carry the reference's names, so
reference-trained weights load unchanged, and the HIP plans are rebuilt on the next
forward (parameter versions change).  Files are read with ``weights_only=True``.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, List, Optional, Tuple

import torch

CHP_M, CHP_O, CHP_LR, CHP_T = "model", "optimizer", "lr_scheduler", "t"
CHP_CP, CHP_TR, CHP_BEST_M = "checkpoint", "tracker", "best_model"
_DEFAULT_CHECKPOINT = {CHP_M: None, CHP_O: None, CHP_LR: None, CHP_T: None, "iter": 0}
_DEFAULT_BEST_MODEL = {"encoder": None, "decoder": None, "classification_head": None,
                       "segmentation_head": None, "reconstruction_head": None,
                       "box_head": None}


def _cpu_sd(m: torch.nn.Module) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu").clone() for k, v in m.state_dict().items()}


def find_last_checkpoint(save_dir: str, key: str) -> Tuple[int, dict]:
    """utils_checkpoints.py:112-150: (iter, dict) of the newest loadable file, or the
    default dict (all None, iter 0) when there is none."""
    if key == CHP_CP:
        checkpoint = dict(_DEFAULT_CHECKPOINT)
    elif key == CHP_BEST_M:
        checkpoint = dict(_DEFAULT_BEST_MODEL)
    elif key == CHP_TR:
        checkpoint = {CHP_TR: None}
    else:
        raise NotImplementedError(f"key: {key}.")
    iters = []
    for f in glob.glob(os.path.join(save_dir, f"*_{key}.pth")):
        m = re.findall(r"(\d+)_{}.pth".format(key), f)
        if m:
            iters.append(int(m[0]))
    for it in sorted(iters, reverse=True):
        try:
            got = torch.load(os.path.join(save_dir, f"{it}_{key}.pth"), map_location="cpu",
                             weights_only=True)
        except Exception:  # noqa: BLE001  (corrupted: try the previous one)
            continue
        checkpoint.update(got)
        return it, checkpoint
    return 0, checkpoint


def keep_last_n_checkpoints(save_dir: str, n: int, key: str = CHP_CP,
                            health: Optional[Dict[str, bool]] = None) -> List[int]:
    """utils_checkpoints.py:155-190: keep the ``n`` newest ``*_<key>.pth``; a kept file
    that fails to load is deleted too.  Returns the iterations kept."""
    assert n > 0
    health = {} if health is None else health
    iters = []
    for f in glob.glob(os.path.join(save_dir, f"*_{key}.pth")):
        m = re.findall(r"(\d+)_{}.pth".format(key), f)
        if m:
            iters.append(int(m[0]))
    kept = []
    for i, it in enumerate(sorted(iters, reverse=True)):
        path = os.path.join(save_dir, f"{it}_{key}.pth")
        if i >= n:
            os.remove(path)
            health.pop(path, None)
            continue
        try:
            if path not in health:
                torch.load(path, map_location="cpu", weights_only=True)
            health[path] = True
            kept.append(it)
        except Exception:  # noqa: BLE001  (unloadable: deleted, as the reference)
            os.remove(path)
            health.pop(path, None)
    return kept


def save_best_model(model: torch.nn.Module, task: str, save_dir: str, step: int) -> str:
    """train_wsol.py:1681-1726 (``_save_model``) -> the file path."""
    os.makedirs(save_dir, exist_ok=True)
    if task == "STD_CL":
        to_save = {"encoder": _cpu_sd(model.encoder),
                   "classification_head": _cpu_sd(model.classification_head)}
    elif task in ("F_CL", "TCAM"):
        to_save = {"encoder": _cpu_sd(model.encoder), "decoder": _cpu_sd(model.decoder),
                   "classification_head": _cpu_sd(model.classification_head),
                   "segmentation_head": _cpu_sd(model.segmentation_head)}
        rec = getattr(model, "reconstruction_head", None)
        if rec is not None:
            to_save["reconstruction_head"] = _cpu_sd(rec)
    else:
        raise NotImplementedError(task)
    path = os.path.join(save_dir, f"{step}_{CHP_BEST_M}.pth")
    torch.save(to_save, path)
    return path


def load_best_model(model: torch.nn.Module, task: str, save_dir: str) -> int:
    """instantiators.py:650-698 (eval load of the best model), strict loads; returns
    the checkpoint's step."""
    it, cpt = find_last_checkpoint(save_dir, CHP_BEST_M)
    if cpt["encoder"] is not None:
        model.encoder.super_load_state_dict(cpt["encoder"], strict=True)
    if cpt["classification_head"] is not None:
        model.classification_head.load_state_dict(cpt["classification_head"], strict=True)
    if task in ("F_CL", "TCAM"):
        if cpt["decoder"] is not None:
            model.decoder.load_state_dict(cpt["decoder"], strict=True)
        if cpt["segmentation_head"] is not None:
            model.segmentation_head.load_state_dict(cpt["segmentation_head"], strict=True)
    return it


def load_pretrained_classifier(model: torch.nn.Module, save_dir: str) -> int:
    """instantiators.py:598-625: the stage-1 STD_CL best model's encoder and
    classification head into a TCAM model (the frozen classifier of TCAM)."""
    it, cpt = find_last_checkpoint(save_dir, CHP_BEST_M)
    assert cpt["encoder"] is not None and cpt["classification_head"] is not None
    model.encoder.super_load_state_dict(cpt["encoder"], strict=True)
    model.classification_head.load_state_dict(cpt["classification_head"], strict=True)
    return it


# process/instantiators.py:746-808 (_get_model_params_for_opt).  Task TCAM (and F_CL /
# C_BOX): ONE group, ``model.parameters()`` at ``lr`` (:751-754).  Other tasks (STD_CL):
# two groups over ALL model.named_parameters() (frozen ones included).
_FEATURE_PARAM_LAYER_PATTERNS = {
    "vgg": ["encoder.features."],
    "resnet": ["encoder.layer4.", "classification_head."],
    "inception": ["encoder.Mixed", "encoder.Conv2d_1", "encoder.Conv2d_2",
                  "encoder.Conv2d_3", "encoder.Conv2d_4"],
}
_ONE_GROUP_TASKS = ("TCAM", "F_CL", "C_BOX")


def reference_param_groups(model: torch.nn.Module) -> Tuple[List[str], List[str]]:
    """(group-0 names, group-1 names) of the reference's SGD: group 0 runs at ``lr``,
    group 1 at ``lr * lr_classifier_ratio``.  ResNet50: group 1 = layer4 + classifier
    (so the decoder trains at lr); VGG16 / InceptionV3: group 0 = the feature layers (so
    the decoder is in group 1, at lr * ratio)."""
    arch = model.encoder.name if hasattr(model.encoder, "name") else "resnet50"
    pats = next(v for k, v in _FEATURE_PARAM_LAYER_PATTERNS.items() if arch.startswith(k))
    g0, g1 = [], []
    for name, _ in model.named_parameters():
        hit = any(q in name for q in pats)
        if arch.startswith("resnet"):
            (g1 if hit else g0).append(name)
        else:
            (g0 if hit else g1).append(name)
    return g0, g1


def trainable_names(model: torch.nn.Module) -> List[str]:
    """DecoderTrainer.params order: decoder.* and segmentation_head.* in named_parameters
    order."""
    return [n for n, _ in model.named_parameters()
            if n.startswith(("decoder.", "segmentation_head."))]


def _model_task(model: torch.nn.Module) -> str:
    return getattr(model, "task", "TCAM")


def optimizer_state_dict(model: torch.nn.Module, hp: dict,
                         momentum: Dict[str, torch.Tensor], lr_classifier_ratio: float = 10.,
                         task: Optional[str] = None, lrs: Optional[List[float]] = None) -> dict:
    """torch.optim.SGD.state_dict() of the reference's optimizer holding ``momentum``
    {name: buffer}.  TCAM: one group over all ``model.parameters()`` at ``hp['lr']``
    (instantiators.py:751-754); other tasks: the two groups of :func:`reference_param_groups`
    (global indices in group order), ``hp['lr']`` being the decoder's rate."""
    task = task or _model_task(model)
    if task in _ONE_GROUP_TASKS:
        layout = [([n for n, _ in model.named_parameters()], hp["lr"])]
    else:
        g0, g1 = reference_param_groups(model)
        train = set(trainable_names(model))
        dec_in_g1 = any(n in train for n in g1)
        lr0 = hp["lr"] / lr_classifier_ratio if dec_in_g1 else hp["lr"]
        lr1 = lr0 * lr_classifier_ratio
        if lrs is not None:   # the stage-1 trainer's own group rates (MyStepLR floors each)
            lr0, lr1 = lrs
        layout = [(g0, lr0), (g1, lr1)]
    groups, state, idx = [], {}, 0
    for names, lr in layout:
        ids = []
        for n in names:
            if n in momentum:
                state[idx] = {"momentum_buffer": momentum[n]}
            ids.append(idx)
            idx += 1
        groups.append({"lr": lr, "momentum": hp["momentum"], "dampening": hp["dampening"],
                       "weight_decay": hp["weight_decay"], "nesterov": hp["nesterov"],
                       "maximize": False, "foreach": None, "differentiable": False,
                       "fused": None, "params": ids})
    return {"state": state, "param_groups": groups}


def momentum_from_state_dict(model: torch.nn.Module, opt: Optional[dict]) -> Dict[str, torch.Tensor]:
    """{parameter name: momentum buffer} from an SGD state_dict: the reference's TCAM
    layout (one group over every model parameter), its two-group layout of the other
    tasks, or this module's round-1 files (one group over the trainable parameters)."""
    if not opt:
        return {}
    groups = opt.get("param_groups", [])
    ids = [i for g in groups for i in g["params"]]
    every = [n for n, _ in model.named_parameters()]
    if len(groups) == 2:
        g0, g1 = reference_param_groups(model)
        names = g0 + g1
    elif len(ids) == len(every):
        names = every
    else:
        names = trainable_names(model)
    if len(ids) != len(names):
        raise ValueError(f"optimizer state has {len(ids)} parameters, the model {len(every)}")
    pos = {pid: names[k] for k, pid in enumerate(ids)}
    out = {}
    for pid, st in opt.get("state", {}).items():
        buf = st.get("momentum_buffer")
        if buf is not None:
            out[pos[int(pid)]] = buf
    return out


def _loss_t(t: float, use=(True, True, True), rgb: bool = False) -> list:
    """MasterLoss.get_t() (losses/master.py:37-41): one [name, t] per instantiated loss in
    get_loss_tcam's order (instantiators.py:148-245: CRF, RGB joint CRF, max-size,
    self-learning); only the ELB-carrying MaxSizePositiveTcams has a t.  ``use`` = (sl,
    crf, size) enabled, ``rgb`` = RgbJointConRanFieldTcams instantiated."""
    sl, crf, size = use
    out = []
    if crf:
        out.append(["con_ran_field_tcams", 0.0])
    if rgb:
        out.append(["rgb_joint_con_ran_field_tcams", 0.0])
    if size:
        out.append(["max_size_positive_tcams", float(t)])
    if sl:
        out.append(["self_learning_tcams", 0.0])
    return out


def _t_from(v) -> Optional[float]:
    if v is None:
        return None
    if isinstance(v, (list, tuple)):
        for name, t in v:
            if name == "max_size_positive_tcams":
                return float(t)
        return None
    return float(torch.as_tensor(v).reshape(-1)[0])


def save_checkpoint(trainer, save_dir: str, current_step: int, key: str = CHP_CP,
                    lr_classifier_ratio: float = 10., lr_scheduler=None) -> str:
    """utils_checkpoints.py:193-213 for a :class:`~.training.DecoderTrainer`: 'model' = the
    full model state_dict (CPU), 'optimizer' = the reference SGD's state_dict (TCAM: one
    group over all model parameters, instantiators.py:746-754, 811-841), 'lr_scheduler' =
    the scheduler's state_dict ({} without one), 't' = MasterLoss.get_t()."""
    os.makedirs(save_dir, exist_ok=True)
    mom = {}
    if trainer.momentum != 0 and trainer.applied_steps > 0:
        off = 0
        for name, p in zip(_trainer_names(trainer), trainer.params):
            k = p.numel()
            mom[name] = trainer.mom[off:off + k].view(p.shape).cpu().clone()
            off += k
    hp = {"lr": trainer.lr, "momentum": trainer.momentum, "dampening": trainer.dampening,
          "weight_decay": trainer.weight_decay, "nesterov": trainer.nesterov}
    ratio = getattr(trainer, "lr_ratio", lr_classifier_ratio)
    if hasattr(trainer, "loss_t"):     # stage 1: MasterLoss([ClLoss]).get_t()
        t = trainer.loss_t()
    else:
        t = _loss_t(trainer.elb.t, trainer.use_cfg, getattr(trainer, "rgb_cfg", None) is not None)
    path = os.path.join(save_dir, f"{current_step}_{key}.pth")
    torch.save({CHP_M: _cpu_sd(trainer.model),
                CHP_O: optimizer_state_dict(trainer.model, hp, mom, ratio,
                                            lrs=getattr(trainer, "lrs", None)),
                CHP_LR: lr_scheduler.state_dict() if lr_scheduler is not None else {},
                CHP_T: t, "iter": current_step}, path)
    return path


def _trainer_names(trainer) -> List[str]:
    """The parameter names of a trainer's flat buffer, in its order (DecoderTrainer: the
    decoder + seg head; ClassifierTrainer: every model parameter)."""
    if hasattr(trainer, "trainable_names"):
        return trainer.trainable_names()
    return trainable_names(trainer.model)


def load_checkpoint(trainer, save_dir: str, key: str = CHP_CP, lr_scheduler=None) -> int:
    """Resume a DecoderTrainer from the newest ``*_checkpoint.pth`` (ours or the
    reference's: main.py:38-59); returns its iter (0 and nothing loaded when there is
    none).  The model load is strict and in place (the trainer's flat parameter buffer
    is written through the Parameters' views); the frozen encoder's plan re-folds on the
    next forward."""
    it, cpt = find_last_checkpoint(save_dir, key)
    if cpt[CHP_M] is None:
        return 0
    trainer.model.load_state_dict(cpt[CHP_M], strict=True)
    if not trainer.views_intact():
        raise RuntimeError("load_checkpoint: the trainer no longer views the parameters")
    mom = momentum_from_state_dict(trainer.model, cpt[CHP_O])
    trainer.mom.zero_()
    off = 0
    for name, p in zip(_trainer_names(trainer), trainer.params):
        k = p.numel()
        if name in mom:
            trainer.mom[off:off + k].copy_(mom[name].reshape(-1))
        off += k
    trainer.steps = 1 if mom else 0
    for cnt in (trainer.step_counts, getattr(trainer, "_counts_g1", None)):
        if cnt is None:
            continue
        cnt.zero_()
        if mom:     # momentum present: the next step is not the optimizer's first
            cnt[0] = 1
    t = _t_from(cpt[CHP_T])
    if t is not None and hasattr(trainer, "elb"):
        trainer.elb.t = t
    if lr_scheduler is not None and cpt[CHP_LR]:
        lr_scheduler.load_state_dict(cpt[CHP_LR])     # main.py:56-57
    trainer.repack()
    from .training import DECODER_PLANS
    trainer.model.invalidate_plans(DECODER_PLANS + ("enc_x6", "enc_f16x3", "enc_amp", "enc"))
    return it


# ------------------------------------------------- performance tracker (model selection)
# train_wsol.py:1280-1325: ``{step}_tracker.pth`` = {"tracker": {split: {metric: vars(
# PerformanceMeter)}}} next to the checkpoints, restored on resume so that the first
# validation after a resume does not count as the best one.  The runner's meters are the
# validation split's localization (best_loc) and classification (best_cl) values.
_MTR = {"best_loc": "localization", "best_cl": "classification"}


def _meter(values: List[float]) -> dict:
    if not values:
        return {"current_value": None, "best_value": None, "best_epoch": None,
                "value_per_epoch": []}
    best = max(values)
    return {"current_value": values[-1], "best_value": best,
            "best_epoch": values.index(best), "value_per_epoch": list(values)}


def save_tracker(save_dir: str, step: int, meters: Dict[str, List[float]]) -> str:
    os.makedirs(save_dir, exist_ok=True)
    path = os.path.join(save_dir, f"{step}_{CHP_TR}.pth")
    torch.save({CHP_TR: {"val": {_MTR[k]: _meter(v) for k, v in meters.items()}}}, path)
    return path


def load_tracker(save_dir: str) -> Dict[str, List[float]]:
    """The validation meters of the newest tracker file ({} when there is none)."""
    _, cpt = find_last_checkpoint(save_dir, CHP_TR)
    tr = cpt.get(CHP_TR)
    if not tr or "val" not in tr:
        return {}
    out = {}
    for k, m in _MTR.items():
        if m in tr["val"]:
            out[k] = [float(v) for v in tr["val"][m]["value_per_epoch"]]
    return out
