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
from typing import Dict, Optional, Tuple

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


def save_checkpoint(trainer, save_dir: str, current_step: int, key: str = CHP_CP) -> str:
    """utils_checkpoints.py:193-213 for a :class:`~.training.DecoderTrainer`:
    'model' = the full model state_dict (CPU), 'optimizer' = torch.optim.SGD's
    state_dict layout over the trainer's parameters (decoder + segmentation head,
    named_parameters order), 'lr_scheduler' = {} (constant lr), 't' = ELB t."""
    os.makedirs(save_dir, exist_ok=True)
    group = {"lr": trainer.lr, "momentum": trainer.momentum, "dampening": trainer.dampening,
             "weight_decay": trainer.weight_decay, "nesterov": trainer.nesterov,
             "maximize": False, "foreach": None, "differentiable": False,
             "fused": None, "params": list(range(len(trainer.params)))}
    state = {}
    if trainer.steps > 0 and trainer.momentum != 0:
        off = 0
        for i, p in enumerate(trainer.params):
            k = p.numel()
            state[i] = {"momentum_buffer": trainer.mom[off:off + k].view(p.shape).cpu().clone()}
            off += k
    path = os.path.join(save_dir, f"{current_step}_{key}.pth")
    t = torch.tensor([float(trainer.elb.t)], dtype=torch.float64)
    torch.save({CHP_M: _cpu_sd(trainer.model),
                CHP_O: {"state": state, "param_groups": [group]},
                CHP_LR: {}, CHP_T: t, "iter": current_step}, path)
    return path


def load_checkpoint(trainer, save_dir: str, key: str = CHP_CP) -> int:
    """Resume a DecoderTrainer from the newest ``*_checkpoint.pth``; returns its iter
    (0 and nothing loaded when there is none)."""
    it, cpt = find_last_checkpoint(save_dir, key)
    if cpt[CHP_M] is None:
        return 0
    trainer.model.load_state_dict(cpt[CHP_M], strict=True)
    # the trainer views parameters / BN buffers through flat buffers: refresh them
    off = 0
    for p in trainer.params:
        k = p.numel()
        trainer.flat[off:off + k].copy_(p.detach().reshape(-1))
        p.data = trainer.flat[off:off + k].view(p.shape)
        off += k
    off = 0
    for bn in trainer.bns:
        k = bn.num_features
        for name in ("running_mean", "running_var"):
            t = getattr(bn, name)
            trainer.bn_flat[off:off + k].copy_(t)
            setattr(bn, name, trainer.bn_flat[off:off + k])
            off += k
    opt: Optional[dict] = cpt[CHP_O]
    state = (opt or {}).get("state", {})
    trainer.mom.zero_()
    off = 0
    for i, p in enumerate(trainer.params):
        k = p.numel()
        st = state.get(i)
        if st is not None and st.get("momentum_buffer") is not None:
            trainer.mom[off:off + k].copy_(st["momentum_buffer"].reshape(-1))
        off += k
    trainer.steps = 1 if state else 0
    if cpt[CHP_T] is not None:
        trainer.elb.t = float(torch.as_tensor(cpt[CHP_T]).reshape(-1)[0])
    trainer.repack()
    return it
