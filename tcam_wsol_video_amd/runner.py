"""The reference's entry points over the device path: ``eval.py`` (the evaluation the
reference's broken eval.py intends, SURVEY.md §0.7: best model -> CAMComputer over a
split -> BoxAcc) and ``main.py`` (the TCAM training loop, /root/reference main.py:33-167
with learning/train_wsol.py's per-batch work).

Data: the reference's WSOL metadata layout (datasets/wsol_loader.py:64-180) —
``<metadata_root>/{image_ids,class_labels,image_sizes,localization}.txt`` — with frames
under ``--data_root`` decoded on the device (``--jpeg_decode device``, the default:
csrc/jpeg.hip, bit-identical to the reference's Image.open(...).convert('RGB'); non-JPEG
files and ``--jpeg_decode host`` use PIL on the host), or ``--synthetic N`` seeded
YTOv2.2-shaped clips when no dataset is present.  Everything after the
file read runs on the device: decode, frame transforms, forward, CAM, bbox sweep,
counters, seeding, losses, backward, SGD.

Multi-GPU: one process per GPU (torchrun); eval shards frames with the reference's
DistributedSampler order (padding duplicates counted, wsol_loader.py:1008-1012) and
all-reduces the counters; training is DDP-equivalent (DecoderTrainer's RCCL all-reduce).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import checkpoints as CK
from . import frames as FR
from . import ops
from .camstore import get_cams_paths
from .inference import CAMComputer
from .metrics import resize_bbox
from .models import TCAM, STD_CL, create_model
from .parallel import TemporalCAM, distributed_sampler_indices, knn_window, rank_world

CROP_SIZE = 224     # constants.CROP_SIZE
RESIZE_SIZE = 256   # constants.RESIZE_SIZE (train Resize before RandomCrop)
# constants.py:189-194, 294: the datasets whose validation sweep uses the fast tau grid
YTOV1, YTOV22 = "YouTube-Objects-v1.0", "YouTube-Objects-v2.2"
FAST_VALID_DATASETS = ("CUB", "ILSVRC", YTOV1, YTOV22)
VALID_FAST_CAM_CURVE_INTERVAL = .004


def _bool(s: str) -> bool:
    if s.lower() in ("true", "1", "yes"):
        return True
    if s.lower() in ("false", "0", "no"):
        return False
    raise argparse.ArgumentTypeError(s)


def parser(train: bool) -> argparse.ArgumentParser:
    """The TCAM subset of parseit.get_args (parseit.py:82-579), same flag names."""
    ap = argparse.ArgumentParser(description="TCAM " + ("training" if train else "evaluation"))
    a = ap.add_argument
    a("--task", default=TCAM, choices=(TCAM, STD_CL))
    a("--dataset", default=YTOV22,
      help="dataset name (constants.py:189-194); CUB / ILSVRC / YTO validate at 250 tau")
    a("--encoder_name", default="resnet50", choices=("resnet50", "vgg16", "inceptionv3"))
    a("--arch", default=None)
    a("--method", default="CAM")
    a("--spatial_pooling", default="WGAP", choices=("WGAP",))
    a("--num_classes", type=int, default=10)
    a("--batch_size", type=int, default=32)
    a("--crop_size", type=int, default=CROP_SIZE)
    a("--cam_curve_interval", type=float, default=.001)
    a("--box_v2_metric", type=_bool, default=False)
    a("--metadata_root", default=None, help="folder with the split sub-folders of metadata")
    a("--data_root", default=None)
    a("--synthetic", type=int, default=0, help="N synthetic 32-frame clips per split")
    a("--jpeg_decode", default="device", choices=("device", "host"),
      help="JPEG frames: device decode (csrc/jpeg.hip) or PIL on the host")
    a("--exp_path", default="exp")
    a("--dist_backend", default="nccl", choices=("nccl", "gloo"))
    a("--sl_tc_knn", type=int, default=0)
    a("--sl_tc_knn_mode", default="instant")
    a("--sl_tc_knn_t", type=float, default=0.0)
    a("--sl_tc_min_t", type=float, default=0.0)
    a("--sl_tc_knn_epoch_switch_uniform", type=int, default=-1)
    a("--fwd_streams", type=int, default=2)
    a("--seed", type=int, default=0)
    # config.py:477-478: autocast fp16 convolutions for training / for inference
    a("--amp", type=_bool, default=False)
    a("--amp_eval", type=_bool, default=False)
    if train:
        # TCAM trains with freeze_cl=True; STD_CL (stage 1) with the classifier unfrozen
        # (parseit.py:873-875 asserts not freeze_cl) — the default follows --task
        a("--freeze_cl", type=_bool, default=None)
        # config.py:236-238: an encoder-freezing switch of C_BOX; stage 1 trains the encoder
        a("--freeze_encoder", type=_bool, default=False)
        a("--support_background", type=_bool, default=False,
          help="accepted for the README's stage-1 command; WGAP has no background class "
               "(poolings/core.py:96-115)")
        a("--opt__lr_classifier_ratio", type=float, default=10.0)
        a("--max_epochs", type=int, default=1)
        a("--checkpoint_save", type=int, default=100)
        a("--keep_last_n_checkpoints", type=int, default=2)   # config.py:171
        a("--opt__lr", type=float, default=0.01)
        a("--opt__momentum", type=float, default=0.9)
        a("--opt__dampening", type=float, default=0.0)
        a("--opt__nesterov", type=_bool, default=True)
        a("--opt__weight_decay", type=float, default=1e-4)
        a("--opt__lr_scheduler", type=_bool, default=True)
        a("--opt__name_lr_scheduler", default="mystep", choices=("mystep",))
        a("--opt__step_size", type=int, default=40)
        a("--opt__gamma", type=float, default=0.1)
        a("--opt__min_lr", type=float, default=1e-7)
        a("--elb_init_t", type=float, default=1.0)
        a("--elb_max_t", type=float, default=10.0)
        a("--elb_mulcoef", type=float, default=1.01)
        a("--sl_tc", type=_bool, default=True)
        a("--sl_tc_lambda", type=float, default=1.0)
        a("--sl_tc_min", type=int, default=1)
        a("--sl_tc_max", type=int, default=1)
        a("--sl_tc_ksz", type=int, default=3)
        a("--sl_tc_max_p", type=float, default=0.6)
        a("--sl_tc_min_p", type=float, default=0.1)
        a("--sl_tc_fg_erode_k", type=int, default=11)
        a("--sl_tc_fg_erode_iter", type=int, default=0)
        a("--sl_tc_seed_tech", default="seed_weighted")
        a("--sl_tc_use_roi", type=_bool, default=True)
        a("--sl_tc_roi_method", default="roi_all")
        a("--sl_tc_roi_min_size", type=float, default=0.05)
        a("--crf_tc", type=_bool, default=True)
        a("--crf_tc_lambda", type=float, default=2e-9)
        a("--crf_tc_sigma_rgb", type=float, default=15.0)
        a("--crf_tc_sigma_xy", type=float, default=100.0)
        a("--crf_tc_scale", type=float, default=1.0)
        a("--max_sizepos_tc", type=_bool, default=True)
        a("--max_sizepos_tc_lambda", type=float, default=0.01)
        # per-term epoch windows (config.py:400-449; end -1 = never stops, core.py:48-49)
        for t in ("sl_tc", "crf_tc", "max_sizepos_tc", "rgb_jcrf_tc"):
            a(f"--{t}_start_ep", type=int, default=0)
            a(f"--{t}_end_ep", type=int, default=-1)
        # RgbJointConRanFieldTcams over knn_tc frame groups (config.py:370-375, 436-442)
        a("--knn_tc", type=int, default=0,
          help="frames each side of a sampled frame (batch = batch_size // (2 knn_tc + 1) "
               "shots, parseit.py:642-643); needs a shot-indexed train split")
        a("--rgb_jcrf_tc", type=_bool, default=False)
        a("--rgb_jcrf_tc_lambda", type=float, default=2e-9)
        a("--rgb_jcrf_tc_sigma_rgb", type=float, default=15.0)
        a("--rgb_jcrf_tc_scale", type=float, default=1.0)
        a("--std_cams_folder", default=None, help="stage-1 CAMs <id>.pt (camstore layout)")
        a("--std_cams_thresh_file", default=None,
          help="train split's id,thresh ROI file (camstore.write_roi_file layout)")
        a("--pretrained_classifier", default=None, help="folder of the STD_CL best model")
        a("--final_test_eval", type=_bool, default=True,
          help="main.py:117-160: evaluate the test split with the best_loc and best_cl "
               "models after training (needs a test split: --synthetic or <metadata>/test)")
    else:
        a("--checkpoint", default=None, help="folder holding <step>_best_model.pth")
        a("--splits", default="test")
    return ap


# ------------------------------------------------------------------ data
def _read_lines(path: str) -> List[str]:
    with open(path) as f:
        return [ln.strip("\n") for ln in f.readlines() if ln.strip("\n")]


def load_metadata(metadata_root: str):
    """wsol_loader.py:64-180: (ids, {id: label}, {id: [(x0,y0,x1,y1)]}, {id: (w, h)})."""
    ids = _read_lines(os.path.join(metadata_root, "image_ids.txt"))
    labels = {}
    for ln in _read_lines(os.path.join(metadata_root, "class_labels.txt")):
        i, c = ln.split(",")
        labels[i] = int(c)
    boxes: Dict[str, list] = {}
    for ln in _read_lines(os.path.join(metadata_root, "localization.txt")):
        i, a, b, c, d = ln.split(",")
        boxes.setdefault(i, []).append((float(a), float(b), float(c), float(d)))
    sizes = {}
    for ln in _read_lines(os.path.join(metadata_root, "image_sizes.txt")):
        i, w, h = ln.split(",")
        sizes[i] = (int(w), int(h))
    return ids, labels, boxes, sizes


class Split:
    """One split's frames, labels and GT boxes resized to the crop (resize_bbox).

    ``shot_ids`` (optional): the split is indexed by shots (constants.DS_SHOTS,
    wsol_loader.py:375-422 — the YTO train splits, whose metadata lists shot folders):
    the dataset index is a shot, ``ids`` are all its frames (sorted file names), and
    training draws one frame per shot per epoch (:520-560)."""

    def __init__(self, ids, labels, gt, frame_fn, std_cam_fn=None, bytes_fn=None,
                 shot_ids: Optional[Sequence[str]] = None):
        self.ids: List[str] = list(ids)
        self.labels: Dict[str, int] = labels
        self.gt: Dict[str, List[Tuple[int, int, int, int]]] = gt
        self.frame_fn = frame_fn          # id -> (H, W, 3) uint8
        self.std_cam_fn = std_cam_fn      # id -> (h', w') float32 stage-1 CAM
        self.bytes_fn = bytes_fn          # id -> JPEG file bytes (device decode), or None
        shots: Dict[str, List[str]] = {}
        for i in self.ids:
            shots.setdefault(os.path.dirname(i), []).append(i)
        self.shot_of = {i: s for s, fr in shots.items() for i in fr}
        self.shots = {s: sorted(fr) for s, fr in shots.items()}
        self.shot_ids: Optional[List[str]] = list(shot_ids) if shot_ids is not None else None

    def __len__(self):
        return len(self.ids)

    @classmethod
    def from_metadata(cls, metadata_root: str, data_root: str, crop: int,
                      std_cams_folder: Optional[str] = None,
                      jpeg_decode: str = "device") -> "Split":
        from PIL import Image
        ids = _read_lines(os.path.join(metadata_root, "image_ids.txt"))
        shot_ids = None
        if ids and os.path.isdir(os.path.join(data_root, ids[0])):
            # DS_SHOTS (get_dataset_mode / index_frames_from_shots, wsol_loader.py:375-422):
            # frames = the shot folder's *.jpg, sorted by name
            labels = {}
            for ln in _read_lines(os.path.join(metadata_root, "class_labels.txt")):
                i, c = ln.split(",")
                labels[i] = int(c)
            shot_ids, frames = ids, []
            for sh in shot_ids:
                fr = sorted(f for f in os.listdir(os.path.join(data_root, sh))
                            if f.endswith(".jpg") and
                            os.path.isfile(os.path.join(data_root, sh, f)))
                if not fr:
                    raise ValueError(f"empty shot {sh} (wsol_loader.py:412)")
                for f in fr:
                    fid = os.path.join(sh, f)
                    frames.append(fid)
                    labels[fid] = labels[sh]
            ids, gt = frames, {i: [] for i in frames}
        else:
            ids, labels, boxes, sizes = load_metadata(metadata_root)
            gt = {i: [resize_bbox(b, sizes[i], (crop, crop)) for b in boxes.get(i, [])]
                  for i in ids}

        def frame(i):
            with Image.open(os.path.join(data_root, i)) as im:
                return np.asarray(im.convert("RGB"))

        std = None
        if std_cams_folder:
            paths = get_cams_paths(std_cams_folder, ids)

            def std(i):
                return torch.load(paths[i], map_location="cpu", weights_only=True)

        def raw(i):
            if not i.lower().endswith((".jpg", ".jpeg")):
                return None
            with open(os.path.join(data_root, i), "rb") as f:
                return f.read()
        return cls(ids, labels, gt, frame, std, raw if jpeg_decode == "device" else None,
                   shot_ids)

    @classmethod
    def synthetic(cls, n_clips: int, crop: int, seed: int, frames_per_clip: int = 32,
                  classes: int = 10, by_shots: bool = False) -> "Split":
        from .utils.seeding import synthetic_boxes, synthetic_clip
        clips, ids, labels, gt = {}, [], {}, {}
        rng = np.random.default_rng(seed)
        for k in range(n_clips):
            clip = synthetic_clip(frames_per_clip, seed=seed * 1000 + k)
            bx = synthetic_boxes(clip, crop)
            c = int(rng.integers(0, classes))
            for t in range(frames_per_clip):
                i = f"synthetic/{k:04d}/shots/000/frame{t:04d}.jpg"
                clips[i] = clip[t]
                ids.append(i)
                labels[i] = c
                gt[i] = [tuple(int(v) for v in bx[t])]
        cam_rng = np.random.default_rng(seed + 7)
        std_cams = {i: torch.from_numpy(cam_rng.random((28, 28)).astype(np.float32)) for i in ids}
        shot_ids = [f"synthetic/{k:04d}/shots/000" for k in range(n_clips)] if by_shots else None
        return cls(ids, labels, gt, clips.__getitem__, std_cams.__getitem__,
                   shot_ids=shot_ids)


def _decode(split: Split, ids: Sequence[str], dev) -> list:
    """Frames as (H, W, 3) uint8: JPEG files decoded on the device in one batch
    (jpeg.JpegDecoder), anything else through split.frame_fn on the host."""
    if split.bytes_fn is None:
        return [split.frame_fn(i) for i in ids]
    datas = [split.bytes_fn(i) for i in ids]
    jp = [k for k, d in enumerate(datas) if d is not None]
    out = [None] * len(ids)
    if jp:
        from . import jpeg
        dec = jpeg.decode([datas[k] for k in jp], dev, names=[ids[k] for k in jp])
        for k, t in zip(jp, dec):
            out[k] = t
    for k, d in enumerate(datas):
        if d is None:
            out[k] = split.frame_fn(ids[k])
    return out


def device_frames(split: Split, ids: Sequence[str], dev, transform, **kw):
    """Decode (device for JPEG files, else host) and transform (device, frames.preprocess)
    a batch; frames of different sizes go through the transform in same-size groups."""
    imgs = _decode(split, ids, dev)
    norm = torch.empty(len(ids), 3, transform.crop_size, transform.crop_size, device=dev)
    raw = torch.empty_like(norm)
    start = 0
    while start < len(imgs):
        end = start + 1
        while end < len(imgs) and imgs[end].shape == imgs[start].shape:
            end += 1
        grp = imgs[start:end]
        if all(isinstance(g, torch.Tensor) for g in grp):
            u8 = torch.stack(grp)
        else:
            u8 = torch.from_numpy(np.ascontiguousarray(np.stack(
                [g.cpu().numpy() if isinstance(g, torch.Tensor) else g for g in grp]))).to(dev)
        sub = {k: (v[start:end] if v is not None else None) for k, v in kw.items()}
        n, r = transform(u8, **sub)
        norm[start:end] = n
        raw[start:end] = r
        start = end
    return norm, raw


def _gt_tensor(split: Split, ids, dev):
    g = max(1, max(len(split.gt[i]) for i in ids))
    gt = np.zeros((len(ids), g, 4), np.int32)
    ngt = np.zeros(len(ids), np.int32)
    for b, i in enumerate(ids):
        boxes = split.gt[i]
        ngt[b] = len(boxes)
        if boxes:
            gt[b, :len(boxes)] = np.asarray(boxes, np.int32)
    return torch.from_numpy(gt).to(dev), torch.from_numpy(ngt).to(dev)


# ----------------------------------------------------------------- eval
def evaluate(model, split: Split, args, dev, collect: Optional[dict] = None,
             cam_curve_interval: Optional[float] = None) -> dict:
    """CAMComputer.compute_and_evaluate_cams over a split (inference_wsol.py:432-457) with
    the reference's sharding, counters all-reduced across ranks.  ``collect`` (tests): a
    dict that receives {frame id: (cam fp32, cam uint8, logits)} as host tensors.
    ``cam_curve_interval``: the tau step (default ``args.cam_curve_interval``)."""
    rank, world = rank_world()
    if split.shot_ids is not None:
        raise NotImplementedError("evaluation of a shot-indexed split (the YTO eval splits "
                                  "list frames)")
    if cam_curve_interval is None:
        cam_curve_interval = args.cam_curve_interval
    temporal = None
    if args.sl_tc_knn_mode != "instant" or args.sl_tc_knn:
        temporal = TemporalCAM(args.sl_tc_knn, args.sl_tc_knn_mode, args.sl_tc_knn_t)
    # box_v2_metric -> multi_contour_eval = multi_iou_eval = True (parseit.py:684-689)
    comp = CAMComputer(model, cam_curve_interval=cam_curve_interval, device=dev,
                       fwd_streams=args.fwd_streams if temporal is None else 1,
                       temporal=temporal, multi_contour_eval=bool(args.box_v2_metric))
    if temporal is None:
        order = distributed_sampler_indices(len(split), rank, world)
        batches = [order[k:k + args.batch_size] for k in range(0, len(order), args.batch_size)]
    else:
        # CAM-TMP needs a shot's neighbouring frames: each call is this rank's contiguous
        # shard of one shot, the rest of the shot is all-gathered (parallel.TemporalCAM)
        pos = {i: j for j, i in enumerate(split.ids)}
        batches = []
        for shot in split.shots.values():
            if len(shot) % world:
                raise ValueError(f"temporal eval: shot of {len(shot)} frames over {world} ranks")
            per = len(shot) // world
            batches.append([pos[f] for f in shot[rank * per:(rank + 1) * per]])
    tf = FR.get_eval_tranforms(args.crop_size)
    t0 = time.perf_counter()
    nframes = 0
    for b in batches:
        ids = [split.ids[j] for j in b]
        nframes += len(ids)
        x, _ = device_frames(split, ids, dev, tf)
        targets = torch.tensor([split.labels[i] for i in ids], device=dev)
        gt, ngt = _gt_tensor(split, ids, dev)
        u8 = comp.evaluate_batch(x, targets, gt, ngt)
        if collect is not None:
            comp.synchronize()
            for j, i in enumerate(ids):
                collect[i] = (comp.last_cam[j].cpu(), u8[j].cpu(), comp.last_logits[j].cpu())
    acc = comp.compute_and_evaluate()
    dt = time.perf_counter() - t0
    ev = comp.evaluator
    # Trainer.evaluate's model-selection score (train_wsol.py:1515-1519): the mean BoxAcc
    # over the IoU thresholds with multi_iou_eval (box_v2_metric), else BoxAcc@50
    if args.box_v2_metric:
        loc = float(np.average(acc))
    else:
        loc = float(acc[ev.iou_threshold_list.index(50)])
    return {"BoxAcc": [float(a) for a in acc], "iou_thresholds": ev.iou_threshold_list,
            "localization": loc, "box_v2_metric": bool(args.box_v2_metric),
            # _compute_accuracy (train_wsol.py:1400-1435): argmax(cl_logits) == target
            "classification_acc": ev.classification_accuracy(),
            "top1_loc": [float(a) for a in ev.top1], "top5_loc": [float(a) for a in ev.top5],
            "best_tau": ev.best_tau_list, "frames": int(ev.cnt),
            "cam_curve_interval": cam_curve_interval,
            "frames_per_s_rank0": round(nframes / dt, 1)}


def _init_dist(args) -> torch.device:
    if not torch.cuda.is_available():
        raise SystemExit("tcam_wsol_video_amd runs on the MI355X HIP path only. The reference's "
                         "CPU evaluation is restated in oracle/ (test infrastructure).")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(args.dist_backend)
    return torch.device("cuda", local)


def _model_kwargs(args):
    from .backbones import encoder_depth_channels
    depth, dec = encoder_depth_channels(args.encoder_name)
    aux = dict(pooling_head=args.spatial_pooling, classes=args.num_classes,
               support_background=False)
    if args.task == TCAM:
        return dict(task=TCAM, arch="UnetTCAM", encoder_name=args.encoder_name,
                    encoder_depth=depth, decoder_channels=dec, seg_h_out_channels=2,
                    aux_params=aux, freeze_cl=True)
    return dict(task=STD_CL, arch="STDClassifier", encoder_name=args.encoder_name,
                encoder_depth=depth, aux_params=aux)


def _splits(args, names: Sequence[str]) -> Dict[str, Split]:
    out = {}
    for k, n in enumerate(names):
        if args.synthetic:
            # knn_tc needs a shot-indexed train split (wsol_loader.py:483-486): the
            # synthetic clips are then one shot each
            by_shots = n == "train" and getattr(args, "knn_tc", 0) > 0
            out[n] = Split.synthetic(args.synthetic, args.crop_size, seed=args.seed + 101 * k,
                                     classes=args.num_classes, by_shots=by_shots)
        else:
            if not (args.metadata_root and args.data_root):
                raise SystemExit("--metadata_root and --data_root (or --synthetic N) required")
            out[n] = Split.from_metadata(os.path.join(args.metadata_root, n), args.data_root,
                                         args.crop_size,
                                         getattr(args, "std_cams_folder", None),
                                         getattr(args, "jpeg_decode", "device"))
    return out


def eval_main(argv=None, collect: Optional[dict] = None) -> int:
    args = parser(train=False).parse_args(argv)
    dev = _init_dist(args)
    model = create_model(**_model_kwargs(args))
    if args.checkpoint:
        step = CK.load_best_model(model, args.task, args.checkpoint)
    else:
        from .utils.seeding import seed_module_
        seed_module_(model, args.seed)
        step = None
    model = model.to(dev).eval()
    if args.amp_eval:   # inference_wsol.py:258-302: autocast(enabled=amp_eval)
        model.conv_precision = "amp"
    res = {}
    for name, split in _splits(args, args.splits.split(",")).items():
        res[name] = evaluate(model, split, args, dev, collect)
    rank, world = rank_world()
    if rank == 0:
        print(json.dumps({"task": args.task, "encoder": args.encoder_name, "checkpoint_step": step,
                          "world": world, "results": res}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


# ---------------------------------------------------------------- train
def _std_cams_batch(split: Split, ids, args, dev, t: float = 0.0) -> torch.Tensor:
    """The loader's CAM-TMP (wsol_loader.py:571-601): max over the sl_tc_knn neighbour
    frames of each frame's shot of the stage-1 CAMs, (B, 1, h', w') on the device, each
    heated with ``t`` first only when sl_tc_knn > 0 (:571, 594; ``decay_temp.heat_t``)."""
    from .decay_temp import heat_t
    k, mode = args.sl_tc_knn, args.sl_tc_knn_mode
    need, rows = {}, []
    for i in ids:
        shot = split.shots[split.shot_of[i]]
        w = knn_window(len(shot), k, mode)[shot.index(i)]
        row = []
        for j in w:
            if j < 0:
                row.append(-1)
                continue
            fid = shot[int(j)]
            if fid not in need:
                need[fid] = len(need)
            row.append(need[fid])
        rows.append(row)
    cams = torch.stack([split.std_cam_fn(f).float() for f in need]).to(dev)
    idx = torch.tensor(rows, dtype=torch.int32, device=dev)
    return ops.temporal_max(cams.contiguous(), idx, heat_t(k, t))[:, None]


def knn_frames(frames: Sequence[str], f: int, k: int) -> List[str]:
    """The knn_tc group of frame f of a shot (wsol_loader.py:447-458, 492-497): up to k
    frames before, the frame, up to k after — ``_get_right_knn`` slices from
    min(f + 1, n - 1), so the last frame of a shot is its own right neighbour."""
    n = len(frames)
    left = list(frames[max(0, f - k):f])
    right = list(frames[min(f + 1, n - 1):min(f + k + 1, n)])
    return left + [frames[f]] + right


def train_batches(train: Split, args, rank: int, world: int, epoch: int,
                  rng: np.random.Generator):
    """The train loader's batches for one epoch: lists (frame ids, seq_iter, frm_iter).

    Frame-indexed split: the DistributedSampler(shuffle) order over frames, batch_size
    frames, seq/frm None.  Shot-indexed split (DS_SHOTS): the sampler runs over shots with
    batch_size // (2 knn_tc + 1) shots per batch (parseit.py:642-643); each shot gives one
    random frame (wsol_loader.py:535-560) or, with knn_tc > 0, its knn group
    (:479-503) whose frames carry seq_iter = the shot's index and frm_iter = the position
    in the group (:616-624), collated flat (_temporal_default_collate, :881-900)."""
    k = getattr(args, "knn_tc", 0)
    if train.shot_ids is None:
        if k > 0:
            raise SystemExit("--knn_tc needs a shot-indexed train split (metadata listing shot "
                             "folders, wsol_loader.py:483-486)")
        order = distributed_sampler_indices(len(train), rank, world, shuffle=True,
                                            seed=args.seed, epoch=epoch)
        for s in range(0, len(order), args.batch_size):
            yield [train.ids[j] for j in order[s:s + args.batch_size]], None, None
        return
    per = args.batch_size // (2 * k + 1) if k > 0 else args.batch_size
    if per <= 0:
        raise SystemExit(f"batch_size {args.batch_size} < 2 knn_tc + 1 (parseit.py:644)")
    order = distributed_sampler_indices(len(train.shot_ids), rank, world, shuffle=True,
                                        seed=args.seed, epoch=epoch)
    for s in range(0, len(order), per):
        ids, seq, frm = [], [], []
        for idx in order[s:s + per]:
            frames = train.shots[train.shot_ids[idx]]
            f = int(rng.integers(0, len(frames)))
            group = knn_frames(frames, f, k) if k > 0 else [frames[f]]
            for i, fid in enumerate(group):
                ids.append(fid)
                seq.append(float(idx))
                frm.append(float(i))
        yield ids, seq, frm


def train_main(argv=None) -> int:
    """main.py:33-167 + Trainer.train (train_wsol.py:944-1233) for task TCAM."""
    from .camstore import load_roi_thresholds
    from .decay_temp import DecayTemp
    from .losses import ELB
    from .seeding import GetRoiSingleCam, TCAMSeeder, prepare_std_cams
    from .training import DecoderTrainer, fill_minibatch, lr_schedule
    args = parser(train=True).parse_args(argv)
    if args.freeze_cl is None:
        args.freeze_cl = args.task == TCAM
    if args.task == STD_CL:
        return train_stdcl_main(args)
    if args.task != TCAM or not args.freeze_cl:
        raise SystemExit("main.py trains TCAM with freeze_cl=True (README.md:273-340)")
    if args.rgb_jcrf_tc and args.knn_tc <= 0:
        raise SystemExit("--rgb_jcrf_tc needs --knn_tc > 0 (parseit.py:912-913)")
    dev = _init_dist(args)
    rank, world = rank_world()
    model = create_model(**_model_kwargs(args))
    from .utils.seeding import seed_module_
    seed_module_(model, args.seed)
    if args.pretrained_classifier:
        CK.load_pretrained_classifier(model, args.pretrained_classifier)
    model = model.to(dev)
    # the loader's temperature manager (wsol_loader.py:240-244, decay_temp.py)
    tmp = DecayTemp(args.sl_tc_knn_t, args.sl_tc_min_t, args.sl_tc_knn, args.sl_tc_knn_mode,
                    args.sl_tc_knn_epoch_switch_uniform, args.sl_tc_seed_tech)
    seeder = TCAMSeeder(seed_tech=args.sl_tc_seed_tech, min_=args.sl_tc_min,
                        max_=args.sl_tc_max, max_p=args.sl_tc_max_p, min_p=args.sl_tc_min_p,
                        fg_erode_k=args.sl_tc_fg_erode_k, fg_erode_iter=args.sl_tc_fg_erode_iter,
                        ksz=args.sl_tc_ksz, support_background=True, multi_label_flag=False,
                        seg_ignore_idx=-255, cuda_id=dev.index, roi_method=args.sl_tc_roi_method,
                        p_min_area_roi=args.sl_tc_roi_min_size, use_roi=args.sl_tc_use_roi,
                        seed=args.seed + rank)
    tr = DecoderTrainer(model, lr=args.opt__lr, momentum=args.opt__momentum,
                        dampening=args.opt__dampening, weight_decay=args.opt__weight_decay,
                        nesterov=args.opt__nesterov, sl_lambda=args.sl_tc_lambda,
                        crf_lambda=args.crf_tc_lambda, size_lambda=args.max_sizepos_tc_lambda,
                        crf_sigma_rgb=args.crf_tc_sigma_rgb, crf_sigma_xy=args.crf_tc_sigma_xy,
                        crf_scale=args.crf_tc_scale, elb=ELB(args.elb_init_t, args.elb_max_t, args.elb_mulcoef),
                        use_sl=args.sl_tc, use_crf=args.crf_tc, use_size=args.max_sizepos_tc,
                        seeder=seeder, amp=args.amp, use_rgb=args.rgb_jcrf_tc,
                        rgb_lambda=args.rgb_jcrf_tc_lambda,
                        rgb_sigma_rgb=args.rgb_jcrf_tc_sigma_rgb,
                        rgb_scale=args.rgb_jcrf_tc_scale,
                        windows={"sl": (args.sl_tc_start_ep, args.sl_tc_end_ep),
                                 "crf": (args.crf_tc_start_ep, args.crf_tc_end_ep),
                                 "size": (args.max_sizepos_tc_start_ep,
                                          args.max_sizepos_tc_end_ep),
                                 "rgb": (args.rgb_jcrf_tc_start_ep, args.rgb_jcrf_tc_end_ep)})
    sched = (lr_schedule(tr, args.opt__step_size, args.opt__gamma, args.opt__min_lr)
             if args.opt__lr_scheduler else None)
    save_dir = os.path.join(args.exp_path, "checkpoints")
    # the two best models of model_selection (train_wsol.py:1735-1756): localization and
    # classification (constants.BEST_LOC / BEST_CL)
    best_dirs = {"best_loc": os.path.join(args.exp_path, "best_loc"),
                 "best_cl": os.path.join(args.exp_path, "best_cl")}
    step = CK.load_checkpoint(tr, save_dir, lr_scheduler=sched)
    data = _splits(args, ["train", "val"])
    train, val = data["train"], data["val"]
    roi_fn = GetRoiSingleCam(args.sl_tc_roi_method, args.sl_tc_roi_min_size)
    roi_th = load_roi_thresholds(args.std_cams_thresh_file) if args.std_cams_thresh_file \
        else None
    tf = FR.get_train_transforms(RESIZE_SIZE, args.crop_size)
    # main.py:78-81: the resumed epoch is floor(step / ceil(len / (batch * gpus))) — the
    # reference's own count (a resumed run replays that epoch, as the reference does); the
    # dataset length counts shots and the batch is the knn-rescaled one in DS_SHOTS mode
    if train.shot_ids is not None:
        per = args.batch_size // (2 * args.knn_tc + 1) if args.knn_tc > 0 else args.batch_size
        per_epoch = math.ceil(len(train.shot_ids) / (max(per, 1) * world))
    else:
        per_epoch = math.ceil(len(train) / (args.batch_size * world))
    current_epoch = step // per_epoch
    log = []
    health: Dict[str, bool] = {}     # checkpoints_health, kept for the whole run
    # Trainer.evaluate (train_wsol.py:1473-1480): the validation split of CUB / ILSVRC /
    # YTOv1 / YTOv2.2 sweeps the fast tau grid (VALID_FAST_CAM_CURVE_INTERVAL, 250 tau)
    valid_interval = VALID_FAST_CAM_CURVE_INTERVAL if args.dataset in FAST_VALID_DATASETS \
        else args.cam_curve_interval

    # PerformanceMeter (train_wsol.py:76-96) of the validation split: the values of every
    # evaluation; best_epoch = the FIRST index of the maximum
    meters: Dict[str, List[float]] = {"best_loc": [], "best_cl": []}
    if step:   # resume: the model-selection meters too (train_wsol.py:1299-1316)
        meters.update(CK.load_tracker(save_dir))
    best_at: Dict[str, int] = {}

    def validate(epoch: int, at_step: int) -> dict:
        model.eval()
        prev = model.conv_precision
        if args.amp_eval:    # autocast(enabled=amp_eval) covers the evaluation only
            model.conv_precision = "amp"
        try:
            res = evaluate(model, val, args, dev, cam_curve_interval=valid_interval)
        finally:
            model.conv_precision = prev
        # LOCALIZATION_MTR: the mean BoxAcc over the IoU thresholds under box_v2_metric
        # (multi_iou_eval), else BoxAcc@50 (train_wsol.py:1515-1519);
        # CLASSIFICATION_MTR: _compute_accuracy (train_wsol.py:1400-1435, 1468-1471)
        for key, v in (("best_loc", res["localization"]), ("best_cl", res["classification_acc"])):
            meters[key].append(v)
            best_at[key] = meters[key].index(max(meters[key]))
            # model_selection (train_wsol.py:1735-1756): this evaluation is the best one
            if rank == 0 and best_at[key] == len(meters[key]) - 1:
                CK.save_best_model(model, TCAM, best_dirs[key], at_step)
        if rank == 0 and at_step:
            CK.save_tracker(save_dir, at_step, meters)
            CK.keep_last_n_checkpoints(save_dir, args.keep_last_n_checkpoints, key=CK.CHP_TR)
        return res

    # main.py:83-88: evaluate (and select) before the first epoch
    res = validate(current_epoch, step)
    if rank == 0:
        print(json.dumps({"epoch": current_epoch, "step": step, "val": res}), flush=True)
    for epoch in range(current_epoch, args.max_epochs):
        zepoch = epoch + 1      # main.py:97: Trainer.train(epoch=epoch + 1)
        # on_epoch_start (train_wsol.py:944-965)
        tmp.set_epoch(zepoch)
        seeder.set_seed_tech(tmp.sl_tc_seed_tech)
        tr.set_epoch(zepoch)    # the loss terms' epoch windows (losses/core.py:64-82)
        torch.manual_seed(args.seed + zepoch)
        frame_rng = np.random.default_rng([args.seed, zepoch, rank])
        t0, losses = time.perf_counter(), None
        def epoch_batches():
            # one batch ahead: batch i+1 is built (same order, same RNG draws) before step i
            # runs, so its frozen-encoder forward overlaps step i's backward (next_images)
            for ids, seq, frm in train_batches(train, args, rank, world, zepoch, frame_rng):
                crops, flips = tf.draw(len(ids))
                x, raw = device_frames(train, ids, dev, tf, crops=crops, flips=flips)
                std, roi = None, None
                if args.sl_tc and train.std_cam_fn is not None:
                    # Resize(256) -> the same crop / flip as the frames (wsol_loader.py:603)
                    std = prepare_std_cams(_std_cams_batch(train, ids, args, dev, tmp.sl_tc_knn_t),
                                           (RESIZE_SIZE, RESIZE_SIZE))
                    s = args.crop_size
                    std = torch.stack([std[b, :, int(c[0]):int(c[0]) + s, int(c[1]):int(c[1]) + s]
                                       for b, c in enumerate(crops.tolist())])
                    fl = flips.to(dev)
                    std = torch.where(fl[:, None, None, None], std.flip(-1), std).contiguous()
                    if args.sl_tc_use_roi:
                        # wsol_loader.py:571-579, 608-613: CAM-TMP re-thresholds (Otsu); a
                        # single-frame CAM uses the stored per-frame threshold when there is one
                        th = None
                        if tmp.sl_tc_knn == 0 and roi_th is not None:
                            th = [roi_th.get(i, float("nan")) for i in ids]
                        roi = roi_fn.batch(std[:, 0], thresh=th)[0][:, None]
                # _fill_minibatch (train_wsol.py:1126-1153): a short last batch is repeated
                x, raw = fill_minibatch(x, args.batch_size), fill_minibatch(raw, args.batch_size)
                std, roi = fill_minibatch(std, args.batch_size), fill_minibatch(roi, args.batch_size)
                if seq is not None:   # _fill_minibatch on seq_iter / frm_iter (:1132-1133)
                    seq = fill_minibatch(torch.tensor(seq), args.batch_size)
                    frm = fill_minibatch(torch.tensor(frm), args.batch_size)
                yield x, raw, std, roi, seq, frm

        batches = epoch_batches()
        cur = next(batches, None)
        while cur is not None:
            nxt = next(batches, None)
            x, raw, std, roi, seq, frm = cur
            losses = tr.step(x, raw, std_cams=std, roi=roi, seq_iter=seq, frm_iter=frm,
                             next_images=nxt[0] if nxt is not None else None,
                             next_raw=nxt[1] if nxt is not None else None)
            cur = nxt
            step += 1
            if step % args.checkpoint_save == 0:
                # never checkpoint weights an overflowed gradient reached; the check is a
                # collective (every rank raises together or none does), so every rank runs it
                tr.check_overflow()
                if rank == 0:
                    CK.save_checkpoint(tr, save_dir, step, lr_scheduler=sched)
                    CK.keep_last_n_checkpoints(save_dir, args.keep_last_n_checkpoints,
                                               health=health)
        tr.close()             # the unused next-batch lattice / features of the last step
        tr.elb.update_t()      # on_epoch_end (train_wsol.py:967-976)
        tr.check_overflow()
        res = validate(zepoch, step)
        if sched is not None:
            sched.step()       # adjust_learning_rate (main.py:114)
        if rank == 0:
            log.append({"epoch": zepoch, "step": step, "tmp_manager": tmp.get_current_status(),
                        "lr": tr.lr, "skipped_steps": tr.skipped_steps,
                        "losses": [float(v) for v in losses.cpu()] if losses is not None else None,
                        "val": res, "epoch_s": round(time.perf_counter() - t0, 2)})
            print(json.dumps(log[-1]), flush=True)
    tr.check_overflow()        # all ranks (a collective)
    if rank == 0:
        CK.save_checkpoint(tr, save_dir, step, lr_scheduler=sched)
    if args.final_test_eval:
        final_test_eval(model, args, dev, best_dirs, rank)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def final_test_eval(model, args, dev, best_dirs: Dict[str, str], rank: int) -> None:
    """main.py:117-160: the test split evaluated with each best model — best_loc, then
    best_cl (best_loc only for ILSVRC) — at --cam_curve_interval."""
    if not args.synthetic and not (args.metadata_root and
                                   os.path.isdir(os.path.join(args.metadata_root, "test"))):
        return      # no test split in this layout
    if dist.is_initialized():
        dist.barrier()          # rank 0 wrote the best models
    test = _splits(args, ["test"])["test"]
    chpts = ["best_loc"] if args.dataset == "ILSVRC" else ["best_loc", "best_cl"]
    out = {}
    for key in chpts:
        step = CK.load_best_model(model, args.task, best_dirs[key])
        model.eval()
        prev = model.conv_precision
        if args.amp_eval:
            model.conv_precision = "amp"
        try:
            out[key] = dict(evaluate(model, test, args, dev), checkpoint_step=step)
        finally:
            model.conv_precision = prev
    if rank == 0:
        print(json.dumps({"final_test": out}), flush=True)


def train_stdcl_main(args) -> int:
    """main.py:33-167 + Trainer.train (train_wsol.py:944-1233) for task STD_CL — stage 1,
    the README.md:239-266 run: the ResNet50 STDClassifier (encoder + WGAP) trained end to
    end with ClLoss (``--freeze_cl False --freeze_encoder False``, ``--amp True`` for
    autocast), validated with the STD_CL CAM (inference_wsol.py, model selection best_loc /
    best_cl), checkpointed as the reference does; its best_loc / best_cl folders are what
    TCAM's ``--pretrained_classifier`` loads (README.md:267-276)."""
    from .cl_training import ClassifierTrainer, lr_schedule as lr_schedule_cl
    from .training import fill_minibatch
    if args.freeze_cl:
        raise SystemExit("STD_CL trains the classifier: --freeze_cl False (parseit.py:873-875)")
    if args.freeze_encoder:
        raise SystemExit("--freeze_encoder True is a C_BOX switch (config.py:236-238); stage 1 "
                         "trains the encoder")
    if args.encoder_name != "resnet50":
        raise SystemExit("stage-1 training runs the ResNet50 encoder (README.md:239-266)")
    dev = _init_dist(args)
    rank, world = rank_world()
    model = create_model(**_model_kwargs(args))
    from .utils.seeding import seed_module_
    seed_module_(model, args.seed)
    model = model.to(dev)
    tr = ClassifierTrainer(model, lr=args.opt__lr, momentum=args.opt__momentum,
                           dampening=args.opt__dampening, weight_decay=args.opt__weight_decay,
                           nesterov=args.opt__nesterov,
                           lr_classifier_ratio=args.opt__lr_classifier_ratio, amp=args.amp)
    sched = (lr_schedule_cl(tr, args.opt__step_size, args.opt__gamma, args.opt__min_lr)
             if args.opt__lr_scheduler else None)
    save_dir = os.path.join(args.exp_path, "checkpoints")
    best_dirs = {"best_loc": os.path.join(args.exp_path, "best_loc"),
                 "best_cl": os.path.join(args.exp_path, "best_cl")}
    step = CK.load_checkpoint(tr, save_dir, lr_scheduler=sched)
    data = _splits(args, ["train", "val"])
    train, val = data["train"], data["val"]
    tf = FR.get_train_transforms(RESIZE_SIZE, args.crop_size)
    per_epoch = math.ceil(len(train) / (args.batch_size * world))
    current_epoch = step // per_epoch
    log = []
    health: Dict[str, bool] = {}
    valid_interval = VALID_FAST_CAM_CURVE_INTERVAL if args.dataset in FAST_VALID_DATASETS \
        else args.cam_curve_interval
    meters: Dict[str, List[float]] = {"best_loc": [], "best_cl": []}
    if step:   # resume: the model-selection meters too (train_wsol.py:1299-1316)
        meters.update(CK.load_tracker(save_dir))

    def validate(at_step: int) -> dict:
        model.eval()
        prev = model.conv_precision
        if args.amp_eval:
            model.conv_precision = "amp"
        try:
            res = evaluate(model, val, args, dev, cam_curve_interval=valid_interval)
        finally:
            model.conv_precision = prev
        for key, v in (("best_loc", res["localization"]), ("best_cl", res["classification_acc"])):
            meters[key].append(v)
            if rank == 0 and meters[key].index(max(meters[key])) == len(meters[key]) - 1:
                CK.save_best_model(model, STD_CL, best_dirs[key], at_step)
        if rank == 0 and at_step:
            CK.save_tracker(save_dir, at_step, meters)
            CK.keep_last_n_checkpoints(save_dir, args.keep_last_n_checkpoints, key=CK.CHP_TR)
        return res

    res = validate(step)
    if rank == 0:
        print(json.dumps({"epoch": current_epoch, "step": step, "val": res}), flush=True)
    for epoch in range(current_epoch, args.max_epochs):
        zepoch = epoch + 1
        torch.manual_seed(args.seed + zepoch)
        frame_rng = np.random.default_rng([args.seed, zepoch, rank])
        t0, loss, nframes = time.perf_counter(), None, 0
        for ids, _, _ in train_batches(train, args, rank, world, zepoch, frame_rng):
            crops, flips = tf.draw(len(ids))
            x, _ = device_frames(train, ids, dev, tf, crops=crops, flips=flips)
            y = torch.tensor([train.labels[i] for i in ids], device=dev, dtype=torch.int32)
            # _fill_minibatch (train_wsol.py:1126-1153): a short last batch is repeated
            x, y = fill_minibatch(x, args.batch_size), fill_minibatch(y, args.batch_size)
            loss = tr.step(x, y)
            nframes += x.shape[0]
            step += 1
            if step % args.checkpoint_save == 0:
                tr.check_overflow()
                if rank == 0:
                    CK.save_checkpoint(tr, save_dir, step, lr_scheduler=sched)
                    CK.keep_last_n_checkpoints(save_dir, args.keep_last_n_checkpoints,
                                               health=health)
        tr.check_overflow()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = validate(step)
        if sched is not None:
            sched.step()
        if rank == 0:
            log.append({"epoch": zepoch, "step": step, "lr": list(tr.lrs),
                        "skipped_steps": tr.skipped_steps,
                        "loss": float(loss) if loss is not None else None,
                        "train_frames_per_s_rank0": round(nframes / dt, 1), "val": res,
                        "epoch_s": round(dt, 2)})
            print(json.dumps(log[-1]), flush=True)
    tr.check_overflow()
    if rank == 0:
        CK.save_checkpoint(tr, save_dir, step, lr_scheduler=sched)
    if args.final_test_eval:
        final_test_eval(model, args, dev, best_dirs, rank)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0
