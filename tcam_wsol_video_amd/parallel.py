"""Multi-GPU plumbing of the hot path: one process per GPU, torch.distributed over
RCCL (backend "nccl") — or gloo, the reference's default ``dist_backend``
(configure/config.py:489).

* :func:`sync_tensor_across_gpus` — dlib/parallel/__init__.py:14-23 (all_gather along
  dim 0, then cat).  Device tensors on RCCL take ONE ``all_gather_into_tensor`` into a
  preallocated buffer; gloo has no device all-gather, so device tensors are staged
  through host memory there.
* :func:`distributed_sampler_indices` — the frame order each rank sees under the
  reference's ``DistributedSampler`` (datasets/wsol_loader.py:1008-1012): interleaved,
  padded with the first frames so every rank gets ceil(N / world) of them.  The padded
  duplicates are evaluated and counted, as in the reference (SURVEY.md §7 v).
* :func:`knn_window` — the neighbour frames of CAM-TMP (wsol_loader.py:447-458,
  544-569): ``sl_tc_knn`` frames before and/or after, clipped at the shot boundary.
* :class:`TemporalCAM` — the temporal CAM of a clip sharded over the ranks (BASELINE
  configs[4]): every rank all-gathers the per-frame CAMs of the clip, then takes the
  max over each of its own frames' windows (wsol_loader.py:591-601, with
  ``re_normalize_cam`` when sl_tc_knn > 0 and t > 0, :571, 594, 630-635) and quantises to uint8 in one kernel
  (``tcam_temporal_cam``).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import ops

# configure/constants.py:335-338
TIME_INSTANT = "instant"
TIME_BEFORE = "before"
TIME_AFTER = "after"
TIME_BEFORE_AFTER = "before-after"
TIME_DEPENDENCY = (TIME_BEFORE, TIME_AFTER, TIME_BEFORE_AFTER, TIME_INSTANT)


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank_world(group=None) -> Tuple[int, int]:
    if not is_distributed():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def sync_tensor_across_gpus(t: Optional[torch.Tensor], group=None) -> Optional[torch.Tensor]:
    """dlib/parallel/__init__.py:14-23: the tensors of all ranks concatenated along
    dim 0 in rank order (every rank must pass the same shape)."""
    if t is None:
        return None
    if not is_distributed():
        return t
    world = dist.get_world_size(group)
    t = t.contiguous()
    if t.is_cuda and dist.get_backend(group) == "nccl":
        # RCCL at any world size (world 1 is a device copy: the same launch path)
        out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out
    if world == 1:
        return t
    host = t.detach().cpu() if t.is_cuda else t
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    out = torch.cat(parts, dim=0)
    return out.to(t.device, non_blocking=False) if t.is_cuda else out


def distributed_sampler_indices(n: int, rank: int, world: int, shuffle: bool = False,
                                seed: int = 0, epoch: int = 0,
                                drop_last: bool = False) -> List[int]:
    """torch.utils.data.DistributedSampler.__iter__ (the reference's eval loaders use
    shuffle=False, wsol_loader.py:1008-1012)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    if drop_last and n % world != 0:
        num_samples = math.ceil((n - world) / world)
    else:
        num_samples = math.ceil(n / world)
    total = num_samples * world
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g).tolist()
    else:
        indices = list(range(n))
    if not drop_last:
        pad = total - len(indices)
        if pad <= len(indices):
            indices += indices[:pad]
        else:
            indices += (indices * math.ceil(pad / len(indices)))[:pad]
    else:
        indices = indices[:total]
    assert len(indices) == total
    return indices[rank:total:world]


def knn_window(n_frames: int, k: int, mode: str) -> np.ndarray:
    """(n_frames, k1) int32: for frame i of one shot, the frames whose CAMs
    CAM-TMP takes the max over — left knn + [i] + right knn (wsol_loader.py:
    447-458, 544-569), -1 where a window is shorter than k1.  Note the reference's
    right window of the LAST frame is [last] itself (`lframes[min(idx+1, n-1):
    min(idx+k+1, n)]`); that duplicate is kept (max is idempotent)."""
    if mode not in TIME_DEPENDENCY:
        raise ValueError(f"mode {mode!r} not in {TIME_DEPENDENCY}")
    if mode == TIME_INSTANT and k != 0:
        raise ValueError("sl_tc_knn_mode 'instant' requires sl_tc_knn == 0")
    if k < 0:
        raise ValueError("sl_tc_knn must be >= 0")
    before = mode in (TIME_BEFORE, TIME_BEFORE_AFTER)
    after = mode in (TIME_AFTER, TIME_BEFORE_AFTER)
    # the right window of the last frame is [last] even for k = 0
    k1 = 1 + k * int(before) + max(k, 1) * int(after)
    out = np.full((n_frames, k1), -1, dtype=np.int32)
    for i in range(n_frames):
        win = []
        if before:
            win += list(range(max(0, i - k), i))
        win.append(i)
        if after:
            win += list(range(min(i + 1, n_frames - 1), min(i + k + 1, n_frames)))
        out[i, :len(win)] = win
    return out


class TemporalCAM:
    """CAM-TMP over a clip whose frames are sharded contiguously over the ranks of
    ``group`` (rank r holds frames [r*B, (r+1)*B) of the clip).

    ``k`` = ``sl_tc_knn``, ``mode`` = ``sl_tc_knn_mode``, ``t`` = ``sl_tc_knn_t``
    (README.md:312-314 runs k=1, 'before', t=0)."""

    def __init__(self, k: int = 1, mode: str = TIME_BEFORE, t: float = 0.0, group=None):
        knn_window(1, k, mode)    # validates
        self.k, self.mode, self.t, self.group = int(k), mode, float(t), group
        self._idx = {}

    def window(self, clip_len: int, rank: int, per_rank: int, device=None) -> torch.Tensor:
        """This rank's rows of :func:`knn_window` (indices into the gathered clip)."""
        key = (clip_len, rank, per_rank, str(device))
        idx = self._idx.get(key)
        if idx is None:
            w = knn_window(clip_len, self.k, self.mode)[rank * per_rank:(rank + 1) * per_rank]
            idx = torch.from_numpy(np.ascontiguousarray(w))
            if device is not None:
                idx = idx.to(device)
            self._idx[key] = idx
        return idx

    def __call__(self, cam_local: torch.Tensor, want_cam: bool = True, want_u8: bool = True):
        """cam_local (B, H, W) fp32 on the device -> (temporal CAM (B, H, W) fp32,
        uint8) for this rank's frames."""
        rank, world = rank_world(self.group)
        full = sync_tensor_across_gpus(cam_local, self.group)
        B = cam_local.shape[0]
        idx = self.window(world * B, rank, B, cam_local.device)
        # heated only when sl_tc_knn > 0 (wsol_loader.py:571, 594)
        t = self.t if self.k > 0 else 0.0
        return ops.temporal_cam(full, idx, t, want_cam=want_cam, want_u8=want_u8)
