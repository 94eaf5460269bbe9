"""Frame preprocessing on the device: the reference's eval / train transforms for a batch of
decoded uint8 RGB frames.

Mirrors datasets/wsol_loader.py:903-908 ``get_eval_tranforms(crop_size)`` (Resize((s, s)),
ToTensor, Normalize(_IMAGE_MEAN_VALUE, _IMAGE_STD_VALUE)) and the train Compose of
:960-970 (Resize((r, r)) -> RandomCrop(s) -> RandomHorizontalFlip -> ToTensor ->
Normalize).  Each call returns ``(image, raw_img)`` like the reference's Compose: the
normalised (B, 3, s, s) fp32 batch and raw_img = the resized frame as float32 (B, 3, s, s)
(wsol_loader.py:603-606), both bit-identical to Pillow's BILINEAR resize + torchvision's
ToTensor / Normalize (see csrc/frames.hip).  JPEG decoding stays with the caller (PIL).
No CPU fallback: CPU tensors are refused.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import check

IMAGE_MEAN_VALUE = [0.485, 0.456, 0.406]   # wsol_loader.py:46
IMAGE_STD_VALUE = [0.229, 0.224, 0.225]    # wsol_loader.py:47

_COEFFS: Dict[Tuple[int, int, torch.device], Tuple[torch.Tensor, torch.Tensor, int]] = {}


def resample_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray]:
    """Pillow's BILINEAR resample coefficients (host C++, tcam_resample_coeffs):
    bounds (out, 2) int32 [first tap, taps], weights (out, ksize) int32 (22 fraction bits)."""
    lib = _lib.load()
    ks = int(lib.tcam_resample_coeffs(in_size, out_size, None, None))
    check(ks if ks < 0 else 0, "tcam_resample_coeffs")
    b = np.zeros((out_size, 2), np.int32)
    k = np.zeros((out_size, ks), np.int32)
    check(min(0, int(lib.tcam_resample_coeffs(in_size, out_size,
                                               b.ctypes.data_as(C.c_void_p),
                                               k.ctypes.data_as(C.c_void_p)))),
          "tcam_resample_coeffs")
    return b, k


def _device_coeffs(in_size: int, out_size: int, dev: torch.device):
    key = (in_size, out_size, dev)
    if key not in _COEFFS:
        b, k = resample_coeffs(in_size, out_size)
        _COEFFS[key] = (torch.from_numpy(b).to(dev), torch.from_numpy(k).to(dev), k.shape[1])
    return _COEFFS[key]


def preprocess(frames: torch.Tensor, resize: Tuple[int, int], crop_size: Tuple[int, int],
               crops: Optional[torch.Tensor] = None, flips: Optional[torch.Tensor] = None,
               want_norm: bool = True, want_raw: bool = True):
    """frames (B, H, W, 3) uint8 on the device -> (norm, raw), each (B, 3, th, tw) fp32 or
    None: Resize(resize) -> crop at crops[b] = (top, left) (default (0, 0)) -> hflip where
    flips[b] -> ToTensor -> Normalize."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.dim() != 4 or \
            frames.shape[3] != 3:
        raise ValueError("frames must be a (B, H, W, 3) uint8 device tensor")
    frames = frames.contiguous()
    B, H, W, _ = frames.shape
    rh, rw = resize
    th, tw = crop_size
    if th > rh or tw > rw:
        raise ValueError(f"crop {crop_size} larger than the resized frame {resize}")
    dev = frames.device
    bh, kh, ksh = _device_coeffs(W, rw, dev)
    bv, kv, ksv = _device_coeffs(H, rh, dev)
    if crops is not None:
        crops = crops.to(dev, torch.int32).contiguous()
        if crops.shape != (B, 2) or bool(((crops < 0) | (crops[:, 0] > rh - th)[:, None] |
                                          (crops[:, 1] > rw - tw)[:, None]).any()):
            raise ValueError("crops must be (B, 2) (top, left) inside the resized frame")
    if flips is not None:
        flips = flips.to(dev, torch.uint8).contiguous()
        if flips.shape != (B,):
            raise ValueError("flips must be (B,)")
    norm = torch.empty(B, 3, th, tw, device=dev) if want_norm else None
    raw = torch.empty(B, 3, th, tw, device=dev) if want_raw else None
    mean = (C.c_float * 3)(*IMAGE_MEAN_VALUE)
    std = (C.c_float * 3)(*IMAGE_STD_VALUE)
    lib = _lib.load()
    check(lib.tcam_frames_preprocess(
        frames.data_ptr(), B, H, W, bh.data_ptr(), kh.data_ptr(), ksh, rw, bv.data_ptr(),
        kv.data_ptr(), ksv, rh, crops.data_ptr() if crops is not None else None,
        flips.data_ptr() if flips is not None else None, th, tw, mean, std,
        norm.data_ptr() if norm is not None else None,
        raw.data_ptr() if raw is not None else None, None,
        torch.cuda.current_stream(dev).cuda_stream), "tcam_frames_preprocess")
    return norm, raw


class EvalTransform:
    """get_eval_tranforms(crop_size) on a device batch: __call__(frames) -> (image, raw_img)."""

    def __init__(self, crop_size: int):
        self.crop_size = crop_size

    def __call__(self, frames: torch.Tensor):
        s = self.crop_size
        return preprocess(frames, (s, s), (s, s))

    def __repr__(self):
        return f"EvalTransform(Resize(({self.crop_size}, {self.crop_size})), ToTensor, Normalize)"


class TrainTransform:
    """The train Compose (Resize((r, r)) -> RandomCrop(s) -> RandomHorizontalFlip(p=.5) ->
    ToTensor -> Normalize) with per-frame crop offsets / flips drawn from torch's RNG like
    RandomCrop.get_params / RandomHorizontalFlip (torch.randint, torch.rand)."""

    def __init__(self, resize_size: int, crop_size: int, p: float = 0.5):
        self.resize_size, self.crop_size, self.p = resize_size, crop_size, p

    def draw(self, B: int):
        r, s = self.resize_size, self.crop_size
        crops = torch.stack([torch.randint(0, r - s + 1, (B,)),
                             torch.randint(0, r - s + 1, (B,))], 1)
        flips = torch.rand(B) < self.p
        return crops, flips

    def __call__(self, frames: torch.Tensor, crops=None, flips=None):
        if crops is None or flips is None:
            c, f = self.draw(frames.shape[0])
            crops = c if crops is None else crops
            flips = f if flips is None else flips
        r, s = self.resize_size, self.crop_size
        return preprocess(frames, (r, r), (s, s), crops=crops, flips=flips)


def get_eval_tranforms(crop_size: int) -> EvalTransform:   # reference spelling
    return EvalTransform(crop_size)


def get_train_transforms(resize_size: int, crop_size: int) -> TrainTransform:
    return TrainTransform(resize_size, crop_size)
