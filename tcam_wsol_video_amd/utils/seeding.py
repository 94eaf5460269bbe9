"""Deterministic, checkpoint-free weights for the TCAM models.

There is no network in this environment, so neither ImageNet nor the stage-1
TCAM checkpoints (instantiators.py:579-616) can be loaded.  Instead every
tensor of a model's ``state_dict`` is filled, in ``state_dict`` order, from a
single numpy ``PCG64(seed)`` stream.  Because the product modules keep the
reference's parameter names, the same call on a reference
``UnetTCAM`` and on ours yields bit-identical weights; the golden-vector
generator (tests/golden/make_golden.py) relies on this.

BatchNorm running statistics and affine parameters are randomised as well
(with default init eval-mode BN is ~identity and would not
exercise the BN fold).  The last BN of every residual branch (``bn3``) gets a
small gain so that 16 stacked bottlenecks keep activations O(1).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def _fill(name: str, shape, rng: np.random.Generator) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        return rng.uniform(-0.1, 0.1, n).reshape(shape)
    if leaf == "running_var":
        return rng.uniform(0.8, 1.2, n).reshape(shape)
    if leaf == "bias":
        return rng.uniform(-0.05, 0.05, n).reshape(shape)
    if leaf == "weight":
        if len(shape) == 1:  # BatchNorm gamma
            if name.endswith("bn3.weight"):
                return rng.uniform(0.1, 0.3, n).reshape(shape)
            return rng.uniform(0.8, 1.2, n).reshape(shape)
        fan_in = int(np.prod(shape[1:]))
        if len(shape) == 4:  # conv: He-normal
            std = np.sqrt(2.0 / fan_in)
        else:  # linear
            std = np.sqrt(1.0 / fan_in)
        return (rng.standard_normal(n) * std).reshape(shape)
    raise KeyError(f"no seeding rule for state_dict entry {name!r}")


def seeded_state_dict(module: torch.nn.Module, seed: int) -> Dict[str, torch.Tensor]:
    """Return a state_dict for ``module`` drawn from ``PCG64(seed)``."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, t in module.state_dict().items():
        arr = _fill(name, tuple(t.shape), rng)
        out[name] = torch.from_numpy(np.ascontiguousarray(arr)).to(t.dtype)
    return out


def seed_module_(module: torch.nn.Module, seed: int) -> torch.nn.Module:
    """Load :func:`seeded_state_dict` into ``module`` (strict)."""
    module.load_state_dict(seeded_state_dict(module, seed), strict=True)
    return module


def synthetic_clip(n_frames: int, seed: int = 0, height: int = 360,
                   width: int = 480) -> np.ndarray:
    """Synthetic YTOv2.2-shaped clip: ``(T, H, W, 3)`` uint8.

    Each frame is a sum of 3-6 Gaussian blobs plus low noise; blobs drift by
    1-2 px per frame for temporal coherence.  Deterministic in ``seed``.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    nb = int(rng.integers(3, 7))
    cy = rng.uniform(0.2 * height, 0.8 * height, nb)
    cx = rng.uniform(0.2 * width, 0.8 * width, nb)
    sy = rng.uniform(0.05 * height, 0.2 * height, nb)
    sx = rng.uniform(0.05 * width, 0.2 * width, nb)
    col = rng.uniform(40, 255, (nb, 3))
    vy = rng.uniform(-2, 2, nb)
    vx = rng.uniform(-2, 2, nb)
    yy = np.arange(height, dtype=np.float64)[:, None]
    xx = np.arange(width, dtype=np.float64)[None, :]
    frames = np.empty((n_frames, height, width, 3), dtype=np.uint8)
    for t in range(n_frames):
        img = np.full((height, width, 3), 20.0)
        for b in range(nb):
            g = np.exp(-0.5 * (((yy - cy[b] - vy[b] * t) / sy[b]) ** 2
                               + ((xx - cx[b] - vx[b] * t) / sx[b]) ** 2))
            img += g[..., None] * col[b][None, None, :]
        img += rng.normal(0.0, 4.0, img.shape)
        frames[t] = np.clip(img, 0, 255).astype(np.uint8)
    return frames


def synthetic_boxes(frames: np.ndarray, size: int = 224) -> np.ndarray:
    """One GT box per frame from the bright-blob extent, (T, 4) x0y0x1y1 at ``size``.

    Mirrors the YTOv1 ``localization.txt`` convention resized with
    ``resize_bbox`` (utils/tools.py:231-250): ``int()`` truncation.
    """
    t, h, w, _ = frames.shape
    out = np.zeros((t, 4), dtype=np.int64)
    for i in range(t):
        g = frames[i].astype(np.float64).mean(-1)
        m = g > (g.min() + 0.5 * (g.max() - g.min()))
        ys, xs = np.nonzero(m)
        if len(xs) == 0:
            x0, y0, x1, y1 = 0, 0, w - 1, h - 1
        else:
            x0, y0, x1, y1 = xs.min(), ys.min(), xs.max(), ys.max()
        out[i] = [int(float(x0) * size / w), int(float(y0) * size / h),
                  int(float(x1) * size / w), int(float(y1) * size / h)]
    return out
