"""Test helper: numpy emulation of the GPU bbox algorithm (csrc/bbox.hip).

Used on CPU to pin the characterisation that the HIP kernels implement
(psi hole-fill + 8-connected components of {psi > L} + window areas +
OpenCV list-order tie-break) against the faithful border-follower oracle
(oracle/contours.c) on many random images.
"""
import numpy as np
from scipy import ndimage


def psi_fill(u8: np.ndarray) -> np.ndarray:
    """min over 4-paths from outside of the max along the path (grayscale fill)."""
    H, W = u8.shape
    img = u8.astype(np.int32)
    pad = np.full((H + 2, W + 2), -1, np.int32)
    psi = np.full((H + 2, W + 2), 255, np.int32)
    psi[0, :] = psi[-1, :] = -1
    psi[:, 0] = psi[:, -1] = -1
    while True:
        nb = np.minimum.reduce([psi[:-2, 1:-1], psi[2:, 1:-1], psi[1:-1, :-2], psi[1:-1, 2:]])
        new = np.maximum(img, np.minimum(psi[1:-1, 1:-1], nb))
        if np.array_equal(new, psi[1:-1, 1:-1]):
            break
        psi[1:-1, 1:-1] = new
    return psi[1:-1, 1:-1]


def box_for_level(psi: np.ndarray, L: int) -> np.ndarray:
    H, W = psi.shape
    F = psi > L
    if not F.any():
        return np.zeros(4, np.int64)
    lab, n = ndimage.label(F, structure=np.ones((3, 3)))
    Fp = np.zeros((H + 2, W + 2), bool)
    Fp[1:-1, 1:-1] = F
    labp = np.zeros((H + 2, W + 2), np.int64)
    labp[1:-1, 1:-1] = lab
    c = (Fp[:-1, :-1].astype(int) + Fp[:-1, 1:] + Fp[1:, :-1] + Fp[1:, 1:])
    wl = np.maximum.reduce([labp[:-1, :-1], labp[:-1, 1:], labp[1:, :-1], labp[1:, 1:]])
    contrib = np.where(c >= 3, c - 2, 0)
    area = np.bincount(wl.ravel(), weights=contrib.ravel(), minlength=n + 1)[1:]
    first = ndimage.minimum(np.arange(H * W).reshape(H, W), lab, index=np.arange(1, n + 1))
    best = area.max()
    cand = np.where(area == best)[0]
    k = cand[np.argmax(np.asarray(first)[cand])] + 1
    ys, xs = np.nonzero(lab == k)
    return np.array([xs.min(), ys.min(), min(xs.max() + 1, W - 1), min(ys.max() + 1, H - 1)])


def boxes_for_levels(u8: np.ndarray, levels) -> np.ndarray:
    psi = psi_fill(u8)
    return np.stack([box_for_level(psi, int(L)) for L in levels])
