"""TEST INFRASTRUCTURE ONLY — CPU oracles of the CRF bilateral filters.

Two independent checkers of ``tcam_bilateral_batch`` / ``tcam_colorbilateral_batch``:

* ``ref_bilateral`` / ``ref_colorbilateral`` call the REFERENCE filters compiled from
  their own sources (``oracle/Makefile`` -> ``oracle/_ref/lib*bilateral_ref.so``; g++
  -O2 -fopenmp, x86-64 => the SSE branch of permutohedral.cpp) through ctypes.
* ``port_bilateral`` restates the same algorithm in numpy fp32
  (crf/crfwrapper/bilateralfilter/permutohedral.cpp:105-571, SSE branch;
  bilateralfilter.cpp:4-55; colorbilateralfilter.cpp:4-54).  numpy fp32 ops are
  IEEE single with no fusion, and ``np.add.at`` accumulates in index order, so the
  port reproduces the reference bit for bit (checked by tests/test_crf_oracle.py).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REF = {"xy": ("libbilateral_ref.so", "_Z21bilateralfilter_batchPfiS_iS_iiiiiff"),
        "color": ("libcolorbilateral_ref.so", "_Z26colorbilateralfilter_batchPfiS_iS_iiiiifi")}
_libs = {}


def ref_available(kind: str = "xy") -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", _REF[kind][0]))


def _ref_fn(kind: str):
    if kind not in _libs:
        lib = C.CDLL(os.path.join(_HERE, "_ref", _REF[kind][0]))
        fn = getattr(lib, _REF[kind][1])
        fn.restype = None
        P, I, F = C.c_void_p, C.c_int, C.c_float
        last = F if kind == "xy" else I
        fn.argtypes = [P, I, P, I, P, I, I, I, I, I, F, last]
        _libs[kind] = fn
    return _libs[kind]


def ref_bilateral(images: np.ndarray, ins: np.ndarray, sigma_rgb: float,
                  sigma_xy: float) -> np.ndarray:
    """bilateralfilter_batch (bilateralfilter.cpp:42-55): images (N,3,H,W), ins (N,K,H,W)."""
    images = np.ascontiguousarray(images, dtype=np.float32)
    ins = np.ascontiguousarray(ins, dtype=np.float32)
    n, k, h, w = ins.shape
    out = np.zeros_like(ins)
    _ref_fn("xy")(images.ctypes.data, images.size, ins.ctypes.data, ins.size, out.ctypes.data,
                  out.size, n, k, h, w, sigma_rgb, sigma_xy)
    return out


def ref_colorbilateral(images: np.ndarray, ins: np.ndarray, sigma_rgb: float,
                       dim: int) -> np.ndarray:
    """colorbilateralfilter_batch (colorbilateralfilter.cpp:41-54)."""
    images = np.ascontiguousarray(images, dtype=np.float32)
    ins = np.ascontiguousarray(ins, dtype=np.float32)
    n, k, h, w = ins.shape
    out = np.zeros_like(ins)
    _ref_fn("color")(images.ctypes.data, images.size, ins.ctypes.data, ins.size,
                     out.ctypes.data, out.size, n, k, h, w, sigma_rgb, dim)
    return out


# ------------------------------------------------------------------ port
def _lattice_constants(d: int):
    """permutohedral.cpp:160-166 (double math, stored as float) and :444."""
    inv_std_dev = np.float32(math.sqrt(2.0 / 3.0) * (d + 1))
    sf = np.array([1.0 / math.sqrt((i + 2) * (i + 1)) * float(inv_std_dev) for i in range(d)],
                  dtype=np.float32)
    alpha = np.float32(1.0) / np.float32(1 + np.float32(2.0 ** -d))
    return sf, alpha


def _init(feat: np.ndarray):
    """Permutohedral::init, SSE branch (permutohedral.cpp:133-315).

    feat: (P, d) fp32.  Returns (offset (P', d+1) int, bary (P', d+1) fp32, keys (M, d)
    int, M) where P' includes the zero-feature padding of the last SSE block of 4.
    """
    f32 = np.float32
    P, d = feat.shape
    pad = (-P) % 4
    if pad:
        feat = np.concatenate([feat, np.zeros((pad, d), np.float32)])
    sf, _ = _lattice_constants(d)
    dp1 = f32(d + 1)
    inv = f32(1.0) / f32(d + 1)
    Q = feat.shape[0]
    el = np.zeros((Q, d + 1), np.float32)
    sm = np.zeros(Q, np.float32)
    for j in range(d, 0, -1):                       # 181-189
        cf = feat[:, j - 1] * sf[j - 1]
        el[:, j] = sm - f32(j) * cf
        sm = sm + cf
    el[:, 0] = sm
    v = np.rint(inv * el)                           # 192-203 (round half to even)
    rem0 = v * dp1
    s = np.zeros(Q, np.float32)
    for i in range(d + 1):
        s = s + v[:, i]
    rank = np.zeros((Q, d + 1), np.float32)         # 206-215
    for i in range(d):
        di = el[:, i] - rem0[:, i]
        for j in range(i + 1, d + 1):
            c = (di < el[:, j] - rem0[:, j]).astype(np.float32)
            rank[:, i] += c
            rank[:, j] += f32(1) - c
    for i in range(d + 1):                          # 218-224
        rank[:, i] += s
        add = np.where(rank[:, i] < 0, dp1, f32(0))
        sub = np.where(rank[:, i] >= dp1, dp1, f32(0))
        rank[:, i] += add - sub
        rem0[:, i] += add - sub
    bary = np.zeros((Q, d + 2), np.float32)         # 227-243
    rows = np.arange(Q)
    for i in range(d + 1):
        vv = (el[:, i] - rem0[:, i]) * inv
        p = (f32(d) - rank[:, i]).astype(np.int64)
        bary[rows, p] += vv
        bary[rows, p + 1] -= vv
    bary[:, 0] += f32(1) + bary[:, d + 1]
    rk = rank.astype(np.int64)
    # canonical[r][rank] = r if rank <= d - r else r - (d+1)       (151-156)
    keys = np.zeros((Q, d + 1, d), np.int64)
    for r in range(d + 1):
        canon = np.where(rk[:, :d] <= d - r, r, r - (d + 1))
        keys[:, r, :] = (rem0[:, :d] + canon.astype(np.float32)).astype(np.int16)
    # hash_table.find(key, true) in point-major, remainder-minor order (249-256).
    flat = keys.reshape(-1, d)
    uniq, first, inv_idx = np.unique(flat, axis=0, return_index=True, return_inverse=True)
    # number vertices by first insertion, as the reference's table does
    order = np.argsort(first, kind="stable")
    rank_of = np.empty_like(order)
    rank_of[order] = np.arange(len(order))
    offset = rank_of[inv_idx.reshape(-1)].reshape(Q, d + 1)
    return offset, bary[:, : d + 1], uniq[order], len(order)


def _blur_neighbors(keys: np.ndarray, d: int):
    """Neighbour table (permutohedral.cpp:283-305); -1 when absent."""
    lut = {tuple(k): i for i, k in enumerate(keys.tolist())}
    M = len(keys)
    nb = np.full((d + 1, M, 2), -1, np.int64)
    for j in range(d + 1):
        n1 = keys - 1
        n2 = keys + 1
        if j < d:
            n1[:, j] = keys[:, j] + d
            n2[:, j] = keys[:, j] - d
        for i in range(M):
            nb[j, i, 0] = lut.get(tuple(n1[i].tolist()), -1)
            nb[j, i, 1] = lut.get(tuple(n2[i].tolist()), -1)
    return nb


def _compute(offset, bary, nb, M, vals_in: np.ndarray, d: int) -> np.ndarray:
    """Permutohedral::compute for value_size 1 (SSE branch, 464-536), vectorised over
    the K channels (each channel is an independent value_size-1 call)."""
    f32 = np.float32
    P, K = vals_in.shape
    _, alpha = _lattice_constants(d)
    values = np.zeros((M + 1, K), np.float32)       # row 0 = the "-1" neighbour
    o = offset[:P] + 1
    # Splat point-major (all j of point i before point i+1), as the reference: np.add.at
    # is unbuffered and applies the updates in index order.
    contrib = (bary[:P, :, None] * vals_in[:, None, :]).reshape(-1, K)
    np.add.at(values, o.reshape(-1), contrib)
    half = f32(0.5)
    for j in range(d + 1):                          # blur
        n1 = nb[j, :, 0] + 1
        n2 = nb[j, :, 1] + 1
        new = values.copy()
        new[1:] = values[1:] + half * (values[n1] + values[n2])
        values = new
    out = np.zeros((P, K), np.float32)              # slice
    for j in range(d + 1):
        w = (bary[:P, j] * alpha)[:, None]
        out = out + w * values[o[:, j]]
    return out


def port_bilateral(images: np.ndarray, ins: np.ndarray, sigma_rgb: float,
                   sigma_xy: float = 1.0, dim: int = 0) -> np.ndarray:
    """numpy restatement; dim = 0 -> (x, y, r, g, b) features (bilateralfilter.cpp:4-20),
    dim > 0 -> colour planes only (colorbilateralfilter.cpp:4-18)."""
    images = np.asarray(images, np.float32)
    ins = np.asarray(ins, np.float32)
    n, k, h, w = ins.shape
    out = np.zeros_like(ins)
    f32 = np.float32
    for b in range(n):
        im = images.reshape(n, 3, h * w)[b]   # the reference's 3-plane image stride
        if dim == 0:
            yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
            feat = np.stack([xx.reshape(-1).astype(np.float32) / f32(sigma_xy),
                             yy.reshape(-1).astype(np.float32) / f32(sigma_xy),
                             im[0] / f32(sigma_rgb), im[1] / f32(sigma_rgb),
                             im[2] / f32(sigma_rgb)], axis=1)
            d = 5
        else:
            feat = np.stack([im[z] / f32(sigma_rgb) for z in range(dim)], axis=1)
            d = dim
        offset, bary, keys, M = _init(np.ascontiguousarray(feat, np.float32))
        nb = _blur_neighbors(keys, d)
        res = _compute(offset, bary, nb, M, ins[b].reshape(k, -1).T.copy(), d)
        out[b] = res.T.reshape(k, h, w)
    return out
