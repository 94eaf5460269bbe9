"""Dense-CRF losses on the gfx950 permutohedral filter.

Drop-in for the reference's CRF stack:

* ``bilateralfilter_batch`` / ``colorbilateralfilter_batch`` — the SWIG module
  functions (crf/crfwrapper/bilateralfilter/bilateralfilter.cpp:42-55,
  colorbilateralfilter/colorbilateralfilter.cpp:41-54) with the same argument list:
  flattened float32 numpy arrays, ``outs`` written in place.  They run the HIP
  filter through the library's host-compat symbols (H2D -> kernel -> D2H).
* ``bilateral_filter`` / ``color_bilateral_filter`` — the device path on torch
  tensors (no host round trip).
* ``DenseCRFLoss`` / ``ColorDenseCRFLoss`` — crf/dense_crf_loss.py:80-133 and
  crf/color_dense_crf_loss.py:81-134: same constructor arguments, same forward
  (images in [0, 255], softmaxed segmentations), same loss and gradient
  (``-sum(S * AS) / N`` and ``-2 g AS / N``), computed on the GPU end to end.

The filter output is bit-identical to the reference's CPU filter.
There is no CPU fallback: CPU tensors are moved to the segmentation's device for
the images (the reference passes images on the CPU) and rejected otherwise.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd import Function

from . import _lib
from ._lib import check

_WS: Dict[Tuple, torch.Tensor] = {}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _workspace(device: torch.device, n: int, k: int, h: int, w: int, dim: int) -> torch.Tensor:
    # one workspace per stream: the lattice tables are live for the whole call, so two
    # streams filtering concurrently (pipelined clips) must not share them
    key = (device, _stream(), n, k, h, w, dim)
    ws = _WS.get(key)
    if ws is None:
        nbytes = _lib.load().tcam_bilateral_ws_bytes(n, k, h, w, dim)
        if nbytes == 0:
            raise ValueError(f"bilateral filter: unsupported shape N={n} K={k} H={h} W={w} "
                             f"dim={dim} (K <= 8, dim <= 5, 32-bit entry counts)")
        if len(_WS) > 8:
            torch.cuda.synchronize(device)   # no stream may still be using an evicted table
            _WS.clear()
        # zero-filled once: every call leaves its lattice hash table empty again
        ws = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


def _prep(images: torch.Tensor, segs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    if not segs.is_cuda:
        raise RuntimeError("the CRF filter runs on the MI355X HIP path only (no CPU fallback)")
    if images.dim() != 4 or segs.dim() != 4 or images.shape[0] != segs.shape[0] or \
            images.shape[2:] != segs.shape[2:] or images.shape[1] != 3:
        raise ValueError(f"images (N,3,H,W) and segmentations (N,K,H,W) expected, got "
                         f"{tuple(images.shape)} and {tuple(segs.shape)}")
    images = images.to(device=segs.device, dtype=torch.float32).contiguous()
    segs = segs.detach().to(torch.float32).contiguous()
    return images, segs


def _status(ws: torch.Tensor, n: int) -> None:
    st = C.c_int(0)
    check(_lib.load().tcam_bilateral_status(ws.data_ptr(), n, C.byref(st)),
          "tcam_bilateral_status")
    if st.value != 0:
        raise ValueError("bilateral filter: lattice coordinates exceed the packed key range "
                         "(features > ~2000: sigma too small for the image range)")


def bilateral_filter(images: torch.Tensor, segs: torch.Tensor, sigma_rgb: float,
                     sigma_xy: float, check_range: bool = False) -> torch.Tensor:
    """AS = bilateral(S) with (x, y, r, g, b) features (bilateralfilter.cpp:4-40)."""
    images, segs = _prep(images, segs)
    n, k, h, w = segs.shape
    out = torch.empty_like(segs)
    ws = _workspace(segs.device, n, k, h, w, 5)
    check(_lib.load().tcam_bilateral_batch(images.data_ptr(), segs.data_ptr(), out.data_ptr(),
                                           ws.data_ptr(), ws.numel(), n, k, h, w,
                                           float(sigma_rgb), float(sigma_xy), _stream()),
          "tcam_bilateral_batch")
    if check_range:
        _status(ws, n)
    return out


class PreparedLattice:
    """The image-only half of :func:`bilateral_filter` launched ahead of the values:
    ``tcam_bilateral_prepare`` (lattice, hash table, sorted vertex runs of ``images``) runs on
    ``stream`` — e.g. a side stream while the network that produces the segmentation runs —
    and :meth:`apply` filters the segmentation through it on the current stream
    (``tcam_bilateral_apply``: splat, blur, slice).  Bit-identical to bilateral_filter; one
    apply per prepare.  Workspaces come from a per-shape pool, so a lattice prepared for the
    next step never overwrites one still waiting for its apply."""

    _POOL: Dict[Tuple, list] = {}

    def __init__(self, images: torch.Tensor, k: int, sigma_rgb: float, sigma_xy: float,
                 stream: "torch.cuda.Stream | None" = None,
                 ready: "torch.cuda.Event | None" = None):
        if not images.is_cuda:
            raise RuntimeError("the CRF filter runs on the MI355X HIP path only (no CPU fallback)")
        if images.dim() != 4 or images.shape[1] != 3:
            raise ValueError(f"images (N,3,H,W) expected, got {tuple(images.shape)}")
        self._src, self._src_version = images, images._version
        src = images
        images = images.to(torch.float32).contiguous()
        n, _, h, w = images.shape
        self.shape = (n, int(k), h, w)
        self.sigma = (float(sigma_rgb), float(sigma_xy))
        dev = images.device
        key = (dev, n, int(k), h, w)
        pool = PreparedLattice._POOL.setdefault(key, [])
        slot = next((e for e in pool if not e["busy"]), None)
        fresh = slot is None
        if slot is None:
            nbytes = _lib.load().tcam_bilateral_ws_bytes(n, int(k), h, w, 5)
            if nbytes == 0:
                raise ValueError(f"bilateral filter: unsupported shape N={n} K={k} H={h} W={w}")
            slot = {"ws": torch.zeros(nbytes, dtype=torch.uint8, device=dev), "busy": False,
                    "done": None}
            pool.append(slot)
        slot["busy"] = True
        self._slot = slot
        cur = torch.cuda.current_stream(dev)
        st = stream if stream is not None else cur
        if ready is not None and images is src and not fresh:
            st.wait_event(ready)                 # the images are ready at `ready`
        else:
            # the images are produced on `cur` — or a conversion / the new workspace's zero
            # fill was just enqueued there, after `ready`
            st.wait_stream(cur)
        if slot["done"] is not None:
            st.wait_event(slot["done"])          # this workspace's previous apply
        ws = slot["ws"]
        with torch.cuda.stream(st):
            check(_lib.load().tcam_bilateral_prepare(images.data_ptr(), ws.data_ptr(), ws.numel(),
                                                     n, int(k), h, w, self.sigma[0],
                                                     self.sigma[1], st.cuda_stream),
                  "tcam_bilateral_prepare")
            self._ready = torch.cuda.Event()
            self._ready.record(st)
        images.record_stream(st)
        self._images = images                    # alive until the apply is enqueued

    def matches(self, images: torch.Tensor, sigma_rgb: float, sigma_xy: float) -> bool:
        """Prepared from this very tensor (unmodified since) with these sigmas."""
        return (self._slot is not None and images is self._src and
                images._version == self._src_version and
                self.sigma == (float(sigma_rgb), float(sigma_xy)))

    def discard(self) -> None:
        """Release an unused lattice: filtering zeros through it empties its hash table."""
        if self._slot is not None:
            n, k, h, w = self.shape
            self.apply(torch.zeros((n, k, h, w), device=self._slot["ws"].device))

    def apply(self, segs: torch.Tensor, check_range: bool = False) -> torch.Tensor:
        if self._slot is None:
            raise RuntimeError("PreparedLattice.apply: already applied (one apply per prepare)")
        if not segs.is_cuda or tuple(segs.shape) != self.shape:
            raise ValueError(f"segmentations {tuple(segs.shape)} vs the prepared {self.shape}")
        segs = segs.detach().to(torch.float32).contiguous()
        cur = torch.cuda.current_stream(segs.device)
        cur.wait_event(self._ready)
        n, k, h, w = self.shape
        out = torch.empty_like(segs)
        ws = self._slot["ws"]
        check(_lib.load().tcam_bilateral_apply(segs.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                               ws.numel(), n, k, h, w, self.sigma[0],
                                               self.sigma[1], cur.cuda_stream),
              "tcam_bilateral_apply")
        done = torch.cuda.Event()
        done.record(cur)
        self._slot["done"], self._slot["busy"] = done, False
        if check_range:
            _status(ws, n)
        self._slot, self._images, self._src = None, None, None
        return out


def color_bilateral_filter(images: torch.Tensor, segs: torch.Tensor, sigma_rgb: float,
                           dim: int = 3, check_range: bool = False) -> torch.Tensor:
    """AS with colour-only features (colorbilateralfilter.cpp:4-39)."""
    images, segs = _prep(images, segs)
    n, k, h, w = segs.shape
    out = torch.empty_like(segs)
    ws = _workspace(segs.device, n, k, h, w, dim)
    check(_lib.load().tcam_colorbilateral_batch(images.data_ptr(), segs.data_ptr(),
                                                out.data_ptr(), ws.data_ptr(), ws.numel(), n, k,
                                                h, w, float(sigma_rgb), int(dim), _stream()),
          "tcam_colorbilateral_batch")
    if check_range:
        _status(ws, n)
    return out


# ---------------------------------------------------- SWIG-compatible API
def _np_f32(a, name):
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
        raise TypeError(f"{name}: expected a C-contiguous float32 numpy array")
    return a


def bilateralfilter_batch(images, ins, outs, N, K, H, W, sigmargb, sigmaxy):
    """bilateralfilter.hpp:11 through numpy.i (IN_ARRAY1 images/ins, INPLACE_ARRAY1 outs)."""
    images, ins, outs = _np_f32(images, "images"), _np_f32(ins, "ins"), _np_f32(outs, "outs")
    _lib.load().bilateralfilter_batch(images.ctypes.data, images.size, ins.ctypes.data, ins.size,
                                      outs.ctypes.data, outs.size, N, K, H, W, sigmargb, sigmaxy)


def colorbilateralfilter_batch(images, ins, outs, N, K, H, W, sigmargb, DIM):
    """colorbilateralfilter.hpp through numpy.i."""
    images, ins, outs = _np_f32(images, "images"), _np_f32(ins, "ins"), _np_f32(outs, "outs")
    _lib.load().colorbilateralfilter_batch(images.ctypes.data, images.size, ins.ctypes.data,
                                           ins.size, outs.ctypes.data, outs.size, N, K, H, W,
                                           sigmargb, DIM)


# ------------------------------------------------------------- losses
_ENERGY_WS: Dict[Tuple, torch.Tensor] = {}


def _energy_ws(device: torch.device) -> torch.Tensor:
    ekey = (device, _stream())
    ws = _ENERGY_WS.get(ekey)
    if ws is None:
        ws = torch.empty(_lib.load().tcam_crf_energy_ws_bytes() // 4, dtype=torch.float32,
                         device=device)
        _ENERGY_WS[ekey] = ws
    return ws


def _energy(segs: torch.Tensor, AS: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    ws = _energy_ws(segs.device)
    loss = torch.empty(1, dtype=torch.float32, device=segs.device)
    check(lib.tcam_crf_energy(segs.data_ptr(), AS.data_ptr(), segs.numel(), segs.shape[0],
                              loss.data_ptr(), ws.data_ptr(), _stream()), "tcam_crf_energy")
    return loss


def _grad(AS: torch.Tensor, grad_output: torch.Tensor, n: int) -> torch.Tensor:
    g = grad_output.detach().to(device=AS.device, dtype=torch.float32).contiguous()
    grad = torch.empty_like(AS)
    check(_lib.load().tcam_crf_grad(AS.data_ptr(), g.data_ptr(), AS.numel(), n,
                                    grad.data_ptr(), _stream()), "tcam_crf_grad")
    return grad


class DenseCRFLossFunction(Function):
    """crf/dense_crf_loss.py:33-77 on the device (no D2H/H2D, no host sync)."""

    @staticmethod
    def forward(ctx, images, segmentations, sigma_rgb, sigma_xy):
        AS = bilateral_filter(images, segmentations, sigma_rgb, sigma_xy)
        ctx.N = segmentations.shape[0]
        ctx.save_for_backward(AS)
        return _energy(segmentations.detach().float().contiguous(), AS)

    @staticmethod
    def backward(ctx, grad_output):
        (AS,) = ctx.saved_tensors
        return None, _grad(AS, grad_output, ctx.N), None, None


class ColorDenseCRFLossFunction(Function):
    """crf/color_dense_crf_loss.py:33-78 (features: the image planes, DIM = C)."""

    @staticmethod
    def forward(ctx, images, segmentations, sigma_rgb):
        AS = color_bilateral_filter(images, segmentations, sigma_rgb, dim=images.shape[1])
        ctx.N = segmentations.shape[0]
        ctx.save_for_backward(AS)
        return _energy(segmentations.detach().float().contiguous(), AS)

    @staticmethod
    def backward(ctx, grad_output):
        (AS,) = ctx.saved_tensors
        return None, _grad(AS, grad_output, ctx.N), None


def _rescale(images, segmentations, scale_factor):
    # dense_crf_loss.py:113-122: nearest for the image, bilinear for the segmentation.
    if scale_factor == 1.0:
        return images, segmentations
    si = F.interpolate(images, scale_factor=scale_factor, mode="nearest",
                       recompute_scale_factor=False)
    ss = F.interpolate(segmentations, scale_factor=scale_factor, mode="bilinear",
                       recompute_scale_factor=False, align_corners=False)
    return si, ss


class DenseCRFLoss(nn.Module):
    """crf/dense_crf_loss.py:80-133."""

    def __init__(self, weight, sigma_rgb, sigma_xy, scale_factor):
        super().__init__()
        self.weight = weight
        self.sigma_rgb = sigma_rgb
        self.sigma_xy = sigma_xy
        self.scale_factor = scale_factor

    def forward(self, images, segmentations):
        images = images.to(segmentations.device)
        si, ss = _rescale(images, segmentations, self.scale_factor)
        return self.weight * DenseCRFLossFunction.apply(si, ss, self.sigma_rgb,
                                                        self.sigma_xy * self.scale_factor)

    def extra_repr(self):
        return "sigma_rgb={}, sigma_xy={}, weight={}, scale_factor={}".format(
            self.sigma_rgb, self.sigma_xy, self.weight, self.scale_factor)


class ColorDenseCRFLoss(nn.Module):
    """crf/color_dense_crf_loss.py:81-134."""

    def __init__(self, weight, sigma_rgb, scale_factor):
        super().__init__()
        self.weight = weight
        self.sigma_rgb = sigma_rgb
        self.scale_factor = scale_factor

    def forward(self, images, segmentations):
        assert images.ndim == 4
        images = images.to(segmentations.device)
        si, ss = _rescale(images, segmentations, self.scale_factor)
        return self.weight * ColorDenseCRFLossFunction.apply(si, ss, self.sigma_rgb)

    def extra_repr(self):
        return "sigma_rgb={}, weight={}, scale_factor={}".format(
            self.sigma_rgb, self.weight, self.scale_factor)
