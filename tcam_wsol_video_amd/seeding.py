"""TCAM pseudo-label seeding on the device (``tcam_tcam_seeder`` / ``tcam_get_roi``).

Mirrors the reference API (dlib/cams/tcam_seeding.py):

* :class:`TCAMSeeder` — same constructor arguments as the reference
  (tcam_seeding.py:53-142), ``forward(x, roi=None) -> (b, h, w) long`` with
  ``seg_ignore_idx`` / 1 (foreground) / 0 (background), ``use_all_roi``,
  ``set_seed_tech``.  One kernel launch seeds the whole batch (the reference
  loops over samples in Python, tcam_seeding.py:230-236).
* :class:`GetRoiSingleCam` — ``__call__(cam, thresh=None) -> (roi, bbox_mask,
  bbox)`` plus a batched ``batch(cams)``.

Sampling: ``torch.multinomial(p, k, replacement=False)`` is ``topk(p / q, k)``
with ``q ~ Exp(1)`` in torch itself; here ``q`` comes from a counter-based
Philox4x32-10 keyed by (pixel, frame, call offset; seed), so a seeder's draws
are reproducible from ``manual_seed`` and independent of batch composition.
There is no CPU fallback: CPU tensors are refused.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import check

SEED_UNIFORM = "seed_uniform"
SEED_WEIGHTED = "seed_weighted"
SEED_TECHS = [SEED_UNIFORM, SEED_WEIGHTED]
ROI_ALL = "roi_all"
ROI_H_DENSITY = "roi_high_density"
ROI_LARGEST = "largest"
ROI_SELECT = [ROI_ALL, ROI_H_DENSITY, ROI_LARGEST]
_ROI_CODE = {ROI_ALL: 0, ROI_H_DENSITY: 1, ROI_LARGEST: 2}
MAX_HW = 320 * 320


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ws(nbytes: int, dev) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), device=dev, dtype=torch.uint8)


def _check_cams(x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        raise RuntimeError("TCAM seeding runs on the GPU only (no CPU fallback)")
    if x.dtype != torch.float32:
        x = x.float()
    return x.contiguous()


def prepare_std_cams(std_cams: torch.Tensor, image_size: Tuple[int, int]) -> torch.Tensor:
    """Trainer.prepare_std_cams_disq (learning/train_wsol.py:417-432): (b, 1, h', w')
    stage-1 CAMs -> nan_to_num -> bilinear (align_corners=False) to image_size ->
    nan_to_num, as (b, 1, H, W) fp32."""
    lib = _lib.load()
    assert std_cams.ndim == 4 and std_cams.shape[1] == 1, std_cams.shape
    x = _check_cams(std_cams.detach())
    b, _, h, w = x.shape
    Ho, Wo = int(image_size[0]), int(image_size[1])
    out = torch.empty((b, 1, Ho, Wo), device=x.device, dtype=torch.float32)
    check(lib.tcam_prepare_std_cams(x.data_ptr(), out.data_ptr(), b, h, w, Ho, Wo, _stream()),
          "tcam_prepare_std_cams")
    return out


class TCAMSeeder(torch.nn.Module):
    """dlib/cams/tcam_seeding.py:53-300 on one kernel per batch."""

    def __init__(self, seed_tech: str, min_: int, max_: int, max_p: float, min_p: float,
                 fg_erode_k: int, fg_erode_iter: int, ksz: int, support_background: bool,
                 multi_label_flag: bool, seg_ignore_idx: int, cuda_id: int, roi_method: str,
                 p_min_area_roi: float, use_roi: bool, seed: int = 0):
        super().__init__()
        assert seed_tech in SEED_TECHS, seed_tech
        assert not multi_label_flag
        assert isinstance(cuda_id, int) and cuda_id >= 0, cuda_id
        assert isinstance(ksz, int) and ksz > 0
        assert isinstance(min_, int) and isinstance(max_, int)
        assert min_ >= 0 and max_ >= 0 and min_ + max_ > 0
        assert isinstance(min_p, float) and 0. <= min_p <= 1.
        assert isinstance(max_p, float) and 0. <= max_p <= 1.
        assert isinstance(fg_erode_k, int) and fg_erode_k >= 1
        assert isinstance(fg_erode_iter, int) and fg_erode_iter >= 0
        if fg_erode_iter > 0:
            assert fg_erode_k > 1
        assert roi_method in ROI_SELECT, roi_method
        assert 0. < p_min_area_roi < 1., p_min_area_roi
        self.seed_tech = seed_tech
        self._device = torch.device(cuda_id)
        self.min_, self.max_ = min_, max_
        self.min_p, self.max_p = min_p, max_p
        self.fg_erode_k, self.fg_erode_iter = fg_erode_k, fg_erode_iter
        self.ksz = ksz
        self.support_background = support_background
        self.multi_label_flag = multi_label_flag
        self.ignore_idx = seg_ignore_idx
        self.roi_method = roi_method
        self.p_min_area_roi = p_min_area_roi
        self.use_roi = use_roi
        self._seed = int(seed) & (2 ** 64 - 1)
        self._offset = 0
        self._ws: Optional[torch.Tensor] = None
        self.last_roi: Optional[torch.Tensor] = None

    def manual_seed(self, seed: int) -> None:
        self._seed = int(seed) & (2 ** 64 - 1)
        self._offset = 0

    def set_seed_tech(self, seed_tech: str) -> None:
        assert seed_tech in SEED_TECHS, seed_tech
        self.seed_tech = seed_tech

    def _workspace(self, B: int, H: int, W: int, dev) -> torch.Tensor:
        need = int(_lib.load().tcam_seeder_ws_bytes(B, H, W))
        if self._ws is None or self._ws.numel() < need or self._ws.device != dev:
            self._ws = _ws(need, dev)
        return self._ws

    def seeds_i32(self, x: torch.Tensor, roi: Optional[torch.Tensor] = None,
                  keep_roi: bool = False) -> torch.Tensor:
        """(b, 1, h, w) cams -> (b, h, w) int32 seeds (the training step's dtype)."""
        lib = _lib.load()
        assert x.ndim == 4 and x.shape[1] == 1, x.shape
        x = _check_cams(x)
        b, _, h, w = x.shape
        assert h * w <= MAX_HW, (h, w)
        r = None
        if roi is not None:
            assert torch.is_tensor(roi) and roi.ndim == 4 and roi.shape[0] == b
            assert roi.shape[1] == 1 and roi.shape[2:] == x.shape[2:]
            r = roi.to(device=x.device, dtype=torch.uint8).contiguous()
        out = torch.empty((b, h, w), device=x.device, dtype=torch.int32)
        roi_out = torch.empty((b, h, w), device=x.device, dtype=torch.uint8) if keep_roi else None
        ws = self._workspace(b, h, w, x.device)
        check(lib.tcam_tcam_seeder(
            x.data_ptr(), None if r is None else r.data_ptr(), out.data_ptr(), b, h, w,
            1 if self.seed_tech == SEED_WEIGHTED else 0, self.min_, self.max_,
            float(self.max_p), float(self.min_p), self.fg_erode_k, self.fg_erode_iter,
            self.ksz, int(self.ignore_idx), _ROI_CODE[self.roi_method],
            float(self.p_min_area_roi), int(bool(self.use_roi)), self._seed, self._offset,
            None if roi_out is None else roi_out.data_ptr(), None, ws.data_ptr(), ws.numel(),
            _stream()), "tcam_tcam_seeder")
        self._offset += 1
        self.last_roi = roi_out
        return out

    def forward(self, x: torch.Tensor, roi: Optional[torch.Tensor] = None) -> torch.Tensor:
        """tcam_seeding.py:187-258 -> (b, h, w) torch.long."""
        return self.seeds_i32(x, roi).long()

    def use_all_roi(self, x: torch.Tensor, roi: torch.Tensor = None) -> torch.Tensor:
        """tcam_seeding.py:260-300: ignore_idx everywhere, 1 where roi == 1."""
        assert x.ndim == 4 and roi is not None and roi.ndim == 4
        assert roi.shape[0] == x.shape[0] and roi.shape[1] == 1 and roi.shape[2:] == x.shape[2:]
        out = torch.full((x.shape[0],) + tuple(x.shape[2:]), self.ignore_idx,
                         dtype=torch.long, device=x.device)
        out[roi.squeeze(1) == 1] = 1
        return out

    def extra_repr(self):
        return (f"min_={self.min_}, max_={self.max_}, min_p={self.min_p},"
                f"max_p={self.max_p}, ksz={self.ksz}, fg_erode_k: "
                f"{self.fg_erode_k}, fg_erode_iter: {self.fg_erode_iter}"
                f"support_background={self.support_background},"
                f"multi_label_flag={self.multi_label_flag}, "
                f"seg_ignore_idx={self.ignore_idx}, seed_tech={self.seed_tech}")


class GetRoiSingleCam:
    """tcam_seeding.py:303-406 (skimage Otsu, 4-connected labels) on the device."""

    def __init__(self, roi_method: str, p_min_area_roi: float):
        assert roi_method in ROI_SELECT, roi_method
        assert 0 < p_min_area_roi < 1., p_min_area_roi
        self.roi_method = roi_method
        self.p_min_area_roi = p_min_area_roi

    def batch(self, cams: torch.Tensor, thresh=None
              ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """cams (B, h, w) -> (roi (B,h,w) uint8, bbox (B,4) int32, th (B,) float32 in
        [0, 255]).  thresh: None (Otsu), a float in [0, 1], or a (B,) sequence / tensor
        of per-frame thresholds (NaN or < 0: Otsu for that frame) — the per-frame
        ``std_cams_thresh_file`` values of wsol_loader.py:573-611."""
        lib = _lib.load()
        cams = _check_cams(cams)
        assert cams.ndim == 3
        B, h, w = cams.shape
        assert h * w <= MAX_HW
        scalar, per = -1.0, None
        if thresh is not None:
            if isinstance(thresh, (int, float)):
                assert thresh >= 0, thresh
                scalar = float(thresh)
            else:
                per = torch.as_tensor(thresh, dtype=torch.float64).to(cams.device)
                assert per.shape == (B,), per.shape
                per = per.contiguous()
        roi = torch.empty((B, h, w), device=cams.device, dtype=torch.uint8)
        bbox = torch.empty((B, 4), device=cams.device, dtype=torch.int32)
        th = torch.empty((B,), device=cams.device, dtype=torch.float32)
        ws = _ws(lib.tcam_seeder_ws_bytes(B, h, w), cams.device)
        check(lib.tcam_get_roi(cams.data_ptr(), B, h, w, _ROI_CODE[self.roi_method],
                               float(self.p_min_area_roi), scalar,
                               None if per is None else per.data_ptr(), roi.data_ptr(),
                               bbox.data_ptr(), th.data_ptr(), ws.data_ptr(), ws.numel(),
                               _stream()), "tcam_get_roi")
        return roi, bbox, th

    def __call__(self, cam: torch.Tensor, thresh: float = None):
        """-> (final_roi long (h,w), bbox_mask float (h,w), bbox float (1,4)), on cam's device."""
        assert torch.is_tensor(cam) and cam.ndim == 2, cam.ndim
        roi, bbox, _ = self.batch(cam[None], thresh)
        h, w = cam.shape
        x0, y0, x1, y1 = [int(v) for v in bbox[0].tolist()]
        mask = torch.zeros((h, w), dtype=torch.float32, device=cam.device)
        mask[y0:y1, x0:x1] = 1.
        return roi[0].long(), mask, bbox.float().reshape(1, 4)
