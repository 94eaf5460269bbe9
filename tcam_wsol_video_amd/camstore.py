"""Stage-1 CAM store and ROI-threshold files.

The reference builds, once per dataset split, one low-resolution CAM per frame with a
batch-1 forward each, stores it as ``<fdout>/<reformat_id(id)>.pt`` (a 2-D CPU float
tensor, ``torch.save``) and optionally a ``<tag>.txt`` of ``id,thresh`` lines whose
threshold is ``STOtsu(floor(bilinear_align_corners(cam, 224) * 255)) / 255``
(learning/inference_wsol.py:1072-1129 ``_build_store_std_cam_low`` and :1136-1163
``_build_roi_from_cams``).  The training loader reads both back
(datasets/wsol_loader.py:183-188 ``get_cams_paths``, :299-317 ``_load_roi_thresholds``)
and turns each frame's temporal max into a ROI with that threshold (:571-611).

Here a whole batch is one forward (the caller's batched extractor), the thresholds are
one ``tcam_stotsu_roi_thresh`` launch, and the ROIs of a batch one ``tcam_get_roi``
launch with per-frame thresholds.  The files are byte-compatible with the reference's:
``torch.save`` of a contiguous 2-D float32 CPU tensor, and ``str(float)`` lines.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import check

CROP_SIZE = 224  # configure/constants.py:234


def reformat_id(img_id: str) -> str:
    """utils/shared.py:212-218."""
    return img_id.replace("/", "_").replace("\\", "_")


def get_cams_paths(root_data_cams: str, image_ids: Sequence[str]) -> Dict[str, str]:
    """datasets/wsol_loader.py:183-188."""
    return {i: os.path.join(root_data_cams, f"{reformat_id(i)}.pt") for i in image_ids}


def roi_thresholds(cams: torch.Tensor, size: int = CROP_SIZE) -> torch.Tensor:
    """STOtsu ROI thresholds in [0, 255] of (B, h, w) device CAMs (float32)."""
    if not cams.is_cuda:
        raise RuntimeError("roi_thresholds runs on the GPU only (no CPU fallback)")
    lib = _lib.load()
    cams = cams.float().contiguous()
    B, h, w = cams.shape
    th = torch.empty(B, device=cams.device, dtype=torch.float32)
    check(lib.tcam_stotsu_roi_thresh(cams.data_ptr(), B, h, w, int(size), th.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream),
          "tcam_stotsu_roi_thresh")
    return th


def write_roi_file(path: str, ids: Sequence[str], th255: torch.Tensor, mode: str = "w"):
    """``id,thresh`` lines, thresh = th / 255. as python floats (inference_wsol.py:1122-1124)."""
    with open(path, mode) as f:
        for i, t in zip(ids, th255.detach().cpu().tolist()):
            f.write(",".join([str(i), str(float(t) / 255.)]) + "\n")


def load_roi_thresholds(path: str) -> Optional[Dict[str, float]]:
    """One split of wsol_loader.py:299-317 (None when the file is absent)."""
    if not os.path.isfile(path):
        return None
    out: Dict[str, float] = {}
    with open(path) as f:
        for line in f.read().splitlines():
            z = line.split(",")
            assert len(z) == 2, line
            assert z[0] not in out
            out[z[0]] = float(z[1])
    return out


def build_store_std_cam_low(extract: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
                            batches: Iterable[Tuple[torch.Tensor, torch.Tensor, Sequence[str]]],
                            fdout: str, cams_roi_file: Optional[str] = None) -> int:
    """inference_wsol.py:1072-1129 over batches.

    ``extract(images, targets) -> (B, h', w')`` device CAMs (e.g. a forward of the
    STD_CL model followed by :class:`~tcam_wsol_video_amd.inference.CAM`, or the TCAM
    ``SegmentationCam``); nan_to_num(0, 1, 0) is applied as the reference.  Returns the
    number of frames stored."""
    os.makedirs(fdout, exist_ok=True)
    roifx = open(cams_roi_file, "w") if cams_roi_file else None
    n = 0
    try:
        for images, targets, ids in batches:
            with torch.no_grad():
                cams = extract(images, targets)
                if cams.ndim == 2:
                    cams = cams[None]
                cams = torch.nan_to_num(cams.float(), nan=0.0, posinf=1.0, neginf=0.0)
                if roifx is not None:
                    th = roi_thresholds(cams)
                    for i, t in zip(ids, th.cpu().tolist()):
                        roifx.write(",".join([str(i), str(float(t) / 255.)]) + "\n")
                host = cams.detach().cpu()
            for i, image_id in enumerate(ids):
                torch.save(host[i].clone(), os.path.join(fdout, f"{reformat_id(image_id)}.pt"))
            n += len(ids)
    finally:
        if roifx is not None:
            roifx.close()
    return n


def load_std_cams(fdcams: str, ids: Sequence[str], device=None) -> torch.Tensor:
    """Read stored CAMs (``torch.load(weights_only=True)``) -> (B, 1, h', w') float32."""
    paths = get_cams_paths(fdcams, ids)
    cams = [torch.load(paths[i], map_location="cpu", weights_only=True) for i in ids]
    for c in cams:
        assert c.ndim == 2, c.ndim
    out = torch.stack(cams).float().unsqueeze(1)
    return out.to(device) if device is not None else out


def build_roi_from_cams(fdcams: str, out_roi_file: str, s_ids: Sequence[str],
                        device=None, batch: int = 1024) -> int:
    """inference_wsol.py:1136-1163: thresholds of stored CAMs, batched per shape."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    ids: List[str] = list(s_ids)
    with open(out_roi_file, "w"):
        pass
    for k in range(0, len(ids), batch):
        chunk = ids[k:k + batch]
        cams = load_std_cams(fdcams, chunk)
        write_roi_file(out_roi_file, chunk, roi_thresholds(cams[:, 0].to(device)), mode="a")
    return len(ids)
