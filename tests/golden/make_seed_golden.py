"""Generate tests/golden/tcam_seeder.npz from the REFERENCE TCAMSeeder.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_seed_golden.py               # tcam_seeder.npz
    python tests/golden/make_seed_golden.py --roi-thresh  # roi_thresh.npz

Imported from the reference (read-only, not copied): dlib/cams/tcam_seeding.py
(TCAMSeeder, _OneSample, _SFG, _SBG, GetRoiSingleCam) and its imports
dlib/cams/core_seeding.py, dlib/cams/decay_temp.py, dlib/configure/constants.py,
dlib/utils/wsol.py.

Third-party modules absent from this image are stubbed by the oracle's
restatements of the pinned versions (oracle/seed_ref.py): skimage 0.17.2
``threshold_otsu`` / ``measure.label``, kornia 0.6.4 ``erosion`` / ``dilation``;
pynvml / cv2 are import-only stubs (the seeder path with roi_all / a given roi
never calls cv2).  TCAMSeeder pins its device to ``cuda_id``; it is built with
ksz=1 / no erosion (so nothing is allocated on CUDA) and then re-pointed at the
CPU with the requested kernel, exactly the attributes __init__ would have set.

Sampling is random in the reference (torch.multinomial); these vectors use
``max_`` / ``min_`` >= the candidate count, where multinomial without
replacement returns every candidate, so the output is deterministic and pins
everything but the draw: the Otsu ROI, the optional erosion, the stable top-n
candidate sets, the ``+1e-8`` / ``cam*roi`` numerics, dilation, conflict removal
and label assignment.  The draw itself is pinned distributionally against
torch.multinomial in tests/test_seed_oracle.py.
"""
from __future__ import annotations

import importlib
import os
import sys
sys.dont_write_bytecode = True  # nothing may be written under /root/reference
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import seed_ref as SR  # noqa: E402
import make_golden  # noqa: E402


def _torch_morph(x: torch.Tensor, kernel: torch.Tensor, dilate: bool) -> torch.Tensor:
    # kornia 0.6.4 flat morphology, all-ones kernel, geodesic border.
    k = kernel.shape[0]
    out = SR._morph(x[0, 0].cpu().numpy().astype(np.int64), k,
                    np.maximum if dilate else np.minimum)
    return torch.from_numpy(out).to(x.dtype)[None, None]


def install_seed_stubs():
    make_golden._install_stubs()
    sk = types.ModuleType("skimage")
    sku = types.ModuleType("skimage.util")
    skud = types.ModuleType("skimage.util.dtype")
    skud.dtype_range = {}
    skf = types.ModuleType("skimage.filters")
    skf.threshold_otsu = lambda image, nbins=256: SR.skimage_otsu(image, nbins)
    skm = types.ModuleType("skimage.measure")

    def label(x, background=0, connectivity=1, return_num=False):
        assert background == 0 and connectivity == 1
        lab, n = SR.label4(x)
        return (lab, n) if return_num else lab

    skm.label = label
    for name, m in (("skimage", sk), ("skimage.util", sku), ("skimage.util.dtype", skud),
                    ("skimage.filters", skf), ("skimage.measure", skm)):
        sys.modules[name] = m
    ko = types.ModuleType("kornia")
    kom = types.ModuleType("kornia.morphology")

    def _batched(fn_dilate):
        def f(t, kernel):
            return torch.cat([_torch_morph(t[i:i + 1], kernel, fn_dilate)
                              for i in range(t.shape[0])], 0)
        return f

    kom.dilation = _batched(True)
    kom.erosion = _batched(False)
    sys.modules["kornia"] = ko
    sys.modules["kornia.morphology"] = kom
    for pkg in ("dlib.utils",):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(make_golden.REF, *pkg.split("."))]
        sys.modules[pkg] = m
    ts = importlib.import_module("dlib.cams.tcam_seeding")
    # GetRoiSingleCam's bbox tail (cv2 RETR_EXTERNAL) is discarded by _OneSample
    # (tcam_seeding.py:478): replace it by a dummy so cv2 is never needed.
    ts.compute_bboxes_from_scoremaps_ext_contours = \
        lambda **kw: ([np.array([[0, 0, 1, 1]])], 1)
    return ts


def ref_seeder(ts, cfg):
    s = ts.TCAMSeeder(
        seed_tech=cfg["seed_tech"], min_=cfg["min_"], max_=cfg["max_"], max_p=cfg["max_p"],
        min_p=cfg["min_p"], fg_erode_k=cfg["fg_erode_k"], fg_erode_iter=0, ksz=1,
        support_background=False, multi_label_flag=False,
        seg_ignore_idx=cfg["seg_ignore_idx"], cuda_id=0, roi_method=cfg["roi_method"],
        p_min_area_roi=cfg["p_min_area_roi"], use_roi=cfg["use_roi"])
    s._device = torch.device("cpu")
    s.ksz = cfg["ksz"]
    s.kernel = torch.ones((s.ksz, s.ksz), dtype=torch.long) if s.ksz > 1 else None
    s.fg_erode_iter = cfg["fg_erode_iter"]
    if s.fg_erode_iter > 0:
        s.fg_kernel_erode = torch.ones((s.fg_erode_k, s.fg_erode_k), dtype=torch.long)
    return s


def synth_cams(rng, b, h, w):
    """Smooth blob CAMs in [0,1] (+ one flat frame and one quantised frame)."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    cams = np.zeros((b, 1, h, w), np.float32)
    for i in range(b):
        c = np.zeros((h, w), np.float32)
        for _ in range(rng.integers(1, 4)):
            cy, cx = rng.uniform(0, h), rng.uniform(0, w)
            s = rng.uniform(0.1, 0.3) * max(h, w)
            c += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s)).astype(np.float32)
        c += 0.05 * rng.random((h, w)).astype(np.float32)
        c = (c - c.min()) / (c.max() - c.min())
        cams[i, 0] = c
    if b > 2:
        cams[1, 0] = 0.25                                  # flat: no seeds
        cams[2, 0] = np.round(cams[2, 0] * 8) / 8          # heavy ties
    return cams


CASES = [
    # name, (b, h, w), cfg overrides
    ("readme_roi_all", (4, 40, 48), dict()),
    ("no_roi_uniform", (3, 33, 29), dict(use_roi=False, seed_tech=SR.SEED_UNIFORM)),
    ("largest_erode", (3, 40, 40), dict(roi_method=SR.ROI_LARGEST, fg_erode_iter=1,
                                        fg_erode_k=3)),
    ("hdensity", (3, 37, 45), dict(roi_method=SR.ROI_H_DENSITY, p_min_area_roi=0.1)),
    ("ksz1_given_roi", (3, 32, 32), dict(ksz=1, roi_method=SR.ROI_ALL, given_roi=True)),
    ("ksz4_even", (3, 36, 30), dict(ksz=4, max_p=0.3, min_p=0.2)),
]


def main():
    ts = install_seed_stubs()
    rng = np.random.default_rng(7)
    out = {}
    for name, (b, h, w), over in CASES:
        over = dict(over)
        given = over.pop("given_roi", False)
        cfg = SR.default_cfg(**over)
        cfg["max_"] = cfg["min_"] = 10 ** 9                 # deterministic: all candidates
        cams = synth_cams(rng, b, h, w)
        roi = None
        if given:
            roi = (rng.random((b, 1, h, w)) < 0.5).astype(np.int64)
        s = ref_seeder(ts, cfg)
        with torch.no_grad():
            seeds = s(torch.from_numpy(cams), None if roi is None else torch.from_numpy(roi))
        out[f"{name}/cams"] = cams
        out[f"{name}/seeds"] = seeds.numpy().astype(np.int16)
        if roi is not None:
            out[f"{name}/roi"] = roi.astype(np.uint8)
        out[f"{name}/cfg"] = np.array(repr(sorted(cfg.items())))
        # GetRoiSingleCam (roi only; bbox needs cv2 and is not golden)
        for m in (SR.ROI_ALL, SR.ROI_LARGEST, SR.ROI_H_DENSITY):
            g = ts.GetRoiSingleCam(roi_method=m, p_min_area_roi=cfg["p_min_area_roi"])
            rois = []
            for i in range(b):
                if cams[i, 0].min() == cams[i, 0].max():
                    rois.append(np.zeros((h, w), np.uint8))
                    continue
                th = g.get_thresh(cams[i, 0])
                out[f"{name}/otsu_{i}"] = np.float32(th)
                if m == SR.ROI_ALL:
                    r, _, _ = g(torch.from_numpy(cams[i, 0]))
                    rois.append(r.numpy().astype(np.uint8))
                else:
                    rois.append(_roi_no_bbox(g, cams[i, 0], m))
            out[f"{name}/roi_{m}"] = np.stack(rois)
        print(name, "seeds: fg", int((seeds == 1).sum()), "bg", int((seeds == 0).sum()))
    np.savez_compressed(os.path.join(HERE, "tcam_seeder.npz"), **out)


def _roi_no_bbox(g, cam, m):
    """GetRoiSingleCam.__call__ up to final_roi (tcam_seeding.py:312-371); the
    cv2 bbox tail is a dummy (install_seed_stubs)."""
    r, _, _ = g(torch.from_numpy(cam))
    return r.numpy().astype(np.uint8)


if __name__ == "__main__" and "--roi-thresh" not in sys.argv:
    main()


def make_roi_thresh_golden():
    """ROI thresholds of stored CAMs by the reference's own STOtsu
    (cams/core_seeding.py:23-56) over F.interpolate(align_corners=True) as
    inference_wsol.py:1144-1159 -> tests/golden/roi_thresh.npz."""
    install_seed_stubs()
    cs = importlib.import_module("dlib.cams.core_seeding")
    import torch.nn.functional as F
    rng = np.random.default_rng(11)
    cams = synth_cams(rng, 12, 28, 28)
    cams[5, 0] = np.round(cams[5, 0] * 3) / 3
    cams[6, 0] = 0.0
    cams[6, 0, 3:9, 4:20] = 1.0
    th = []
    for i in range(cams.shape[0]):
        full = F.interpolate(torch.from_numpy(cams[i, 0])[None, None], size=(224, 224),
                             mode="bilinear", align_corners=True)
        th.append(float(cs.STOtsu()(torch.floor(full * 255)).item()))
    np.savez_compressed(os.path.join(HERE, "roi_thresh.npz"), cams=cams[:, 0],
                        th=np.array(th, np.float32),
                        lines=np.array([str(t / 255.) for t in th]))


if __name__ == "__main__" and "--roi-thresh" in sys.argv:
    make_roi_thresh_golden()
