"""Generate tests/golden/tcam_losses.npz (and rgb_joint_crf.npz) from the REFERENCE TCAM
training losses.

Run in the build container only (needs /root/reference and oracle/_ref; never on the
GPU box):

    make -C oracle && python tests/golden/make_train_golden.py [losses] [rgb]

Imported from the reference (read-only, not copied): dlib/losses/{master,core,tcam,elb}.py
(MasterLoss, ElementaryLoss, SelfLearningTcams, ConRanFieldTcams, MaxSizePositiveTcams,
RgbJointConRanFieldTcams, ELB) and dlib/crf/{dense,color_dense}_crf_loss.py, assembled the
way process/instantiators.py:143-245 does for task TCAM with the README's settings
(README.md:297-333: crf_tc_lambda 2e-9, sigma 15/100, scale 1; max_sizepos_tc_lambda 0.01;
sl_tc_lambda 1; elb_init_t 1, max_t 10, mulcoef 1.01).

Environment patches, none of which touches the arithmetic:
  * ``bilateralfilter`` / ``colorbilateralfilter`` (SWIG modules, not buildable: swig is
    absent) are shims that call the reference's own bilateralfilter_batch /
    colorbilateralfilter_batch compiled from its sources into oracle/_ref by
    oracle/Makefile;
  * ELB creates its buffers on ``cuda:<current_device>`` (elb.py:52-69) and
    DenseCRFLossFunction calls torch.cuda.synchronize (dense_crf_loss.py:43): both are
    pointed at the CPU while the modules are built and run;
  * the losses get ``cuda_id="cpu"`` (ElementaryLoss/MasterLoss take a torch device).

Each case stores the inputs (fcams, seeds, raw images, ELB t) and the reference's
per-term losses, total, and d total / d fcams from its autograd.
"""
from __future__ import annotations

import importlib
import os
import sys
sys.dont_write_bytecode = True  # nothing may be written under /root/reference
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import crf_ref  # noqa: E402


def _install():
    sys.path.insert(0, REF)
    for pkg in ("dlib", "dlib.losses", "dlib.crf"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, *pkg.split("."))]
        sys.modules[pkg] = m

    def bilateralfilter_batch(images, segs, out, n, k, h, w, sigma_rgb, sigma_xy):
        res = crf_ref.ref_bilateral(np.asarray(images).reshape(n, 3, h, w),
                                    np.asarray(segs).reshape(n, k, h, w), sigma_rgb, sigma_xy)
        out[:] = res.reshape(-1)

    bf = types.ModuleType("bilateralfilter")
    bf.bilateralfilter = None
    bf.bilateralfilter_batch = bilateralfilter_batch
    def colorbilateralfilter_batch(images, segs, out, n, k, h, w, sigma_rgb, dim):
        res = crf_ref.ref_colorbilateral(np.asarray(images).reshape(n, dim, h, w),
                                         np.asarray(segs).reshape(n, k, h, w), sigma_rgb, dim)
        out[:] = res.reshape(-1)

    cbf = types.ModuleType("colorbilateralfilter")
    cbf.colorbilateralfilter = None
    cbf.colorbilateralfilter_batch = colorbilateralfilter_batch
    sys.modules["bilateralfilter"] = bf
    sys.modules["colorbilateralfilter"] = cbf
    # ELB buffers on cuda:<current_device>, DenseCRFLossFunction's synchronize -> CPU
    torch.cuda.current_device = lambda: 0
    torch.cuda.synchronize = lambda *a, **k: None
    _tensor = torch.tensor

    def _cpu_tensor(*a, device=None, **k):
        if device is not None and torch.device(device).type == "cuda":
            device = "cpu"
        return _tensor(*a, device=device, **k)

    torch.tensor = _cpu_tensor
    master = importlib.import_module("dlib.losses.master")
    tcam = importlib.import_module("dlib.losses.tcam")
    elb = importlib.import_module("dlib.losses.elb")
    return master, tcam, elb


def reference_loss(mods, elb_t: float, lam_size: float = 0.01):
    master, tcam, elb_mod = mods
    ml = master.MasterLoss(cuda_id="cpu")
    elb = elb_mod.ELB(init_t=1., max_t=10., mulcoef=1.01)
    ml.add(tcam.ConRanFieldTcams(cuda_id="cpu", lambda_=2e-9, sigma_rgb=15., sigma_xy=100.,
                                 scale_factor=1., support_background=False,
                                 multi_label_flag=False))
    size = tcam.MaxSizePositiveTcams(cuda_id="cpu", lambda_=lam_size, elb=elb,
                                     support_background=False, multi_label_flag=False)
    size.set_t(float(elb_t))
    ml.add(size)
    ml.add(tcam.SelfLearningTcams(cuda_id="cpu", lambda_=1., support_background=False,
                                  multi_label_flag=False, seg_ignore_idx=-255))
    return ml


def make_case(mods, n, h, w, seed, elb_t, empty_frame=False):
    g = torch.Generator().manual_seed(seed)
    fcams = torch.randn(n, 2, h, w, generator=g) * 2.0
    if empty_frame:   # frame 0 predicts background everywhere: its ELB argument crosses ct
        fcams[0, 0] += 30.0
        fcams[0, 1] -= 30.0
    raw = (torch.rand(n, 3, h, w, generator=g) * 255).round()
    seeds = torch.randint(-1, 2, (n, h, w), generator=g)
    seeds[seeds < 0] = -255
    ml = reference_loss(mods, elb_t)
    f = fcams.clone().requires_grad_(True)
    total = ml(epoch=0, fcams=f, raw_img=raw, seeds=seeds)
    total.backward()
    crf, size, sl = [float(t.detach().sum()) for t in ml.l_holder[1:]]
    return dict(fcams=fcams.numpy(), raw=raw.numpy(), seeds=seeds.numpy().astype(np.int32),
                elb_t=np.float64(elb_t), total=np.float64(float(total.detach().sum())),
                sl=np.float64(sl), crf=np.float64(crf), size=np.float64(size),
                grad=f.grad.numpy())


# RgbJointConRanFieldTcams cases: (seq_iter, frm_iter, h, w, seed).  Frame order within
# a batch is shuffled (group_ordered_frames sorts it), "b" is a knn_tc batch repeated by
# _fill_minibatch (duplicate frames, tied frame ids), "c" holds a one-frame group (skipped),
# "d" one 3-frame group at 224^2 (knn_tc = 1, the README crop).
RGB_CASES = {
    "a": ([1, 0, 1, 0, 0, 1], [2, 1, 0, 0, 2, 1], 32, 40, 11),
    "b": ([3, 3, 3, 7, 7, 3, 3, 3], [0, 1, 2, 0, 1, 0, 1, 2], 24, 20, 12),
    "c": ([0, 1, 1, 2], [0, 0, 1, 0], 16, 24, 13),
    "d": ([5, 5, 5], [1, 0, 2], 224, 224, 14),
}


def make_rgb_case(mods, seq, frm, h, w, seed, lam=2e-9, sigma_rgb=15.):
    master, tcam, _ = mods
    n = len(seq)
    g = torch.Generator().manual_seed(seed)
    fcams = torch.randn(n, 2, h, w, generator=g) * 2.0
    raw = (torch.rand(n, 3, h, w, generator=g) * 255).round()
    ml = master.MasterLoss(cuda_id="cpu")
    ml.add(tcam.RgbJointConRanFieldTcams(cuda_id="cpu", lambda_=lam, sigma_rgb=sigma_rgb,
                                         scale_factor=1., support_background=False,
                                         multi_label_flag=False))
    f = fcams.clone().requires_grad_(True)
    seq_t = torch.tensor(seq, dtype=torch.float)
    frm_t = torch.tensor(frm, dtype=torch.float)
    total = ml(epoch=0, fcams=f, raw_img=raw, seq_iter=seq_t, frm_iter=frm_t)
    total.backward()
    return dict(fcams=fcams.numpy(), raw=raw.numpy().astype(np.uint8), seq=seq_t.numpy(),
                frm=frm_t.numpy(),
                lam=np.float64(lam), sigma_rgb=np.float64(sigma_rgb),
                total=np.float64(float(total.detach().sum())), grad=f.grad.numpy())


def main():
    if not (crf_ref.ref_available("xy") and crf_ref.ref_available("color")):
        raise SystemExit("build oracle/_ref first: make -C oracle")
    torch.set_num_threads(8)
    mods = _install()
    which = sys.argv[1:] or ["losses", "rgb"]
    cases = {"a": (2, 64, 64, 1, 1.0, False), "b": (3, 40, 56, 2, 1.7, True),
             "c": (1, 224, 224, 3, 10.0, False)}
    out = {}
    if "losses" in which:
        for name, (n, h, w, seed, t, empty) in cases.items():
            for k, v in make_case(mods, n, h, w, seed, t, empty).items():
                out[f"{name}_{k}"] = v
        np.savez_compressed(os.path.join(HERE, "tcam_losses.npz"), **out)
        print("wrote tcam_losses.npz", sorted(cases))
    if "rgb" not in which:
        return
    rgb = {}
    for name, (seq, frm, h, w, seed) in RGB_CASES.items():
        for k, v in make_rgb_case(mods, seq, frm, h, w, seed).items():
            rgb[f"{name}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "rgb_joint_crf.npz"), **rgb)
    print("wrote rgb_joint_crf.npz", sorted(RGB_CASES))


if __name__ == "__main__":
    main()
