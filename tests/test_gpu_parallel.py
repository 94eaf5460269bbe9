"""GPU tests of CAM-TMP over a sharded clip (BASELINE configs[4]):

* ``tcam_temporal_cam`` vs the oracle's temporal max (wsol_loader.py:591-601,
  re_normalize_cam :630-635) and the eval quantisation (wsol_metrics.py:153);
* two ranks on one GPU (gloo; each rank its own frames of one clip) give exactly the
  temporal CAMs and BoxEvaluator counters of one process over the whole clip.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import model_ref as R
from tcam_wsol_video_amd import ops
from tcam_wsol_video_amd import parallel as P

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(28, 28), (299, 299), (57, 61)])
@pytest.mark.parametrize("mode,k", [("before", 1), ("after", 2), ("before-after", 1),
                                    ("instant", 0)])
@pytest.mark.parametrize("t", [0.0, 0.7])
def test_temporal_cam_matches_oracle(cuda, shape, mode, k, t):
    """Through the API (TemporalCAM at world 1): the CAMs are heated only when
    sl_tc_knn > 0 (wsol_loader.py:571, 594), so ("instant", 0, t > 0) must leave
    every CAM unchanged."""
    g = torch.Generator().manual_seed(shape[0] * 7 + k * 3 + len(mode))
    n = 7
    cams = torch.rand((n,) + shape, generator=g)
    idx = P.knn_window(n, k, mode)
    out, u8 = P.TemporalCAM(k, mode, t)(cams.to(cuda))
    out, u8 = out.cpu(), u8.cpu().numpy()
    if k == 0:
        assert torch.equal(out, cams)
    for i in range(n):
        ref = R.temporal_max([cams[j] for j in idx[i] if j >= 0], t, sl_tc_knn=k)
        if t == 0 or k == 0:
            assert torch.equal(out[i], ref), i
            np.testing.assert_array_equal(u8[i], R.quantize_u8(ref.double().numpy()))
        else:   # device expf vs torch-CPU exp: <= 1 ulp-level differences
            np.testing.assert_allclose(out[i].numpy(), ref.numpy(), rtol=2e-6, atol=1e-7)
            d = np.abs(u8[i].astype(int) - R.quantize_u8(ref.double().numpy()).astype(int))
            assert d.max() <= 1 and np.mean(d) < 1e-3


@pytest.mark.parametrize("t", [0.0, 0.7])
def test_temporal_cam_kernel_heats_when_asked(cuda, t):
    """The kernel primitive itself (ops.temporal_cam) heats whenever t > 0."""
    g = torch.Generator().manual_seed(5)
    cams = torch.rand((5, 33, 40), generator=g)
    idx = P.knn_window(5, 1, "before")
    out, _ = ops.temporal_cam(cams.to(cuda), torch.from_numpy(idx).to(cuda), t)
    for i in range(5):
        ref = R.temporal_max([cams[j] for j in idx[i] if j >= 0], t, sl_tc_knn=1)
        np.testing.assert_allclose(out[i].cpu().numpy(), ref.numpy(), rtol=2e-6, atol=1e-7)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CLIP, SIZE = 8, 64


def _clip():
    from tcam_wsol_video_amd.utils.seeding import synthetic_clip
    clip = synthetic_clip(CLIP, seed=31, height=SIZE, width=SIZE)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    x = ((x - 0.45) / 0.225).contiguous()
    gen = torch.Generator().manual_seed(4)
    lo = torch.randint(0, 30, (CLIP, 1, 2), generator=gen)
    gt = torch.cat([lo, lo + torch.randint(8, 30, (CLIP, 1, 2), generator=gen)], 2)
    return x, torch.randint(0, 10, (CLIP,), generator=gen), gt.to(torch.int32)


def _run(dev, rank, world):
    from tcam_wsol_video_amd import _lib
    from tcam_wsol_video_amd.inference import CAMComputer
    from tcam_wsol_video_amd.models import build_r50_tcam
    # batch-invariant conv schedule (no stream-K, no fill-dependent tile choice): a rank's
    # 4 frames then give bit for bit what the same frames give inside the 8-frame batch
    _lib.load().tcam_conv_x6_force_streamk(0)
    model = build_r50_tcam(seed=12).to(dev)
    x, t, gt = _clip()
    per = CLIP // world
    sl = slice(rank * per, (rank + 1) * per)
    comp = CAMComputer(model, cam_curve_interval=0.01, device=dev, keep_fcams=True,
                       temporal=P.TemporalCAM(k=1, mode="before-after"))
    u8 = comp.evaluate_batch(x[sl].to(dev), t[sl].to(dev), gt[sl].to(dev))
    comp.synchronize()
    acc = comp.compute_and_evaluate()
    cams = model.cam.cpu()
    _lib.load().tcam_conv_x6_force_streamk(-1)
    return (u8.cpu(), comp.last_tmp_cam.cpu(), cams, acc,
            {thr: comp.evaluator.num_correct[thr].copy() for thr in (30, 50, 70)})


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u8, tmp, _, acc, nc = _run(torch.device("cuda:0"), rank, world)
    torch.save({"u8": u8, "tmp": tmp, "acc": torch.tensor(acc),
                "nc": {k: torch.from_numpy(v) for k, v in nc.items()}}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_two_ranks_temporal_eval_equals_single_process(cuda, tmp_path):
    u8, tmp, cams, acc, nc = _run(cuda, 0, 1)
    # the single-process temporal CAM is the oracle's max over the window
    win = P.knn_window(CLIP, 1, "before-after")
    for i in range(CLIP):
        ref = R.temporal_max([cams[j] for j in win[i] if j >= 0], sl_tc_knn=1)
        assert torch.equal(tmp[i], ref), i
    out = str(tmp_path / "r")
    mp.start_processes(_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    parts = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    assert torch.equal(torch.cat([p["u8"] for p in parts]), u8)
    assert torch.equal(torch.cat([p["tmp"] for p in parts]), tmp)
    for p in parts:
        assert p["acc"].tolist() == list(acc)
        for thr in (30, 50, 70):
            np.testing.assert_array_equal(p["nc"][thr].numpy(), nc[thr])
