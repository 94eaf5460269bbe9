"""The collectives of the hot path on the RCCL ("nccl") backend — every other multi-rank
test runs gloo.  One GPU box holds one device, and RCCL refuses two ranks on one device,
so this is a world-1 process group: the same all-reduce / all-gather / broadcast launches
as at N ranks, checked against the process-group-free run:

* the BoxEvaluator int32 counter all-reduce (wsol_metrics.py:372-388);
* the CAM all-gather of CAM-TMP (TemporalCAM, parallel/__init__.py:14-23);
* DecoderTrainer's flat-gradient (+ loss slot) all-reduce and BN-statistics broadcast
  (DDP, main.py:49).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _work(dev):
    from tcam_wsol_video_amd import _lib
    from tcam_wsol_video_amd import parallel as P
    from tcam_wsol_video_amd.inference import CAMComputer
    from tcam_wsol_video_amd.models import build_r50_tcam
    from tcam_wsol_video_amd.training import DecoderTrainer
    from tcam_wsol_video_amd.utils.seeding import synthetic_clip
    _lib.load().tcam_conv_x6_force_streamk(0)
    clip = synthetic_clip(8, seed=5, height=64, width=64)
    x = ((torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0 - 0.45) / 0.225)
    x = x.contiguous().to(dev)
    g = torch.Generator().manual_seed(2)
    tg = torch.randint(0, 10, (8,), generator=g).to(dev)
    lo = torch.randint(0, 30, (8, 1, 2), generator=g)
    gt = torch.cat([lo, lo + 20], 2).to(torch.int32).to(dev)
    model = build_r50_tcam(seed=6).to(dev)
    comp = CAMComputer(model, cam_curve_interval=0.01, device=dev, keep_fcams=True,
                       temporal=P.TemporalCAM(k=1, mode="before"))
    comp.evaluate_batch(x, tg, gt)
    acc = comp.compute_and_evaluate()
    out = {"acc": torch.tensor(acc), "tmp": comp.last_tmp_cam.cpu(),
           "nc": torch.from_numpy(np.stack([comp.evaluator.num_correct[t] for t in (30, 50, 70)]))}
    # one training step (gradient all-reduce + BN broadcast under a process group)
    tmodel = build_r50_tcam(seed=7).to(dev)
    tr = DecoderTrainer(tmodel)
    raw = (torch.rand(8, 3, 64, 64, generator=g) * 255).round().to(dev)
    seeds = torch.randint(-1, 2, (8, 64, 64), generator=g)
    seeds[seeds < 0] = -255
    tr.step(x, raw, seeds.to(dev))
    torch.cuda.synchronize()
    out["w"] = tr.flat.cpu()
    out["bn"] = tr.bn_flat.cpu()
    out["steps"] = torch.tensor([tr.applied_steps])
    _lib.load().tcam_conv_x6_force_streamk(-1)
    return out


def _worker(rank, port, path):
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ref = _work(dev)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    got = _work(dev)
    dist.barrier()
    dist.destroy_process_group()
    torch.save({"ref": ref, "got": got}, path)


def test_rccl_world1_collectives_equal_single_process(tmp_path):
    path = str(tmp_path / "r.pt")
    mp.start_processes(_worker, args=(_port(), path), nprocs=1, join=True,
                       start_method="spawn")
    d = torch.load(path, weights_only=True)
    ref, got = d["ref"], d["got"]
    for k in ("acc", "tmp", "nc", "w", "bn", "steps"):
        assert torch.equal(ref[k], got[k]), k
    assert int(got["steps"]) == 1
