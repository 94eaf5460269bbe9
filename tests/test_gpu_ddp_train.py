"""The DDP path of the training step (flat-gradient all-reduce + BN-buffer broadcast +
1/world averaging in the SGD kernel), exercised with two processes on one GPU over
gloo: identical batches on both ranks must give exactly the single-process step."""
import os
import socket

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


def _batch():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 64, 64, generator=g)
    raw = (torch.rand(2, 3, 64, 64, generator=g) * 255).round()
    seeds = torch.randint(-1, 2, (2, 64, 64), generator=g)
    seeds[seeds < 0] = -255
    return x, raw, seeds


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from tcam_wsol_video_amd.models import build_r50_tcam
    from tcam_wsol_video_amd.training import DecoderTrainer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    model = build_r50_tcam(seed=8).to(dev)
    tr = DecoderTrainer(model)
    x, raw, seeds = _batch()
    tr.step(x.to(dev), raw.to(dev), seeds.to(dev))
    torch.cuda.synchronize()
    torch.save({"flat": tr.flat.cpu(), "bn": tr.bn_flat.cpu()}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_ddp_two_ranks_equal_single_process(cuda, tmp_path):
    from tcam_wsol_video_amd.models import build_r50_tcam
    from tcam_wsol_video_amd.training import DecoderTrainer
    model = build_r50_tcam(seed=8).to(cuda)
    tr = DecoderTrainer(model)
    x, raw, seeds = _batch()
    tr.step(x.to(cuda), raw.to(cuda), seeds.to(cuda))
    ref_flat, ref_bn = tr.flat.cpu(), tr.bn_flat.cpu()
    out = str(tmp_path / "r")
    mp.start_processes(_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        assert torch.equal(d["flat"], ref_flat), r
        assert torch.equal(d["bn"], ref_bn), r
