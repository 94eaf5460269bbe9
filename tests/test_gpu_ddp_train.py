"""The DDP path of the training step (flat-gradient all-reduce + BN-buffer broadcast +
1/world averaging in the SGD kernel), exercised with two processes on one GPU over
gloo.  Each rank trains on its OWN frames: the result must equal one process that computes
both ranks' gradients, averages them and applies rank 0's BN statistics."""
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


def _batch(rank=0):
    g = torch.Generator().manual_seed(3 + 17 * rank)
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
    x, raw, seeds = _batch(rank)
    tr.step(x.to(dev), raw.to(dev), seeds.to(dev))
    torch.cuda.synchronize()
    torch.save({"flat": tr.flat.cpu(), "bn": tr.bn_flat.cpu()}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_ddp_two_ranks_equal_single_process(cuda, tmp_path):
    from tcam_wsol_video_amd.models import build_r50_tcam
    from tcam_wsol_video_amd.training import DecoderTrainer, tcam_losses
    grads, bns = [], []
    for rank in range(2):
        tr = DecoderTrainer(build_r50_tcam(seed=8).to(cuda))
        x, raw, seeds = _batch(rank)
        _, fcams, st = tr.forward(x.to(cuda))
        _, dF = tcam_losses(fcams, raw.to(cuda), seeds.to(cuda), tr.lam, tr.elb.t, tr.sigma)
        tr.backward(dF, st)
        grads.append(tr.grad.clone())
        bns.append(tr.bn_flat)
    assert not torch.equal(grads[0], grads[1])
    from tcam_wsol_video_amd import _lib
    from tcam_wsol_video_amd._lib import check
    ref = DecoderTrainer(build_r50_tcam(seed=8).to(cuda))
    ref.grad.copy_(grads[0] + grads[1])
    ref.set_bn_flat(bns[0])
    check(_lib.load().tcam_sgd_step(ref.flat.data_ptr(), ref.grad.data_ptr(), ref.mom.data_ptr(),
                                    ref.flat.numel(), ref.lr, ref.momentum, ref.dampening,
                                    ref.weight_decay, 1 if ref.nesterov else 0, 1, 0.5,
                                    torch.cuda.current_stream().cuda_stream), "sgd")
    torch.cuda.synchronize()
    ref_flat, ref_bn = ref.flat.cpu(), ref.bn_flat.cpu()
    out = str(tmp_path / "r")
    mp.start_processes(_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        assert torch.equal(d["bn"], ref_bn), r
        # gloo sums in its own order: a + b is exact for two ranks
        assert torch.equal(d["flat"], ref_flat), r


def _amp_worker(rank, world, port, out):
    """--amp over two ranks: rank 1's scale (2^40) makes its scaled fp16 gradients overflow
    while rank 0's (2^10) do not; the found_inf flag rides in the gradient all-reduce, so
    rank 0 skips the step too and both back their scale off (torch DDP + GradScaler: the
    all-reduced inf reaches every rank's unscale_); the next clean step is applied on both."""
    import torch.distributed as dist
    from tcam_wsol_video_amd.models import build_r50_tcam
    from tcam_wsol_video_amd.training import DecoderTrainer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    tr = DecoderTrainer(build_r50_tcam(seed=8).to(dev), amp=True,
                        init_scale=2.0 ** (40 if rank else 10))
    w0 = tr.flat.clone()
    x, raw, seeds = _batch(rank)
    tr.step(x.to(dev), raw.to(dev), seeds.to(dev))
    torch.cuda.synchronize()
    res = {"unchanged": bool(torch.equal(tr.flat, w0)), "scale1": float(tr.scale.item()),
           "counts1": tr.step_counts.cpu()}
    tr.scale.fill_(2.0 ** 10)
    tr.step(x.to(dev), raw.to(dev), seeds.to(dev))
    torch.cuda.synchronize()
    res.update(counts2=tr.step_counts.cpu(), flat=tr.flat.cpu())
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_amp_ddp_found_inf_skips_on_every_rank(cuda, tmp_path):
    out = str(tmp_path / "a")
    mp.start_processes(_amp_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    d = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    for r in range(2):
        assert d[r]["unchanged"], r                       # the overflow step was skipped
        assert d[r]["scale1"] == 2.0 ** (39 if r else 9), r   # and the scales backed off
        assert d[r]["counts1"].tolist() == [0, 1], r
        assert d[r]["counts2"].tolist() == [1, 1], r      # the clean step applied
    assert torch.equal(d[0]["flat"], d[1]["flat"])        # the same averaged update


def _cl_batch(rank=0):
    g = torch.Generator().manual_seed(5 + 11 * rank)
    return torch.randn(2, 3, 64, 64, generator=g), torch.tensor([rank, 3 + rank])


def _cl_worker(rank, world, port, out):
    import torch.distributed as dist
    from tcam_wsol_video_amd.cl_training import ClassifierTrainer
    from tcam_wsol_video_amd.models import build_r50_stdcl
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    tr = ClassifierTrainer(build_r50_stdcl(seed=8).to(dev), lr=0.01)
    x, y = _cl_batch(rank)
    tr.step(x.to(dev), y.to(dev))
    torch.cuda.synchronize()
    torch.save({"flat": tr.flat.cpu(), "bn": tr.bn_flat.cpu()}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_stage1_ddp_two_ranks_equal_single_process(cuda, tmp_path):
    """Stage 1 (ClassifierTrainer) under DDP: each rank's own frames, the flat gradient
    all-reduced and averaged, rank 0's BN statistics broadcast, both SGD groups — equal to
    one process that sums the two ranks' gradients and steps with 1/2 (exact for two ranks)."""
    from tcam_wsol_video_amd.cl_training import ClassifierTrainer
    from tcam_wsol_video_amd.models import build_r50_stdcl
    grads, bns = [], []
    for rank in range(2):
        tr = ClassifierTrainer(build_r50_stdcl(seed=8).to(cuda), lr=0.01)
        x, y = _cl_batch(rank)
        logits, st = tr.forward(x.to(cuda))
        loss, dl = tr.loss_and_grad(logits, y.to(cuda))
        tr.backward(dl, st)
        grads.append(tr._gbuf.clone())
        grads[-1][-1] = loss
        bns.append(tr.bn_flat)
    assert not torch.equal(grads[0], grads[1])
    ref = ClassifierTrainer(build_r50_stdcl(seed=8).to(cuda), lr=0.01)
    ref._gbuf.copy_(grads[0] + grads[1])
    ref.set_bn_flat(bns[0])
    import torch.distributed as dist
    import tcam_wsol_video_amd.cl_training as CT
    assert not dist.is_initialized()
    # the DDP step on the summed gradient with a world of 2 (its all-reduce and broadcast
    # already applied above): the SGD kernels read the sum times 1/2
    real = CT.dist
    try:

        class _D:
            ReduceOp = real.ReduceOp

            @staticmethod
            def is_available():
                return True

            @staticmethod
            def is_initialized():
                return True

            @staticmethod
            def all_reduce(t, op=None):
                return None

            @staticmethod
            def broadcast(t, src=0):
                return None

            @staticmethod
            def get_world_size():
                return 2
        CT.dist = _D
        ref.all_reduce_and_step()
    finally:
        CT.dist = real
    torch.cuda.synchronize()
    ref_flat, ref_bn = ref.flat.cpu(), ref.bn_flat.cpu()
    out = str(tmp_path / "c")
    mp.start_processes(_cl_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        assert torch.equal(d["bn"], ref_bn), r
        assert torch.equal(d["flat"], ref_flat), r
