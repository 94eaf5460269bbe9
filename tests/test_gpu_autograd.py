"""The reference training loop drives the model directly (SURVEY.md §8b B1,
train_wsol.py:1162-1184): ``model.train(); loss = MasterLoss(...)(fcams=model(x)[1], ...);
loss.backward(); optimizer.step()`` — here through UnetTCAM's train-mode autograd forward
(training._TrainForward) and losses.MasterLoss.  It must give exactly DecoderTrainer's
gradients, and DDP (torch's DistributedDataParallel, what MyDDP wraps,
parallel/my_ddp.py:13-16) must average them across ranks fed DIFFERENT frames."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tcam_wsol_video_amd import losses as L
from tcam_wsol_video_amd.models import build_r50_tcam, build_vgg16_tcam
from tcam_wsol_video_amd.training import DecoderTrainer, tcam_losses

pytestmark = pytest.mark.gpu


def _batch(n, size, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, size, size, generator=g)
    raw = (torch.rand(n, 3, size, size, generator=g) * 255).round()
    seeds = torch.randint(-1, 2, (n, size, size), generator=g)
    seeds[seeds < 0] = -255
    return x, raw, seeds


def _master_loss(t=1.0):
    """instantiators.py:143-245 with the README's TCAM settings."""
    ml = L.MasterLoss(cuda_id=0)
    elb = L.ELB(init_t=1., max_t=10., mulcoef=1.01)
    ml.add(L.ConRanFieldTcams(cuda_id=0, lambda_=2e-9, sigma_rgb=15., sigma_xy=100.,
                              scale_factor=1.))
    size = L.MaxSizePositiveTcams(cuda_id=0, lambda_=0.01, elb=elb)
    size.set_t(float(t))
    ml.add(size)
    ml.add(L.SelfLearningTcams(cuda_id=0, lambda_=1., seg_ignore_idx=-255))
    return ml


def _trainer_grads(model, x, raw, seeds):
    tr = DecoderTrainer(model)
    _, fcams, st = tr.forward(x)
    losses, dF = tcam_losses(fcams, raw, seeds, tr.lam, tr.elb.t, tr.sigma)
    tr.backward(dF, st)
    torch.cuda.synchronize()
    named = dict(model.named_parameters())
    return losses, {k: tr.g(named[k]).clone() for k in named if named[k].requires_grad}, tr


@pytest.mark.parametrize("build", [build_r50_tcam, build_vgg16_tcam])
def test_reference_loop_matches_decoder_trainer(cuda, build):
    x, raw, seeds = _batch(2, 64, 3)
    x, raw, seeds = x.to(cuda), raw.to(cuda), seeds.to(cuda)
    ref_model = build(seed=31).to(cuda)
    ref_losses, ref_grads, tr = _trainer_grads(ref_model, x, raw, seeds)

    model = build(seed=31).to(cuda)
    model.train()
    assert model.assert_cl_is_frozen()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, lr=0.01, momentum=0.9, dampening=0., weight_decay=1e-4,
                          nesterov=True)
    ml = _master_loss()
    opt.zero_grad()
    cl_logits, fcams, im_recon = model(x)
    assert im_recon is None and fcams.requires_grad and not cl_logits.requires_grad
    loss = ml(epoch=0, fcams=fcams, raw_img=raw, seeds=seeds, cl_logits=cl_logits)
    assert torch.equal(loss.detach(), ref_losses[:1])
    assert [float(v) for v in ml.l_holder[1:]] == [float(ref_losses[2]), float(ref_losses[3]),
                                                   float(ref_losses[1])]
    loss.backward()
    for k, p in model.named_parameters():
        if p.requires_grad:
            assert torch.equal(p.grad, ref_grads[k]), k
    # BN running statistics and counters as nn.BatchNorm2d in train mode
    sd, rsd = model.state_dict(), ref_model.state_dict()
    for k in sd:
        if k.startswith("decoder.") and "running_" in k:
            assert torch.equal(sd[k], rsd[k]), k
        if k.startswith("decoder.") and k.endswith("num_batches_tracked"):
            assert int(sd[k]) == 1, k
    # optimizer step: torch's SGD vs the trainer's SGD kernel (same formula)
    opt.step()
    tr.all_reduce_and_step()
    named = dict(ref_model.named_parameters())
    for k, p in model.named_parameters():
        if p.requires_grad:
            ref = named[k].detach()
            assert (p.detach() - ref).abs().max().item() <= 1e-6 * max(1.0, ref.abs().max().item())
    # the next forward re-packs the stepped weights
    with torch.no_grad():
        _, f2, _ = model(x)
    _, f2_ref, _ = tr.forward(x)
    assert (f2 - f2_ref).abs().max().item() <= 1e-4 * f2_ref.abs().max().item()
    # eval after training: the fused inference plan (folded BN with the updated running
    # statistics) sees the trained decoder — CAM vs the oracle over the trained weights
    from oracle import model_ref as R
    model.eval()
    with torch.no_grad():
        lo, fe, _ = model(x)
    sd_trained = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    lo_ref, fc_ref, _ = R.tcam_forward(sd_trained, x.cpu())
    assert (lo.cpu() - lo_ref).abs().max().item() < 1e-3
    cam_ref = R.segmentation_cam(fc_ref)
    assert (model.cam.cpu() - cam_ref).abs().max().item() < 1e-4


def test_single_term_elementary_loss(cuda):
    x, raw, seeds = _batch(2, 64, 4)
    model = build_r50_tcam(seed=2).to(cuda).train()
    _, fcams, _ = model(x.to(cuda))
    sl = L.SelfLearningTcams(cuda_id=0, lambda_=1.)
    v = sl(epoch=0, fcams=fcams, seeds=seeds.to(cuda))
    ref = torch.nn.functional.cross_entropy(fcams.detach(), seeds.to(cuda).long(),
                                            ignore_index=-255)
    assert abs(float(v) - float(ref)) <= 1e-5 * abs(float(ref))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    model = build_r50_tcam(seed=40).to(dev).train()
    ddp = DDP(model, device_ids=None)      # MyDDP(model) is this plus attribute passthrough
    x, raw, seeds = _batch(2, 64, 100 + rank)  # each rank its own frames
    _, fcams, _ = ddp(x.to(dev))
    loss = _master_loss()(epoch=0, fcams=fcams, raw_img=raw.to(dev), seeds=seeds.to(dev))
    loss.backward()
    torch.cuda.synchronize()
    torch.save({k: p.grad.cpu() for k, p in model.named_parameters() if p.requires_grad},
               f"{out}.{rank}")
    dist.destroy_process_group()


def test_ddp_averages_gradients_of_different_frames(cuda, tmp_path):
    grads = []
    for rank in range(2):
        model = build_r50_tcam(seed=40).to(cuda)
        x, raw, seeds = _batch(2, 64, 100 + rank)
        _, g, _ = _trainer_grads(model, x.to(cuda), raw.to(cuda), seeds.to(cuda))
        grads.append(g)
    out = str(tmp_path / "g")
    mp.start_processes(_ddp_worker, args=(2, _port(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    for k in got[0]:
        assert torch.equal(got[0][k], got[1][k]), k
        ref = ((grads[0][k] + grads[1][k]) / 2).cpu()
        assert (got[0][k] - ref).abs().max().item() <= 1e-6 * max(1e-6, ref.abs().max().item()), k
        # the two ranks really saw different frames
    assert any(not torch.equal(grads[0][k], grads[1][k]) for k in grads[0])
