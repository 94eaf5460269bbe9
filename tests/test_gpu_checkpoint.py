"""GPU: a DecoderTrainer saved as a reference-format training checkpoint
(utils_checkpoints.py:193-213) and resumed continues bit-identically."""
import pytest
import torch

from tcam_wsol_video_amd import checkpoints as CK
from tcam_wsol_video_amd.models import build_r50_tcam
from tcam_wsol_video_amd.training import DecoderTrainer

pytestmark = pytest.mark.gpu


def test_trainer_resume_is_exact(cuda, tmp_path):
    g = torch.Generator().manual_seed(0)
    x = [torch.randn(2, 3, 64, 64, generator=g).to(cuda) for _ in range(3)]
    raw = (torch.rand(2, 3, 64, 64, generator=g) * 255).round().to(cuda)
    seeds = torch.randint(-1, 2, (2, 64, 64), generator=g)
    seeds[seeds < 0] = -255
    seeds = seeds.to(cuda)
    a = DecoderTrainer(build_r50_tcam(seed=1).to(cuda))
    a.step(x[0], raw, seeds)
    a.elb.update_t()
    CK.save_checkpoint(a, str(tmp_path), 1)
    b = DecoderTrainer(build_r50_tcam(seed=2).to(cuda))
    assert CK.load_checkpoint(b, str(tmp_path)) == 1
    assert b.elb.t == pytest.approx(a.elb.t)
    for xi in x[1:]:
        la = a.step(xi, raw, seeds).cpu()
        lb = b.step(xi, raw, seeds).cpu()
        assert torch.equal(la, lb)
    assert torch.equal(a.flat.cpu(), b.flat.cpu())
    assert torch.equal(a.bn_flat.cpu(), b.bn_flat.cpu())
    assert torch.equal(a.mom.cpu(), b.mom.cpu())


def test_load_checkpoint_after_steps_refolds_encoder(cuda, tmp_path):
    """a trainer that already stepped (its frozen-encoder plan folded) and then
    loads a checkpoint whose ENCODER differs must continue exactly like a fresh trainer
    built from that checkpoint — the encoder plan is version-tracked."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 64, 64, generator=g).to(cuda)
    raw = (torch.rand(2, 3, 64, 64, generator=g) * 255).round().to(cuda)
    seeds = torch.randint(-1, 2, (2, 64, 64), generator=g)
    seeds[seeds < 0] = -255
    seeds = seeds.to(cuda)
    src = DecoderTrainer(build_r50_tcam(seed=11).to(cuda))
    src.step(x, raw, seeds)
    CK.save_checkpoint(src, str(tmp_path), 3)
    a = DecoderTrainer(build_r50_tcam(seed=12).to(cuda))
    a.step(x, raw, seeds)                      # folds seed-12's encoder
    assert CK.load_checkpoint(a, str(tmp_path)) == 3
    b = DecoderTrainer(build_r50_tcam(seed=13).to(cuda))
    assert CK.load_checkpoint(b, str(tmp_path)) == 3
    la, lb = a.step(x, raw, seeds).cpu(), b.step(x, raw, seeds).cpu()
    assert torch.equal(la, lb)
    assert torch.equal(a.flat.cpu(), b.flat.cpu())
