"""Diagnostic: train-step gradient error vs the fp64 oracle over several input seeds
(tells a ReLU-kink flip, which is seed-dependent, from a systematic kernel error)."""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import test_gpu_train as G
from oracle import train_ref as T
from tcam_wsol_video_amd.models import build_r50_tcam
from tcam_wsol_video_amd.training import DecoderTrainer
cuda = torch.device("cuda:0")
for ms, xs in [(21, 5), (21, 6), (22, 7), (23, 8), (24, 9)]:
    model = build_r50_tcam(seed=ms)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(cuda)
    x, raw, seeds = G._batch(2, 64, seed=xs)
    _, grads, _, _ = T.train_step(sd, x, raw, seeds)
    _, g32, _, _ = T.train_step(sd, x, raw, seeds, dtype=torch.float32)
    tr = DecoderTrainer(model)
    tr.step(x.to(cuda), raw.to(cuda), seeds.to(cuda))
    torch.cuda.synchronize()
    named = dict(model.named_parameters())
    e = max(G._rel(tr.g(named[k]), g) for k, g in grads.items())
    c = max(G._rel(g32[k], g) for k, g in grads.items())
    print(f"nolw={os.environ.get('TCAM_X6_NOLW','0')} seeds ({ms},{xs}): ours {e:.2e} torch-fp32 {c:.2e}", flush=True)
