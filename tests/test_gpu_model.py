"""GPU parity of the full ResNet50-TCAM / STD_CL forward against the oracle and
the reference's own golden outputs (tests/golden, generated from
/root/reference by tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import bbox_ref as BR
from oracle import model_ref as R
from tcam_wsol_video_amd.inference import CAM, CAMComputer, SegmentationCam
from tcam_wsol_video_amd.models import build_r50_stdcl, build_r50_tcam
from tcam_wsol_video_amd.utils.seeding import seeded_state_dict, synthetic_clip

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")

# north_star: "CAMs match the reference PyTorch CPU path within 1e-4 fp32"
CAM_TOL = 1e-4


@pytest.fixture(scope="module", params=["x6", "f16x3", "fp32"])
def precision(request):
    return request.param


@pytest.fixture(scope="module")
def tcam(cuda, precision):
    d = np.load(os.path.join(G, "r50_tcam.npz"))
    m = build_r50_tcam(seed=int(d["seed"])).to(cuda)
    m.conv_precision = precision
    return m, d


def test_tcam_matches_reference_golden(cuda, tcam):
    model, d = tcam
    for size in (64, 224):
        x = torch.from_numpy(d[f"tcam_x{size}"]).to(cuda)
        with torch.no_grad():
            logits, fcams, _ = model(x)
        torch.cuda.synchronize()
        assert np.abs(logits.cpu().numpy() - d[f"tcam_logits{size}"]).max() < 1e-3
        assert np.abs(fcams.cpu().numpy() - d[f"tcam_fcams{size}"]).max() < 1e-3
        cam = model.cam.cpu().double().numpy()
        assert np.abs(cam - d[f"tcam_cam{size}"]).max() < CAM_TOL
        # SegmentationCam API (builtincam.py:187-225)
        ext = SegmentationCam(model)
        c0 = ext(argmax=False)
        assert c0.shape == ((224, 224) if size == 224 else (2, 64, 64))


def test_tcam_batch_matches_oracle(cuda, tcam):
    model, d = tcam
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    clip = synthetic_clip(4, seed=11, height=224, width=224)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    x = ((x - torch.tensor([0.485, .456, .406])[None, :, None, None]) /
         torch.tensor([.229, .224, .225])[None, :, None, None]).contiguous()
    with torch.no_grad():
        logits, fcams, _ = model(x.to(cuda))
    lo_ref, fc_ref, _ = R.tcam_forward(sd, x)
    cam_ref = R.cam_to_scoremap(R.segmentation_cam(fc_ref), (224, 224))
    assert np.abs(logits.cpu().numpy() - lo_ref.numpy()).max() < 1e-3
    cam = model.cam.cpu().double().numpy()
    assert np.abs(cam - cam_ref).max() < CAM_TOL
    # uint8 quantisation: identical except where the fp32 CAM straddles a
    # 1/255 boundary within the 1e-4 tolerance.
    u8_ref = R.quantize_u8(cam_ref)
    u8 = model.cam_u8.cpu().numpy()
    assert np.mean(u8 != u8_ref) < 1e-3
    assert np.abs(u8.astype(int) - u8_ref.astype(int)).max() <= 1


def test_stdcl_cam_matches_reference_golden(cuda, precision):
    d = np.load(os.path.join(G, "r50_stdcl.npz"))
    model = build_r50_stdcl(seed=int(d["seed"])).to(cuda)
    model.conv_precision = precision
    x = torch.from_numpy(d["std_x224"]).to(cuda)
    with torch.no_grad():
        logits = model(x)
    assert np.abs(logits.cpu().numpy() - d["std_logits224"]).max() < 1e-3
    ext = CAM(model, "encoder.layer4.2.relu3", "classification_head.fc")
    low = ext(class_idx=int(d["std_class"][0]))
    assert np.abs(low.cpu().numpy() - d["std_low224"][0]).max() < CAM_TOL
    cam = ext(class_idx=int(d["std_class"][0]), reshape=(224, 224))
    assert np.abs(cam.cpu().double().numpy() - d["std_cam224"][0]).max() < CAM_TOL


def test_end_to_end_eval_counters_bit_exact(cuda, tcam):
    """CAMComputer.evaluate_batch vs the oracle BoxEvaluator fed the same uint8
    CAMs (bit-exact), and vs the oracle's own CAMs (1e-4 CAM tolerance)."""
    model, _ = tcam
    clip = synthetic_clip(3, seed=5, height=224, width=224)
    x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
    x = ((x - torch.tensor([0.485, .456, .406])[None, :, None, None]) /
         torch.tensor([.229, .224, .225])[None, :, None, None]).contiguous()
    gt = torch.tensor([[[30, 40, 150, 170]], [[10, 10, 200, 120]], [[60, 60, 100, 100]]],
                      dtype=torch.int32)
    targets = torch.tensor([1, 4, 7])
    comp = CAMComputer(model, cam_curve_interval=0.001, device=cuda)
    u8 = comp.evaluate_batch(x.to(cuda), targets.to(cuda), gt.to(cuda)).cpu().numpy()
    acc = comp.compute_and_evaluate()
    ref = BR.BoxEvaluatorRef(comp.cam_threshold_list)
    lo = model(x.to(cuda))[0].cpu()
    for b in range(3):
        sm = np.minimum((u8[b].astype(np.float64) + 0.5) / 255.0, 1.0)
        _, order = torch.sort(lo[b], descending=True, stable=True)
        ref.accumulate(sm, gt[b].numpy(), int(targets[b]), order.numpy())
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(comp.evaluator.num_correct[thr], ref.num_correct[thr])
        np.testing.assert_array_equal(comp.evaluator.num_correct_top1[thr],
                                      ref.num_correct_top1[thr])
    assert acc == ref.compute()


def test_pipelined_forward_streams_match_single_stream(cuda, tcam):
    """fwd_streams>1 (clips in flight on round-robin streams, bench default 2) must give
    exactly the counters of the one-stream path over the same sequence of clips."""
    model, _ = tcam
    clips = []
    for k in range(5):
        clip = synthetic_clip(4, seed=20 + k, height=224, width=224)
        x = torch.from_numpy(clip).float().permute(0, 3, 1, 2) / 255.0
        x = ((x - 0.45) / 0.225).contiguous().to(cuda)
        gen = torch.Generator().manual_seed(k)
        lo = torch.randint(0, 100, (4, 1, 2), generator=gen)
        gt = torch.cat([lo, lo + torch.randint(20, 120, (4, 1, 2), generator=gen)], 2)
        clips.append((x, torch.randint(0, 10, (4,), generator=gen).to(cuda),
                      gt.to(torch.int32).to(cuda)))
    res = []
    for n in (1, 3):
        comp = CAMComputer(model, cam_curve_interval=0.01, device=cuda, fwd_streams=n)
        for x, t, g in clips:
            comp.evaluate_batch(x, t, g)
        comp.synchronize()
        res.append((comp.compute_and_evaluate(),
                    {thr: comp.evaluator.num_correct[thr].copy() for thr in (30, 50, 70)}))
    assert res[0][0] == res[1][0]
    for thr in (30, 50, 70):
        np.testing.assert_array_equal(res[0][1][thr], res[1][1][thr])
