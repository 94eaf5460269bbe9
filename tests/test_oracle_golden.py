"""CPU: pin the torch-CPU oracle (oracle/model_ref.py) against golden vectors
produced by the reference's own modules (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import model_ref as R
from tcam_wsol_video_amd.models import build_r50_stdcl, build_r50_tcam
from tcam_wsol_video_amd.utils.seeding import seeded_state_dict

G = os.path.join(os.path.dirname(__file__), "golden")


def test_tcam_state_dict_names_match_reference():
    d = np.load(os.path.join(G, "r50_tcam.npz"))
    m = build_r50_tcam()
    sd = m.state_dict()
    assert list(sd.keys()) == list(d["tcam_keys"])
    shapes = [",".join(map(str, v.shape)) for v in sd.values()]
    assert shapes == list(d["tcam_shapes"])


def test_stdcl_state_dict_names_match_reference():
    d = np.load(os.path.join(G, "r50_stdcl.npz"))
    assert list(build_r50_stdcl().state_dict().keys()) == list(d["std_keys"])


def test_oracle_tcam_matches_reference_golden():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    d = np.load(os.path.join(G, "r50_tcam.npz"))
    sd = seeded_state_dict(build_r50_tcam(), int(d["seed"]))
    for size in (64, 224):
        x = torch.from_numpy(d[f"tcam_x{size}"])
        lo, fc, _ = R.tcam_forward(sd, x)
        cam = R.cam_to_scoremap(R.segmentation_cam(fc), x.shape[2:])
        np.testing.assert_allclose(lo.numpy(), d[f"tcam_logits{size}"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(fc.numpy(), d[f"tcam_fcams{size}"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(cam, d[f"tcam_cam{size}"], atol=1e-5, rtol=0)


def test_oracle_stdcl_cam_matches_reference_golden():
    d = np.load(os.path.join(G, "r50_stdcl.npz"))
    sd = seeded_state_dict(build_r50_stdcl(), int(d["seed"]))
    x = torch.from_numpy(d["std_x224"])
    lo, A = R.stdcl_forward(sd, x)
    low, cam = R.std_cam(sd, A, int(d["std_class"][0]), (224, 224))
    np.testing.assert_allclose(lo.numpy(), d["std_logits224"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(low.numpy(), d["std_low224"][0], atol=1e-5, rtol=0)
    np.testing.assert_allclose(cam, d["std_cam224"][0], atol=1e-5, rtol=0)


def test_temporal_max_oracle():
    # datasets/wsol_loader.py:591-601, 630-635
    g = torch.Generator().manual_seed(0)
    cams = [torch.rand(1, 28, 28, generator=g) for _ in range(3)]
    out = R.temporal_max(cams, t=0.0)
    assert torch.equal(out, torch.maximum(torch.maximum(cams[0], cams[1]), cams[2]))
    out = R.temporal_max(cams, t=2.0)
    e = [torch.exp((c + 1e-6) * 2.0) for c in cams]
    e = [x / x.max() for x in e]
    assert torch.allclose(out, torch.maximum(torch.maximum(e[0], e[1]), e[2]))
    # sl_tc_knn == 0: the loader never heats (``_is_tmp``, wsol_loader.py:571, 594)
    assert torch.equal(R.temporal_max(cams[:1], t=2.0, sl_tc_knn=0), cams[0])


def _family(name):
    from tcam_wsol_video_amd.models import build_inceptionv3_tcam, build_vgg16_tcam
    return {"vgg16": build_vgg16_tcam, "inceptionv3": build_inceptionv3_tcam}[name]


@pytest.mark.parametrize("name", ["vgg16", "inceptionv3"])
def test_family_state_dict_names_match_reference(name):
    d = np.load(os.path.join(G, f"{name}_tcam.npz"))
    sd = _family(name)().state_dict()
    assert list(sd.keys()) == list(d["keys"])
    assert [",".join(map(str, v.shape)) for v in sd.values()] == list(d["shapes"])


@pytest.mark.parametrize("name,small,big", [("vgg16", 64, 224), ("inceptionv3", 96, 299)])
def test_oracle_family_matches_reference_golden(name, small, big):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    d = np.load(os.path.join(G, f"{name}_tcam.npz"))
    # the weights as LOADED (the state_dict repeats shared modules — VGG full_features,
    # Inception features — and the last repeat wins on load, as in the reference)
    sd = _family(name)(seed=int(d["seed"])).state_dict()
    for size in (small, big):
        x = torch.from_numpy(d[f"x{size}"])
        lo, fc, _ = R.tcam_forward(sd, x)
        cam = R.cam_to_scoremap(R.segmentation_cam(fc), x.shape[2:])
        np.testing.assert_allclose(lo.numpy(), d[f"logits{size}"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(cam, d[f"cam{size}"], atol=1e-5, rtol=0)
        if f"fcams{size}" in d.files:
            np.testing.assert_allclose(fc.numpy(), d[f"fcams{size}"], atol=1e-4, rtol=0)
