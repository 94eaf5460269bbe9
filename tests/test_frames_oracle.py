"""CPU: the frame-transform oracle (oracle/frames_ref.py) against Pillow itself (the
reference's Resize is torchvision 0.12 TF.resize on a PIL image = Image.resize(BILINEAR)),
torch's ToTensor / Normalize arithmetic, and the library's host coefficient function."""
import ctypes as C

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import frames_ref as FR

SIZES = [(360, 480, 224, 224), (450, 360, 224, 224), (100, 150, 224, 224),
         (224, 224, 224, 224), (37, 53, 19, 71), (256, 256, 224, 224), (360, 480, 256, 256)]


@pytest.mark.parametrize("h,w,oh,ow", SIZES)
def test_oracle_resize_matches_pillow(h, w, oh, ow):
    rng = np.random.default_rng(h * 1000 + w)
    img = (rng.random((h, w, 3)) * 256).astype(np.uint8)
    ref = np.array(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    np.testing.assert_array_equal(FR.resize_bilinear(img, oh, ow), ref)


def test_oracle_normalize_matches_torch():
    rng = np.random.default_rng(1)
    u8 = (rng.random((31, 17, 3)) * 256).astype(np.uint8)
    t = torch.from_numpy(u8).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    t = t.sub_(torch.as_tensor(FR.MEAN)[:, None, None]).div_(torch.as_tensor(FR.STD)[:, None, None])
    np.testing.assert_array_equal(FR.to_tensor_normalize(u8), t.numpy())


@pytest.mark.parametrize("n_in,n_out", [(480, 224), (360, 224), (150, 224), (224, 224),
                                        (53, 71), (37, 19), (1, 5), (7, 1)])
def test_library_coeffs_match_oracle(n_in, n_out):
    from tcam_wsol_video_amd import frames
    b, k = frames.resample_coeffs(n_in, n_out)
    rb, rk = FR.resample_coeffs(n_in, n_out)
    np.testing.assert_array_equal(b, rb)
    np.testing.assert_array_equal(k, rk)


def test_transform_crop_flip_matches_pillow_chain():
    rng = np.random.default_rng(2)
    img = (rng.random((90, 120, 3)) * 256).astype(np.uint8)
    pil = Image.fromarray(img).resize((70, 70), Image.BILINEAR).crop((5, 3, 5 + 64, 3 + 64))
    pil = pil.transpose(Image.FLIP_LEFT_RIGHT)
    norm, raw = FR.transform(img, 70, 64, top=3, left=5, flip=True)
    np.testing.assert_array_equal(raw, np.array(pil, np.float32).transpose(2, 0, 1))
    np.testing.assert_array_equal(norm, FR.to_tensor_normalize(np.array(pil)))
