"""CPU: the seeder oracle (oracle/seed_ref.py) against golden vectors produced by
the reference TCAMSeeder (tests/golden/make_seed_golden.py), and the Gumbel-top-k
draw against torch.multinomial's distribution."""
import ast
import os

import numpy as np
import pytest
import torch

from oracle import seed_ref as SR

GOLD = os.path.join(os.path.dirname(__file__), "golden", "tcam_seeder.npz")


def _cases():
    z = np.load(GOLD)
    names = sorted({k.split("/")[0] for k in z.files})
    return z, names


@pytest.mark.parametrize("name", _cases()[1])
def test_oracle_matches_reference_seeder(name):
    z, _ = _cases()
    cfg = dict(ast.literal_eval(str(z[f"{name}/cfg"])))
    cams = z[f"{name}/cams"]
    roi = z[f"{name}/roi"].astype(np.int64) if f"{name}/roi" in z.files else None
    out = SR.seeder(cams, cfg, roi=roi, seed=3, offset=0)
    np.testing.assert_array_equal(out, z[f"{name}/seeds"].astype(np.int64))
    b = cams.shape[0]
    for i in range(b):
        c = cams[i, 0]
        if c.min() == c.max():
            continue
        assert SR.otsu_threshold(c) == z[f"{name}/otsu_{i}"]
        for m in (SR.ROI_ALL, SR.ROI_LARGEST, SR.ROI_H_DENSITY):
            r, _, _ = SR.get_roi(c, m, cfg["p_min_area_roi"])
            np.testing.assert_array_equal(r, z[f"{name}/roi_{m}"][i])


def test_otsu_known_answer():
    # two-level image: the threshold separates the levels (skimage semantics:
    # the returned centre is the last bin of the lower class).
    cam = np.zeros((10, 10), np.float32)
    cam[:, 5:] = 200.0 / 255.0
    th = SR.otsu_threshold(cam)
    assert 0.0 <= th < 199.0
    assert ((cam * np.float32(255.0) >= th) == (cam > 0)).all()
    # flat image -> 0
    assert SR.otsu_threshold(np.full((4, 4), 0.3, np.float32)) == 0.0


def test_morphology_geodesic():
    x = np.zeros((5, 6), np.int64)
    x[0, 0] = 1
    d = SR.dilate(x, 3)
    assert d[:2, :2].all() and d.sum() == 4          # border pixels ignored, not padded
    e = SR.erode(np.ones((5, 6), np.int64), 3, 1)
    assert e.all()                                    # geodesic: the border does not erode
    d4 = SR.dilate(x, 4)                              # even kernel: origin (2, 2),
    assert d4[:3, :3].all() and d4.sum() == 9         # window rows i-2 .. i+1


def test_philox_known_answer():
    # Random123 kat_vectors: philox4x32 10 rounds, ctr=0, key=0
    out = SR.philox4x32(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in out] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    out = SR.philox4x32(0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff,
                        0xffffffff, 0xffffffff)
    assert [int(v) for v in out] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]


def test_gumbel_topk_matches_multinomial_distribution():
    """multinomial(p, k, replacement=False) == topk(p / Exp(1), k) in law:
    compare first-draw and pair frequencies against torch.multinomial."""
    p = np.array([0.05, 0.1, 0.15, 0.3, 0.4], np.float32)
    n, k, trials = p.size, 2, 40000
    rng = np.random.default_rng(0)
    q = rng.exponential(size=(trials, n))
    keys = p[None, :] / q
    ours = np.argsort(-keys, axis=1)[:, :k]
    g = torch.Generator().manual_seed(0)
    ref = torch.stack([torch.from_numpy(p).multinomial(k, replacement=False, generator=g)
                       for _ in range(trials)]).numpy()

    def pair_freq(s):
        f = np.zeros((n, n))
        np.add.at(f, (s[:, 0], s[:, 1]), 1)
        return f / len(s)

    a, b = pair_freq(ours), pair_freq(ref)
    # binomial std <= sqrt(.25/40000) = 2.5e-3; allow 5 sigma
    assert np.abs(a - b).max() < 0.0125, np.abs(a - b).max()
    # exact law of the first draw: p_i / sum p
    first = np.bincount(ours[:, 0], minlength=n) / trials
    assert np.abs(first - p / p.sum()).max() < 0.0125


def test_sampling_is_subset_of_candidates():
    rng = np.random.default_rng(1)
    cams = rng.random((2, 1, 20, 24)).astype(np.float32)
    cfg = SR.default_cfg(max_=5, min_=7, ksz=1)
    out = SR.seeder(cams, cfg, seed=11, offset=2)
    for i in range(2):
        assert (out[i] == 1).sum() == 5 and (out[i] == 0).sum() == 7
        full = SR.seeder(cams[i:i + 1], dict(cfg, max_=10 ** 9, min_=10 ** 9))
        assert (full[0][out[i] == 1] == 1).all()
        assert (full[0][out[i] == 0] == 0).all()


def test_roi_threshold_oracle_matches_reference_stotsu():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "roi_thresh.npz"))
    for cam, th, line in zip(z["cams"], z["th"], z["lines"]):
        t = SR.roi_threshold(cam)
        assert t == th
        assert str(float(t) / 255.) == str(line)


def test_camstore_host_format(tmp_path):
    """ROI file / id mapping helpers (no GPU): wsol_loader.py:183-188, 299-317."""
    from tcam_wsol_video_amd import camstore as CS
    assert CS.reformat_id("a/b\\c.jpg") == "a_b_c.jpg"
    p = tmp_path / "roi.txt"
    CS.write_roi_file(str(p), ["v/1", "v/2"], torch.tensor([78.0, 0.0]))
    assert p.read_text() == f"v/1,{78.0 / 255.}\nv/2,0.0\n"
    assert CS.load_roi_thresholds(str(p)) == {"v/1": 78.0 / 255., "v/2": 0.0}
    assert CS.load_roi_thresholds(str(tmp_path / "absent.txt")) is None
