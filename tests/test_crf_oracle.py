"""CPU: pin the CRF oracles.  The numpy restatement (oracle/crf_ref.port_bilateral)
must reproduce the reference filters bit for bit: against the golden vectors the
reference produced (tests/golden/make_crf_golden.py) and, when oracle/_ref is
built, against the compiled reference on fresh random inputs."""
import os

import numpy as np
import pytest

from oracle import crf_ref as R

G = os.path.join(os.path.dirname(__file__), "golden", "crf_bilateral.npz")


def _cases():
    d = np.load(G)
    names = sorted({k.split("_")[0] for k in d.files})
    return d, names


def test_port_matches_reference_golden_bitexact():
    d, names = _cases()
    assert len(names) >= 4
    for nm in names:
        n, k, h, w, sr, sx = d[f"{nm}_meta"]
        kind = str(d[f"{nm}_kind"])
        img, seg = d[f"{nm}_img"], d[f"{nm}_seg"]
        if kind == "xy":
            out = R.port_bilateral(img, seg, sr, sx)
        else:
            out = R.port_bilateral(img, seg, sr, dim=int(kind[-1]))
        assert np.array_equal(out, d[f"{nm}_out"]), nm


@pytest.mark.skipif(not R.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("shape,sr,sx", [((1, 2, 40, 33), 15.0, 100.0),
                                         ((2, 1, 17, 19), 3.0, 5.0),
                                         ((1, 2, 64, 48), 15.0, 100.0)])
def test_port_matches_compiled_reference(shape, sr, sx):
    rng = np.random.default_rng(sum(shape))
    n, k, h, w = shape
    img = (rng.random((n, 3, h, w)) * 255).astype(np.float32)
    seg = rng.random(shape).astype(np.float32)
    assert np.array_equal(R.port_bilateral(img, seg, sr, sx), R.ref_bilateral(img, seg, sr, sx))
    for dim in (1, 2, 3):
        assert np.array_equal(R.port_bilateral(img, seg, sr, dim=dim),
                              R.ref_colorbilateral(img, seg, sr, dim))


def test_port_filter_properties():
    # A constant signal stays (nearly) constant up to the lattice normalisation; a
    # linear combination of inputs filters linearly (splat/blur/slice are linear).
    rng = np.random.default_rng(3)
    img = (rng.random((1, 3, 12, 10)) * 255).astype(np.float32)
    a = rng.random((1, 1, 12, 10)).astype(np.float32)
    b = rng.random((1, 1, 12, 10)).astype(np.float32)
    fa = R.port_bilateral(img, a, 10.0, 5.0)
    fb = R.port_bilateral(img, b, 10.0, 5.0)
    fab = R.port_bilateral(img, np.concatenate([a, b], 1), 10.0, 5.0)
    assert np.array_equal(fab[:, :1], fa) and np.array_equal(fab[:, 1:], fb)
    f2 = R.port_bilateral(img, 2 * a, 10.0, 5.0)
    assert np.allclose(f2, 2 * fa, rtol=1e-6, atol=0)
