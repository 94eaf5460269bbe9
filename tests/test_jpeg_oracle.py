"""CPU: the JPEG decode restatement (oracle/jpeg_ref.py) is bit-identical to Pillow itself
(the reference loader's Image.open(...).convert('RGB'), wsol_loader.py:581-582) over the
case matrix, and the C-ABI host packer (tcam_jpeg_pack, no device work) agrees with the
restatement's marker walk: dimensions, restart segmentation, refusal of progressive files."""
import ctypes as C

import numpy as np
import pytest

import jpeg_cases as JC
from oracle import jpeg_ref as J

CASES = JC.matrix(small=True)
CRAFTED = JC.crafted(small=True)


@pytest.mark.parametrize("name,data", CASES, ids=[c[0] for c in CASES])
def test_restatement_matches_pillow(name, data):
    np.testing.assert_array_equal(J.decode_rgb(data), J.pil_decode_rgb(data))


@pytest.mark.parametrize("name,data", CRAFTED, ids=[c[0] for c in CRAFTED])
def test_restatement_matches_pillow_crafted_sampling(name, data):
    """4:4:0 / 4:1:1 / h4v2 / h3v1 / mixed chroma factors (tests/jpeg_encode.py)."""
    np.testing.assert_array_equal(J.decode_rgb(data), J.pil_decode_rgb(data))


def test_restatement_refuses_progressive():
    with pytest.raises(J.Unsupported):
        J.parse(JC.progressive())


def _pack(datas, blob=None, cap=0):
    from tcam_wsol_video_amd import _lib
    lib = _lib.load()
    n = len(datas)
    ptrs = (C.c_char_p * n)(*datas)
    lens = (C.c_size_t * n)(*[len(d) for d in datas])
    sizes = np.zeros(4, np.int64)
    dims = np.zeros((n, 3), np.int32)
    rc = lib.tcam_jpeg_pack(C.cast(ptrs, C.c_void_p), C.cast(lens, C.c_void_p), n,
                            blob, cap, sizes.ctypes.data_as(C.c_void_p),
                            dims.ctypes.data_as(C.c_void_p))
    return rc, sizes, dims


def test_host_pack_sizes_and_dims():
    datas = [d for _, d in CASES]
    rc, sizes, dims = _pack(datas)
    assert rc == 0
    total_blocks = 0
    for k, d in enumerate(datas):
        P = J.parse(d)
        assert tuple(dims[k]) == (P.height, P.width, 0)
        hs, vs, hmax, vmax, mx, my = J.geometry(P)
        total_blocks += sum(mx * hs[c] * my * vs[c] for c in range(P.ncomp))
    assert sizes[3] == total_blocks
    assert sizes[2] == sum(int(d0) * int(d1) * 3 for d0, d1, _ in dims)
    buf = np.zeros(int(sizes[0]), np.uint8)
    rc2, sizes2, _ = _pack(datas, buf.ctypes.data_as(C.c_void_p), buf.nbytes)
    assert rc2 == 0 and (sizes2 == sizes).all()
    rc3, _, _ = _pack(datas, buf.ctypes.data_as(C.c_void_p), buf.nbytes - 16)
    assert rc3 == -2   # TCAM_E_NOMEM


def test_host_pack_restart_segments_and_unstuffing():
    """The packed entropy bytes equal the restatement's unstuffed restart segments."""
    d = dict(CASES)["rst_rows1_420"]
    P = J.parse(d)
    assert P.restart > 0 and len(P.segments) > 1
    rc, sizes, _ = _pack([d])
    buf = np.zeros(int(sizes[0]), np.uint8)
    assert _pack([d], buf.ctypes.data_as(C.c_void_p), buf.nbytes)[0] == 0
    hdr = buf[:128].view(np.int64)
    off_bytes = int(hdr[11])   # JHdr.off_bytes (csrc/jpeg.hip: 8 ints, total_pixels, 6 offsets)
    pos = off_bytes
    for seg in P.segments:
        assert bytes(buf[pos:pos + len(seg)]) == seg
        pos += (len(seg) + 15) // 16 * 16


def test_host_pack_refuses_unsupported():
    rc, _, dims = _pack([JC.progressive(), dict(CASES)["gray"], b"not a jpeg"])
    assert rc == -21   # TCAM_JPEG_E_UNSUPPORTED (first failing file)
    assert list(dims[:, 2]) == [-21, 0, -20]
    assert tuple(dims[1, :2]) == (33, 47)


def test_host_pack_survives_corrupt_files():
    """Random byte damage / truncation anywhere in the file: tcam_jpeg_pack returns 0 or a
    TCAM_JPEG_E_* code, never crashes (the header walk bounds every read)."""
    rng = np.random.default_rng(3)
    base = [d for _, d in CASES[::9]]
    seen = set()
    for it in range(400):
        d = bytearray(base[it % len(base)])
        kind = it % 3
        if kind == 0:        # random bytes
            for _ in range(int(rng.integers(1, 8))):
                d[int(rng.integers(0, len(d)))] = int(rng.integers(0, 256))
        elif kind == 1:      # truncation
            d = d[:int(rng.integers(2, len(d)))]
        else:                # damaged marker lengths
            for _ in range(3):
                p = int(rng.integers(2, min(len(d), 400)))
                d[p] = 0xFF
        rc, sizes, dims = _pack([bytes(d)])
        assert rc in (0, -20, -21, -22), rc
        seen.add(rc)
        if rc == 0:
            assert sizes[0] > 0 and dims[0, 2] == 0
    assert len(seen) >= 2
