"""GPU: device JPEG decode (csrc/jpeg.hip through tcam_jpeg_pack / tcam_jpeg_decode) is
bit-identical to the reference loader's Image.open(...).convert('RGB')
(wsol_loader.py:581-582, Pillow / libjpeg-turbo) over the whole case matrix in one ragged
batch, at frame sizes up to 720x1280, for same-size clips, for files with thousands of
restart segments (many Huffman workgroups), and end to end through the eval transform."""
import numpy as np
import pytest
import torch

import jpeg_cases as JC
from oracle import frames_ref as FR
from oracle import jpeg_ref as J
from tcam_wsol_video_amd import frames, jpeg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec(cuda):
    return jpeg.JpegDecoder(cuda)


def _check(out, datas, names):
    assert len(out) == len(datas)
    for o, d, n in zip(out, datas, names):
        ref = J.pil_decode_rgb(d)
        got = o.cpu().numpy()
        assert got.shape == ref.shape, n
        if not np.array_equal(got, ref):
            bad = np.argwhere(got != ref)
            raise AssertionError(f"{n}: {len(bad)} samples differ, first at {bad[0]}: "
                                 f"{got[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")


def test_case_matrix_one_ragged_batch(dec):
    cases = JC.matrix(small=False)
    names, datas = [c[0] for c in cases], [c[1] for c in cases]
    out = dec.decode(datas, names)
    torch.cuda.synchronize()
    _check(out, datas, names)


def test_crafted_sampling_layouts(dec):
    """4:4:0 (h1v2 fancy), 4:1:1 / h3v1 / h4v2 (box replication), mixed chroma factors,
    restart intervals -- files from tests/jpeg_encode.py, one ragged batch."""
    cases = JC.crafted(small=False)
    names, datas = [c[0] for c in cases], [c[1] for c in cases]
    _check(dec.decode(datas, names), datas, names)


def test_each_case_alone(dec):
    for name, d in JC.matrix(small=True)[::7]:
        _check(dec.decode([d], [name]), [d], [name])


def test_same_size_clip_batch(dec):
    datas = [JC.encode(JC.frame(240, 320, seed=100 + t), quality=90, subsampling=2)
             for t in range(32)]
    clip = dec.decode_batch(datas)
    assert clip.shape == (32, 240, 320, 3) and clip.dtype == torch.uint8
    ref = np.stack([J.pil_decode_rgb(d) for d in datas])
    np.testing.assert_array_equal(clip.cpu().numpy(), ref)


def test_many_restart_segments(dec):
    """restart every MCU: ~3600 segments -> ~57 Huffman workgroups for one file, plus a
    second file with other (optimized) tables in the same batch."""
    datas = [JC.encode(JC.frame(480, 640, 11), quality=85, subsampling=2,
                       restart_marker_blocks=1),
             JC.encode(JC.frame(64, 96, 12), quality=70, optimize=True,
                       restart_marker_rows=2)]
    P = J.parse(datas[0])
    assert len(P.segments) > 1000
    _check(dec.decode(datas), datas, ["rst1", "opt_rst"])


def test_decoder_reuse_and_growth(dec):
    small = [JC.encode(JC.frame(16, 16, 20), quality=50)]
    big = [JC.encode(JC.frame(360, 480, 21 + k), quality=95, subsampling=k % 3)
           for k in range(6)]
    a = dec.decode(small)
    b = dec.decode(big)
    c = dec.decode(small)
    _check(a, small, ["s0"])
    _check(b, big, [f"b{k}" for k in range(6)])
    _check(c, small, ["s1"])


def test_consecutive_decodes_on_different_streams(dec, cuda):
    """The decoder's device blob / workspace are shared across calls: decodes enqueued on
    alternating streams (big then small, so a late kernel would see overwritten inputs)
    must each match Pillow."""
    big = [JC.encode(JC.frame(480, 640, 30 + k), quality=95) for k in range(4)]
    small = [JC.encode(JC.frame(24, 40, 40 + k), quality=60) for k in range(4)]
    s1, s2 = torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)
    outs = []
    for r in range(3):
        for st, datas in ((s1, big), (s2, small)):
            with torch.cuda.stream(st):
                outs.append((dec.decode(datas), datas))
    torch.cuda.synchronize()
    for o, d in outs:
        _check(o, d, [f"f{k}" for k in range(len(d))])


def test_corrupt_entropy_data_does_not_fault(dec):
    """Bit flips in the entropy-coded data (headers intact, so the files pack): the decode
    must finish without a device fault (a garbage parse stays inside the coefficient
    buffer), and the decoder keeps working afterwards.  The pixels of a corrupt stream are
    not a parity target (libjpeg's recovery differs)."""
    rng = np.random.default_rng(5)
    good = [JC.encode(JC.frame(96, 128, 70 + k), quality=90, subsampling=k % 3,
                      **({"restart_marker_blocks": 2} if k % 2 else {})) for k in range(6)]
    bad = []
    for k in range(48):
        d = bytearray(good[k % len(good)])
        sos = d.index(b"\xff\xda")
        start = sos + 2 + int.from_bytes(d[sos + 2:sos + 4], "big")
        for _ in range(int(rng.integers(1, 6))):
            p = int(rng.integers(start, len(d) - 2))
            if d[p] != 0xFF and d[p - 1] != 0xFF:
                d[p] ^= 1 << int(rng.integers(0, 8))
                if d[p] == 0xFF:
                    d[p] = 0xFE
        bad.append(bytes(d))
    outs = dec.decode(bad)
    torch.cuda.synchronize()
    assert all(o.shape == (96, 128, 3) for o in outs)
    _check(dec.decode(good), good, [f"g{k}" for k in range(len(good))])


def test_empty_batch_bytearray_and_dims(dec):
    assert dec.decode([]) == []
    d = JC.encode(JC.frame(21, 34, 80), quality=70)
    assert jpeg.image_dims(d) == (21, 34)
    _check(dec.decode([bytearray(d), memoryview(d)]), [d, d], ["ba", "mv"])


def test_refuses_progressive_and_non_jpeg(dec):
    with pytest.raises(jpeg.UnsupportedJPEG, match="f1"):
        dec.decode([JC.encode(JC.frame(8, 8)), JC.progressive()], names=["f0", "f1"])
    with pytest.raises(jpeg.UnsupportedJPEG, match="not a JPEG"):
        dec.decode([b"\x89PNG...."])
    with pytest.raises(ValueError):
        jpeg.JpegDecoder("cpu")


def test_decode_then_eval_transform(dec):
    """files -> device decode -> get_eval_tranforms(224) == PIL decode -> Pillow resize ->
    ToTensor/Normalize (the reference loader's __getitem__ image path)."""
    datas = [JC.encode(JC.frame(240, 320, seed=200 + t), quality=92, subsampling=2)
             for t in range(8)]
    clip = dec.decode_batch(datas)
    norm, raw = frames.get_eval_tranforms(224)(clip)
    for t, d in enumerate(datas):
        n_ref, r_ref = FR.transform(J.pil_decode_rgb(d), 224, 224)
        np.testing.assert_array_equal(raw[t].cpu().numpy(), r_ref)
        np.testing.assert_array_equal(norm[t].cpu().numpy(), n_ref)
