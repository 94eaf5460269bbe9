"""JPEG test files, encoded here by Pillow (libjpeg-turbo) -- the library whose decode the
reference loader calls (wsol_loader.py:581-582): every chroma subsampling, qualities 5-100,
odd and tiny sizes (fancy-upsampling edge rules), restart intervals, optimized Huffman
tables, grayscale, Adobe RGB, plus the progressive variant the device path must refuse."""
import io

import numpy as np
from PIL import Image


def frame(h, w, seed=0, mode="RGB"):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([x * 255 // max(w - 1, 1), y * 255 // max(h - 1, 1),
                     ((x + y) * 7) % 256], -1).astype(np.float64)
    base += rng.normal(0, 25, base.shape)
    im = Image.fromarray(np.clip(base, 0, 255).astype(np.uint8))
    return im.convert("L") if mode == "L" else im


def encode(im, **kw):
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def matrix(small=True):
    """[(name, bytes)] over the case matrix (small=True: sizes the CPU restatement finishes
    in seconds)."""
    sizes = [(16, 16), (24, 40), (37, 53), (8, 8), (5, 3), (3, 5), (1, 9), (9, 1), (2, 2),
             (4, 6), (17, 130)]
    if not small:
        sizes += [(240, 320), (360, 480), (299, 301), (720, 1280)]
    out = []
    for k, (h, w) in enumerate(sizes):
        for sub in (0, 1, 2):
            for q in (30, 75, 95):
                out.append((f"{h}x{w}_s{sub}_q{q}",
                            encode(frame(h, w, seed=k), quality=q, subsampling=sub)))
    out += [
        ("opt_420", encode(frame(40, 56, 1), quality=80, subsampling=2, optimize=True)),
        ("rst_blocks3", encode(frame(40, 56, 2), quality=80, restart_marker_blocks=3)),
        ("rst_rows1_420", encode(frame(41, 57, 3), quality=60, subsampling=2,
                                 restart_marker_rows=1)),
        ("gray", encode(frame(33, 47, 4, "L"), quality=90)),
        ("gray_rst", encode(frame(35, 49, 5, "L"), quality=70, restart_marker_blocks=2)),
        ("q5_420", encode(frame(120, 160, 6), quality=5, subsampling=2)),
        ("q100_444", encode(frame(120, 160, 7), quality=100, subsampling=0)),
        ("adobe_rgb", encode_adobe_rgb(frame(24, 24, 8))),
    ]
    return out


def encode_adobe_rgb(im):
    """An RGB-colour-space JPEG (Adobe APP14 transform 0, component ids R, G, B)."""
    return encode(im.convert("RGB"), quality=85, subsampling=0, keep_rgb=True)


def progressive(h=32, w=32):
    return encode(frame(h, w, 9), quality=75, progressive=True)


def crafted(small=True):
    """Files Pillow cannot write (tests/jpeg_encode.py): 4:4:0, 4:1:1, h4v2, h3v1, mixed
    chroma factors, restart intervals -- the h1v2 fancy and box-replication paths."""
    import jpeg_encode as JE
    sizes = [(37, 53), (9, 7)] + ([] if small else [(120, 161), (64, 64)])
    out = []
    for k, (h, w) in enumerate(sizes):
        rgb = np.asarray(frame(h, w, seed=60 + k))
        for name, smp in JE.SAMPLINGS.items():
            for rst in (0, 3):
                out.append((f"enc_{name}_{h}x{w}_r{rst}",
                            JE.encode(rgb, smp, quality=75, restart=rst)))
    return out
