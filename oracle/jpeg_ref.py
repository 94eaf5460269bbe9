"""CPU restatement of the reference's frame decode (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker, never by the product path).

The reference decodes frames with ``Image.open(path).convert('RGB')``
(datasets/wsol_loader.py:581-582), i.e. Pillow 12.2 over libjpeg-turbo (the
third-party dependency; not in /root/reference) with its defaults: JDCT_ISLOW, fancy
upsampling, YCbCr -> RGB by jdcolor.c's fixed-point tables.  This module restates the
published libjpeg algorithm for baseline (SOF0/SOF1, Huffman, 8-bit) JPEGs:

* ``parse``            marker walk + byte unstuffing + restart segmentation (jdmarker.c)
* ``huffman_decode``   jdhuff.c decode_mcu (lookahead-free canonical decode, HUFF_EXTEND,
                       DC prediction reset per restart interval)
* ``idct_islow``       jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2, the
                       IDCT range-limit table of jdmaster.c prepare_range_limit_table)
* ``upsample``         jdsample.c h2v1 / h1v2 / h2v2 fancy upsampling (triangle filter,
                       context rows replicated at the component edges, jdmainct.c) and
                       box replication otherwise
* ``ycc_to_rgb``       jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)

Pinned: ``decode_rgb`` is checked bit-for-bit against Pillow itself (tests/test_jpeg_oracle.py)
over qualities, all chroma subsamplings, odd sizes, restart intervals, optimized Huffman
tables and grayscale.  ``pil_decode_rgb`` is the reference call itself.
"""
from __future__ import annotations

import io
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

# jpeg_natural_order (jutils.c): zigzag index -> natural (row-major) index
ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], np.int64)


def pil_decode_rgb(data: bytes) -> np.ndarray:
    """The reference's call (wsol_loader.py:581-582) on in-memory bytes."""
    from PIL import Image
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))


class Unsupported(ValueError):
    pass


@dataclass
class Parsed:
    width: int = 0
    height: int = 0
    comp_ids: List[int] = field(default_factory=list)
    hs: List[int] = field(default_factory=list)
    vs: List[int] = field(default_factory=list)
    tq: List[int] = field(default_factory=list)
    td: List[int] = field(default_factory=list)
    ta: List[int] = field(default_factory=list)
    quant: Dict[int, np.ndarray] = field(default_factory=dict)   # natural order
    dc: Dict[int, Tuple[List[int], List[int]]] = field(default_factory=dict)
    ac: Dict[int, Tuple[List[int], List[int]]] = field(default_factory=dict)
    restart: int = 0
    jfif: bool = False
    adobe: Optional[int] = None
    segments: List[bytes] = field(default_factory=list)      # unstuffed entropy bytes

    @property
    def ncomp(self):
        return len(self.comp_ids)

    @property
    def colorspace(self) -> str:
        """jdapimin.c default_decompress_parms."""
        if self.ncomp == 1:
            return "gray"
        if self.jfif:
            return "ycc"
        if self.adobe is not None:
            return "rgb" if self.adobe == 0 else "ycc"
        return "rgb" if self.comp_ids == [82, 71, 66] else "ycc"


def _u16(d, p):
    return (d[p] << 8) | d[p + 1]


def unstuff(d: bytes, p: int) -> Tuple[List[bytes], int]:
    """Entropy-coded data from p: drop 0xFF00 stuffing and fill bytes, split at RSTn.
    Returns (segments, position of the terminating marker's 0xFF)."""
    segs, cur = [], bytearray()
    n = len(d)
    while p < n:
        b = d[p]
        if b != 0xFF:
            cur.append(b)
            p += 1
            continue
        q = p + 1
        while q < n and d[q] == 0xFF:
            q += 1
        if q >= n:
            p = n
            break
        m = d[q]
        if m == 0x00:
            cur.append(0xFF)
            p = q + 1
        elif 0xD0 <= m <= 0xD7:
            segs.append(bytes(cur))
            cur = bytearray()
            p = q + 1
        else:
            break
    segs.append(bytes(cur))
    return segs, p


def parse(d: bytes) -> Parsed:
    """jdmarker.c read_markers for a baseline single-scan file."""
    if len(d) < 4 or d[0] != 0xFF or d[1] != 0xD8:
        raise Unsupported("not a JPEG (no SOI)")
    P = Parsed()
    p, n, seen_sof, seen_sos = 2, len(d), False, False
    while p < n:
        if d[p] != 0xFF:
            raise Unsupported(f"marker expected at {p}")
        while p < n and d[p] == 0xFF:
            p += 1
        m = d[p]
        p += 1
        if m == 0xD9:
            break
        if 0xD0 <= m <= 0xD7 or m == 0x01:
            continue
        L = _u16(d, p)
        seg = d[p + 2:p + L]
        if m in (0xC0, 0xC1):
            if seg[0] != 8:
                raise Unsupported("sample precision != 8")
            P.height, P.width, nc = _u16(seg, 1), _u16(seg, 3), seg[5]
            for i in range(nc):
                cid, hv, tq = seg[6 + 3 * i], seg[7 + 3 * i], seg[8 + 3 * i]
                P.comp_ids.append(cid)
                P.hs.append(hv >> 4)
                P.vs.append(hv & 15)
                P.tq.append(tq)
            seen_sof = True
        elif 0xC2 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            raise Unsupported(f"SOF{m - 0xC0} (progressive / lossless / arithmetic)")
        elif m == 0xC4:
            q = 0
            while q < len(seg):
                tc, th = seg[q] >> 4, seg[q] & 15
                bits = list(seg[q + 1:q + 17])
                nv = sum(bits)
                vals = list(seg[q + 17:q + 17 + nv])
                (P.ac if tc else P.dc)[th] = ([0] + bits, vals)
                q += 17 + nv
        elif m == 0xDB:
            q = 0
            while q < len(seg):
                pq, tq = seg[q] >> 4, seg[q] & 15
                if pq:
                    v = np.frombuffer(bytes(seg[q + 1:q + 129]), ">u2").astype(np.int64)
                    q += 129
                else:
                    v = np.frombuffer(bytes(seg[q + 1:q + 65]), np.uint8).astype(np.int64)
                    q += 65
                nat = np.zeros(64, np.int64)
                nat[ZIGZAG] = v
                P.quant[tq] = nat
        elif m == 0xDD:
            P.restart = _u16(seg, 0)
        elif m == 0xE0 and seg[:5] == b"JFIF\0":
            P.jfif = True
        elif m == 0xEE and seg[:5] == b"Adobe" and len(seg) >= 12:
            P.adobe = seg[11]
        elif m == 0xDA:
            if seen_sos:
                raise Unsupported("more than one scan")
            if not seen_sof:
                raise Unsupported("SOS before SOF")
            ns = seg[0]
            if ns != P.ncomp:
                raise Unsupported("non-interleaved multi-scan file")
            ids = [seg[1 + 2 * i] for i in range(ns)]
            if ids != P.comp_ids:
                raise Unsupported("scan component order differs from the frame's")
            P.td = [seg[2 + 2 * i] >> 4 for i in range(ns)]
            P.ta = [seg[2 + 2 * i] & 15 for i in range(ns)]
            ss, se, ahal = seg[1 + 2 * ns], seg[2 + 2 * ns], seg[3 + 2 * ns]
            if ss != 0 or se != 63 or ahal != 0:
                raise Unsupported("not a sequential scan")
            P.segments, p = unstuff(d, p + L)
            seen_sos = True
            continue
        p += L
    if not seen_sos:
        raise Unsupported("no scan")
    if P.ncomp not in (1, 3):
        raise Unsupported(f"{P.ncomp} components")
    return P


def derived_table(bits, vals):
    """jdhuff.c jpeg_make_d_derived_tbl: maxcode / valoffset (canonical codes)."""
    huffsize = [l for l in range(1, 17) for _ in range(bits[l])]
    huffcode, code, si, k = [], 0, huffsize[0] if huffsize else 0, 0
    while k < len(huffsize):
        while k < len(huffsize) and huffsize[k] == si:
            huffcode.append(code)
            code += 1
            k += 1
        code <<= 1
        si += 1
    maxcode, valoff, k = [-1] * 18, [0] * 18, 0
    for l in range(1, 17):
        if bits[l]:
            valoff[l] = k - huffcode[k]
            k += bits[l]
            maxcode[l] = huffcode[k - 1]
    maxcode[17] = 0xFFFFF
    return maxcode, valoff, vals


class BitReader:
    """jdhuff.c bit buffer over one unstuffed segment; zeros past its end (the decoder's
    behaviour after a marker)."""

    def __init__(self, data: bytes):
        self.v = int.from_bytes(data, "big") if data else 0
        self.n = 8 * len(data)
        self.pos = 0

    def bits(self, k: int) -> int:
        if k == 0:
            return 0
        end = self.pos + k
        if end <= self.n:
            r = (self.v >> (self.n - end)) & ((1 << k) - 1)
        else:
            have = max(0, self.n - self.pos)
            r = (self.v & ((1 << have) - 1)) << (k - have) if have else 0
        self.pos = end
        return r

    def huff(self, tbl) -> int:
        maxcode, valoff, vals = tbl
        l, code = 1, self.bits(1)
        while l <= 16 and code > maxcode[l]:
            code = (code << 1) | self.bits(1)
            l += 1
        if l > 16:
            return 0
        return vals[code + valoff[l]]


def _extend(r, s):
    return r - (1 << s) + 1 if r < (1 << (s - 1)) else r


def geometry(P: Parsed):
    if P.ncomp == 1:
        hs, vs, hmax, vmax = [1], [1], 1, 1
    else:
        hs, vs = P.hs, P.vs
        hmax, vmax = max(hs), max(vs)
    mx = -(-P.width // (8 * hmax))
    my = -(-P.height // (8 * vmax))
    return hs, vs, hmax, vmax, mx, my


def huffman_decode(P: Parsed) -> List[np.ndarray]:
    """Coefficient blocks per component, (bh, bw, 64) int16 in natural order (jdhuff.c)."""
    hs, vs, hmax, vmax, mx, my = geometry(P)
    dc = [derived_table(*P.dc[t]) for t in P.td]
    ac = [derived_table(*P.ac[t]) for t in P.ta]
    coef = [np.zeros((my * vs[c], mx * hs[c], 64), np.int16) for c in range(P.ncomp)]
    total = mx * my
    ri = P.restart if P.restart else total
    nseg = -(-total // ri)
    if len(P.segments) != nseg:
        raise Unsupported(f"{len(P.segments)} restart segments, expected {nseg}")
    for s, data in enumerate(P.segments):
        br = BitReader(data)
        pred = [0] * P.ncomp
        for m in range(s * ri, min(total, (s + 1) * ri)):
            y0, x0 = divmod(m, mx)
            for c in range(P.ncomp):
                for v in range(vs[c]):
                    for h in range(hs[c]):
                        blk = coef[c][y0 * vs[c] + v, x0 * hs[c] + h]
                        t = br.huff(dc[c])
                        diff = _extend(br.bits(t), t) if t else 0
                        pred[c] += diff
                        blk[0] = np.int16(((pred[c] + 32768) & 0xFFFF) - 32768)
                        k = 1
                        while k < 64:
                            rs = br.huff(ac[c])
                            r, t = rs >> 4, rs & 15
                            if t:
                                k += r
                                blk[ZIGZAG[min(k, 63)]] = _extend(br.bits(t), t)
                                k += 1
                            elif r == 15:
                                k += 16
                            else:
                                break
    return coef


CONST_BITS, PASS1_BITS = 13, 2
FIX = dict(f0298=2446, f0390=3196, f0541=4433, f0765=6270, f0899=7373, f1175=9633,
           f1501=12299, f1847=15137, f1961=16069, f2053=16819, f2562=20995, f3072=25172)


def _idct_1d(v, shift, rnd):
    """One islow butterfly over axis 0 of int64 array v (8, ...), jidctint.c."""
    f = FIX
    z2, z3 = v[2], v[6]
    z1 = (z2 + z3) * f["f0541"]
    tmp2 = z1 + z3 * (-f["f1847"])
    tmp3 = z1 + z2 * f["f0765"]
    tmp0 = (v[0] + v[4]) << CONST_BITS
    tmp1 = (v[0] - v[4]) << CONST_BITS
    t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    tmp0, tmp1, tmp2, tmp3 = v[7], v[5], v[3], v[1]
    z1, z2, z3, z4 = tmp0 + tmp3, tmp1 + tmp2, tmp0 + tmp2, tmp1 + tmp3
    z5 = (z3 + z4) * f["f1175"]
    tmp0 = tmp0 * f["f0298"]
    tmp1 = tmp1 * f["f2053"]
    tmp2 = tmp2 * f["f3072"]
    tmp3 = tmp3 * f["f1501"]
    z1 = z1 * (-f["f0899"])
    z2 = z2 * (-f["f2562"])
    z3 = z3 * (-f["f1961"]) + z5
    z4 = z4 * (-f["f0390"]) + z5
    tmp0 += z1 + z3
    tmp1 += z2 + z4
    tmp2 += z2 + z3
    tmp3 += z1 + z4
    out = [t10 + tmp3, t11 + tmp2, t12 + tmp1, t13 + tmp0,
           t13 - tmp0, t12 - tmp1, t11 - tmp2, t10 - tmp3]
    return np.stack([(o + rnd) >> shift for o in out])


def idct_range_limit(x: np.ndarray) -> np.ndarray:
    """jdmaster.c prepare_range_limit_table seen through IDCT_range_limit (& RANGE_MASK)."""
    i = x & 1023
    return np.where(i < 128, i + 128, np.where(i < 512, 255, np.where(i < 896, 0, i - 896)))


def idct_islow(coef: np.ndarray, q: np.ndarray) -> np.ndarray:
    """(bh, bw, 64) int16 + natural-order quant -> (bh*8, bw*8) uint8 (jpeg_idct_islow)."""
    bh, bw, _ = coef.shape
    c = coef.astype(np.int64).reshape(bh * bw, 8, 8) * q.reshape(1, 8, 8)
    # pass 1: columns (axis 1 = row index u), DESCALE by CONST_BITS - PASS1_BITS
    s1 = CONST_BITS - PASS1_BITS
    ws = _idct_1d(np.moveaxis(c, 1, 0), s1, 1 << (s1 - 1))        # (8 rows, n, 8 cols)
    # pass 2: rows, DESCALE by CONST_BITS + PASS1_BITS + 3
    s2 = CONST_BITS + PASS1_BITS + 3
    out = _idct_1d(np.moveaxis(ws, 2, 0), s2, 1 << (s2 - 1))      # (8 cols, 8 rows, n)
    px = idct_range_limit(out).astype(np.uint8)                   # [x, y, n]
    px = np.transpose(px, (2, 1, 0)).reshape(bh, bw, 8, 8)
    return px.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)


def upsample(plane: np.ndarray, rh: int, rv: int, dsw: int, dsh: int, W: int, H: int):
    """jdsample.c: component plane (real size dsh x dsw) -> (H, W)."""
    p = plane[:dsh, :dsw].astype(np.int64)
    if rh == 1 and rv == 1:
        return p[:H, :W].astype(np.uint8)
    fancy_h = dsw > 2
    if rh == 2 and rv == 1 and fancy_h:
        prev = np.concatenate([p[:, :1], p[:, :-1]], 1)
        nxt = np.concatenate([p[:, 1:], p[:, -1:]], 1)
        ev = (3 * p + prev + 1) >> 2
        ev[:, 0] = p[:, 0]
        od = (3 * p + nxt + 2) >> 2
        od[:, -1] = p[:, -1]
        out = np.stack([ev, od], 2).reshape(dsh, 2 * dsw)
        return out[:H, :W].astype(np.uint8)
    if rh == 1 and rv == 2:
        up = np.concatenate([p[:1], p[:-1]], 0)
        dn = np.concatenate([p[1:], p[-1:]], 0)
        out = np.stack([(3 * p + up + 1) >> 2, (3 * p + dn + 2) >> 2], 1).reshape(2 * dsh, dsw)
        return out[:H, :W].astype(np.uint8)
    if rh == 2 and rv == 2 and fancy_h:
        res = []
        for nb, b_even, b_odd in ((np.concatenate([p[:1], p[:-1]], 0), 8, 7),
                                  (np.concatenate([p[1:], p[-1:]], 0), 8, 7)):
            cs = 3 * p + nb
            prev = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
            nxt = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
            ev = (3 * cs + prev + b_even) >> 4
            ev[:, 0] = (cs[:, 0] * 4 + 8) >> 4
            od = (3 * cs + nxt + b_odd) >> 4
            od[:, -1] = (cs[:, -1] * 4 + 7) >> 4
            res.append(np.stack([ev, od], 2).reshape(dsh, 2 * dsw))
        out = np.stack(res, 1).reshape(2 * dsh, 2 * dsw)
        return out[:H, :W].astype(np.uint8)
    out = np.repeat(np.repeat(p, rv, 0), rh, 1)   # int_upsample / non-fancy: box replication
    return out[:H, :W].astype(np.uint8)


def _fix(x):
    return int(x * 65536 + 0.5)


def ycc_tables():
    """jdcolor.c build_ycc_rgb_table (SCALEBITS 16)."""
    x = np.arange(256, dtype=np.int64) - 128
    half = 1 << 15
    cr_r = (_fix(1.40200) * x + half) >> 16
    cb_b = (_fix(1.77200) * x + half) >> 16
    cr_g = -_fix(0.71414) * x
    cb_g = -_fix(0.34414) * x + half
    return cr_r, cb_b, cr_g, cb_g


def ycc_to_rgb(y, cb, cr):
    cr_r, cb_b, cr_g, cb_g = ycc_tables()
    y = y.astype(np.int64)
    r = np.clip(y + cr_r[cr], 0, 255)
    g = np.clip(y + ((cb_g[cb] + cr_g[cr]) >> 16), 0, 255)
    b = np.clip(y + cb_b[cb], 0, 255)
    return np.stack([r, g, b], -1).astype(np.uint8)


def decode_rgb(data: bytes) -> np.ndarray:
    """Restated Image.open(...).convert('RGB') for a baseline JPEG -> (H, W, 3) uint8."""
    P = parse(data)
    hs, vs, hmax, vmax, mx, my = geometry(P)
    coef = huffman_decode(P)
    planes = []
    for c in range(P.ncomp):
        plane = idct_islow(coef[c], P.quant[P.tq[c]])
        dsw = -(-P.width * hs[c] // hmax)
        dsh = -(-P.height * vs[c] // vmax)
        planes.append(upsample(plane, hmax // hs[c], vmax // vs[c], dsw, dsh, P.width,
                               P.height))
    if P.ncomp == 1:
        return np.repeat(planes[0][:, :, None], 3, 2)
    if P.colorspace == "rgb":
        return np.stack(planes, -1)
    return ycc_to_rgb(*planes)
