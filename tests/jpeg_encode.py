"""A small baseline-JPEG encoder (test helper) for the sampling layouts Pillow cannot write
(4:4:0 = h1v2, 4:1:1 = h4v1, h4v2, luma 1x2 / 2x1 with full chroma, ...): float FDCT,
ITU-T T.81 Annex K quantisation and Huffman tables, optional restart intervals.  The files
are then decoded by Pillow -- the reference's decode -- and by the code under test."""
import numpy as np

ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
          41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15,
          23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]

Q_LUMA = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40,
          57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35,
          55, 64, 81, 104, 113, 92, 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112,
          100, 103, 99]
Q_CHROMA = [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99,
            99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32

# Annex K.3 tables: (bits[1..16], values)
DC_L = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
DC_C = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
AC_L = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])
AC_C = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])


def _codes(spec):
    bits, vals = spec
    code, k, out = 0, 0, {}
    for l in range(1, 17):
        for _ in range(bits[l - 1]):
            out[vals[k]] = (code, l)
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc, self.n = 0, 0

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc, self.n = 0, 0

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)


def _dct_matrix():
    c = np.zeros((8, 8))
    for u in range(8):
        for x in range(8):
            c[u, x] = (np.sqrt(0.5) if u == 0 else 1.0) * np.cos((2 * x + 1) * u * np.pi / 16) / 2
    return c


_C = _dct_matrix()


def _scaled_q(q, quality):
    s = 5000 / quality if quality < 50 else 200 - 2 * quality
    return [min(255, max(1, (v * s + 50) // 100)) for v in q]


def encode(rgb: np.ndarray, sampling=((2, 2), (1, 1), (1, 1)), quality=80, restart=0,
           gray=False) -> bytes:
    """rgb (H, W, 3) uint8 -> baseline JPEG bytes with the given (h, v) factors per
    component (Y, Cb, Cr), or one gray component."""
    H, W = rgb.shape[:2]
    x = rgb.astype(np.float64)
    if gray:
        planes = [0.299 * x[..., 0] + 0.587 * x[..., 1] + 0.114 * x[..., 2]]
        sampling = ((1, 1),)
    else:
        y = 0.299 * x[..., 0] + 0.587 * x[..., 1] + 0.114 * x[..., 2]
        cb = -0.168736 * x[..., 0] - 0.331264 * x[..., 1] + 0.5 * x[..., 2] + 128
        cr = 0.5 * x[..., 0] - 0.418688 * x[..., 1] - 0.081312 * x[..., 2] + 128
        planes = [y, cb, cr]
    nc = len(planes)
    hmax = max(s[0] for s in sampling)
    vmax = max(s[1] for s in sampling)
    mx, my = -(-W // (8 * hmax)), -(-H // (8 * vmax))
    qt = [_scaled_q(Q_LUMA, quality), _scaled_q(Q_CHROMA, quality)]
    comps = []
    for c in range(nc):
        h, v = sampling[c]
        fx, fy = hmax // h, vmax // v
        pw, ph = mx * h * 8, my * v * 8
        p = planes[c]
        # pad to MCU multiples by edge replication, then box-downsample
        big = np.pad(p, ((0, ph * fy - H), (0, pw * fx - W)), mode="edge")
        ds = big.reshape(ph, fy, pw, fx).mean(axis=(1, 3)) - 128.0
        q = np.asarray(qt[0 if c == 0 else 1], np.float64)
        qnat = np.zeros(64)
        qnat[ZIGZAG] = q
        blocks = ds.reshape(ph // 8, 8, pw // 8, 8).transpose(0, 2, 1, 3)
        coef = np.einsum("ux,abxy,vy->abuv", _C, blocks, _C).reshape(ph // 8, pw // 8, 64)
        comps.append(np.round(coef / qnat).astype(np.int64))
    dcs = [_codes(DC_L), _codes(DC_C)]
    acs = [_codes(AC_L), _codes(AC_C)]
    bits = _Bits()
    data = bytearray()
    pred = [0] * nc
    total = mx * my
    for m in range(total):
        if restart and m and m % restart == 0:
            bits.flush()
            data += bits.out + bytes([0xFF, 0xD0 + ((m // restart - 1) & 7)])
            bits = _Bits()
            pred = [0] * nc
        yy, xx = divmod(m, mx)
        for c in range(nc):
            h, v = sampling[c]
            t = 0 if c == 0 else 1
            for vv in range(v):
                for hh in range(h):
                    blk = comps[c][yy * v + vv, xx * h + hh][ZIGZAG]
                    diff = int(blk[0]) - pred[c]
                    pred[c] = int(blk[0])
                    s = int(abs(diff)).bit_length()
                    code, l = dcs[t][s]
                    bits.put(code, l)
                    if s:
                        bits.put(diff if diff > 0 else diff + (1 << s) - 1, s)
                    run = 0
                    for k in range(1, 64):
                        a = int(blk[k])
                        if a == 0:
                            run += 1
                            continue
                        while run > 15:
                            code, l = acs[t][0xF0]
                            bits.put(code, l)
                            run -= 16
                        s = abs(a).bit_length()
                        code, l = acs[t][(run << 4) | s]
                        bits.put(code, l)
                        bits.put(a if a > 0 else a + (1 << s) - 1, s)
                        run = 0
                    if run:
                        code, l = acs[t][0x00]
                        bits.put(code, l)
    bits.flush()
    data += bits.out

    def seg(marker, payload):
        return bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload

    out = bytearray(b"\xff\xd8")
    out += seg(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    for t in range(1 if gray else 2):
        out += seg(0xDB, bytes([t]) + bytes(qt[t]))
    sof = bytes([8]) + H.to_bytes(2, "big") + W.to_bytes(2, "big") + bytes([nc])
    for c in range(nc):
        h, v = sampling[c]
        sof += bytes([c + 1, (h << 4) | v, 0 if c == 0 else 1])
    out += seg(0xC0, sof)
    for tc, th, spec in ((0, 0, DC_L), (1, 0, AC_L), (0, 1, DC_C), (1, 1, AC_C))[:2 if gray else 4]:
        out += seg(0xC4, bytes([(tc << 4) | th] + spec[0] + spec[1]))
    if restart:
        out += seg(0xDD, restart.to_bytes(2, "big"))
    sos = bytes([nc])
    for c in range(nc):
        t = 0 if c == 0 else 1
        sos += bytes([c + 1, (t << 4) | t])
    out += seg(0xDA, sos + bytes([0, 63, 0]))
    out += data + b"\xff\xd9"
    return bytes(out)


SAMPLINGS = {
    "440_h1v2": ((1, 2), (1, 1), (1, 1)),
    "411_h4v1": ((4, 1), (1, 1), (1, 1)),
    "h4v2": ((4, 2), (1, 1), (1, 1)),
    "h2v2_cb_h2v1": ((2, 2), (2, 1), (1, 1)),
    "h1v1_cb_h1v1_422": ((2, 1), (1, 1), (1, 1)),
    "h3v1": ((3, 1), (1, 1), (1, 1)),
}
