// Batched baseline-JPEG decode on gfx950: the frame decode of the reference's loader,
// Image.open(path).convert('RGB') (datasets/wsol_loader.py:581-582; Pillow 12.2 over
// libjpeg-turbo with its defaults: JDCT_ISLOW, fancy upsampling, jdcolor.c YCbCr->RGB),
// bit-identical to it (tests/test_gpu_jpeg.py; CPU restatement oracle/jpeg_ref.py).
//
// Split of the work:
//   host (tcam_jpeg_pack): marker walk (SOF0/SOF1, DHT, DQT, DRI, SOS, APP0/APP14), byte
//     unstuffing and restart segmentation while the entropy bytes are copied into one
//     staging blob, canonical Huffman tables (9-bit lookahead + maxcode/valoffset)
//     deduplicated over the batch.  O(file bytes), no per-coefficient work.
//   device (tcam_jpeg_decode), four launches on one stream:
//     1. jpeg_huff_kernel   chunk-parallel self-synchronising Huffman decode: every entropy
//        segment (restart interval, or the whole scan) is cut into <= 256 chunks of
//        >= 1024 bits, one lane each; lanes decode their chunk from a guessed entry state
//        and hand the exit state to the next chunk until no entry changes (the first
//        chunk's entry is exact, so the fixpoint is the true parse; Huffman codes resync
//        within a few symbols, so this takes 2 rounds in practice), then a prefix of
//        block counts gives each chunk its block ordinal and a last pass scatters the
//        coefficients (natural order) and DC differences into zeroed int16 blocks.
//        Workgroups hold whole segments of one Huffman table set (tables in LDS).
//     1b. jpeg_dc_kernel    DC prediction: running sums per (segment, component).
//     2. jpeg_idct_kernel   jpeg_idct_islow: 8 lanes per block (column pass, LDS
//        transpose, row pass), dequantisation folded in, range-limit table as arithmetic.
//     3. jpeg_color_kernel  one lane per 4 pixels of a row: h2v1 / h1v2 / h2v2 triangle
//        upsampling (jdsample.c) with edge-replicated context rows (jdmainct.c), box
//        replication for other integral factors, jdcolor.c ycc_rgb_convert, gray -> RGB.
#include "common.h"

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace {

constexpr int kMagic = 0x4a504731;   // "JPG1"
constexpr int kLutBits = 10;
constexpr int kMaxSigTabs = 6;
#ifndef TCAM_JPEG_CHUNK_BITS
#define TCAM_JPEG_CHUNK_BITS 1024
#endif
#ifndef TCAM_JPEG_HUFF_THREADS
#define TCAM_JPEG_HUFF_THREADS 256
#endif
constexpr int kChunkBits = TCAM_JPEG_CHUNK_BITS;     // minimum Huffman chunk length
constexpr int kHuffThreads = TCAM_JPEG_HUFF_THREADS; // chunks per Huffman workgroup (one per lane)

struct JHdr {
    int magic, n, ncomp_desc, nseg, nhblk, ntab;
    int total_blocks, pad0;
    int64_t total_pixels;
    int64_t off_img, off_comp, off_seg, off_hblk, off_tab, off_q, off_bytes, blob_bytes;
    int64_t coef_bytes, plane_bytes, out_bytes;
    int64_t off_chunk;
    int nchunk, max_runs;          // max_runs: max over images of h * ceil(w / 4)
};

struct JImg {
    int w, h, ncomp, cs;          // cs: 0 gray, 1 YCbCr, 2 RGB
    int hmax, vmax, mcus_x, mcus_y;
    int comp0, pad0;
    int64_t out_off, pix_first;
};

struct JComp {
    int img, hs, vs, bw, bh, dsw, dsh, first_block;
    int qoff, dc_slot, ac_slot, stride;
    int64_t coef_off;             // int16 elements
    int64_t plane_off;            // bytes
};

struct JSeg {
    int img, mcu0, nmcu, nchunks;  // nchunks: 16-byte chunks of unstuffed data
    int64_t byte_off;
};

struct JChunk {                    // bits [bit0, bit1) of segment seg
    int seg, bit0, bit1;
};

struct JHBlk {                     // one Huffman workgroup: chunks [ch0, ch0 + nch)
    int ch0, nch, ntabs, pad0;
    int tab[8];
};

struct JTab {
    // Fast path: code + extra bits <= kLutBits decoded in one lookup:
    // (value << 16) | (k advance << 8) | bits consumed; k advance = run + 1 for an AC
    // coefficient, 16 for ZRL, 64 for EOB, 1 for a DC difference.  0 = symbol path.
    uint32_t fast[1 << kLutBits];
    uint16_t lut[1 << kLutBits];   // (len << 8) | symbol for codes <= kLutBits, else 0
    int maxcode[18];
    int valoff[18];
    uint8_t val[256];
};
static_assert(sizeof(JTab) % 16 == 0, "JTab size");

__device__ __constant__ uint8_t kNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ------------------------------------------------------------------ host parsing

struct HSpec {
    uint8_t bits[17];
    uint8_t vals[256];
    int nv;
    bool def;
};

struct Parsed {
    int w = 0, h = 0, nc = 0;
    int cid[4], hs[4], vs[4], tq[4], td[4], ta[4];
    int quant[4][64];
    bool qdef[4] = {false, false, false, false};
    HSpec dc[4], ac[4];
    int ri = 0;
    bool jfif = false;
    int adobe = -1;
    size_t ent = 0;                 // first entropy byte
    std::vector<size_t> seg_bytes;  // unstuffed bytes per restart segment
};

const int kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                      12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                      35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                      58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Walk the entropy-coded data from p; sink(byte) gets every unstuffed byte, cut() every
// RSTn boundary.  Returns the index of the terminating marker's first 0xFF (or len).
template <class Sink, class Cut>
size_t scan_entropy(const uint8_t* d, size_t len, size_t p, Sink sink, Cut cut) {
    while (p < len) {
        // fast path: run of non-0xFF bytes
        const uint8_t* f = (const uint8_t*)memchr(d + p, 0xFF, len - p);
        size_t e = f ? (size_t)(f - d) : len;
        if (e > p) sink(d + p, e - p);
        p = e;
        if (p >= len) break;
        size_t q = p + 1;
        while (q < len && d[q] == 0xFF) ++q;
        if (q >= len) return len;
        uint8_t m = d[q];
        if (m == 0x00) {
            static const uint8_t ff = 0xFF;
            sink(&ff, 1);
            p = q + 1;
        } else if (m >= 0xD0 && m <= 0xD7) {
            cut();
            p = q + 1;
        } else {
            return p;
        }
    }
    return len;
}

inline int u16(const uint8_t* d) { return (d[0] << 8) | d[1]; }

// jdmarker.c read_markers for a baseline single-scan file.  0 or TCAM_JPEG_E_* code.
int parse(const uint8_t* d, size_t len, Parsed& P) {
    if (len < 4 || d[0] != 0xFF || d[1] != 0xD8) return TCAM_JPEG_E_NOTJPEG;
    size_t p = 2;
    bool sof = false, sos = false;
    for (int i = 0; i < 4; ++i) P.dc[i].def = P.ac[i].def = false;
    while (p < len) {
        if (d[p] != 0xFF) return TCAM_JPEG_E_CORRUPT;
        while (p < len && d[p] == 0xFF) ++p;
        if (p >= len) break;
        const int m = d[p++];
        if (m == 0xD9) break;
        if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (p + 2 > len) return TCAM_JPEG_E_CORRUPT;
        const int L = u16(d + p);
        if (L < 2 || p + L > len) return TCAM_JPEG_E_CORRUPT;
        const uint8_t* s = d + p + 2;
        const int sl = L - 2;
        if (m == 0xC0 || m == 0xC1) {
            if (sl < 6) return TCAM_JPEG_E_CORRUPT;
            if (s[0] != 8) return TCAM_JPEG_E_UNSUPPORTED;
            P.h = u16(s + 1);
            P.w = u16(s + 3);
            P.nc = s[5];
            if (P.h == 0 || P.w == 0) return TCAM_JPEG_E_UNSUPPORTED;   // DNL
            if (P.nc != 1 && P.nc != 3) return TCAM_JPEG_E_UNSUPPORTED;
            if (sl < 6 + 3 * P.nc) return TCAM_JPEG_E_CORRUPT;
            for (int c = 0; c < P.nc; ++c) {
                P.cid[c] = s[6 + 3 * c];
                P.hs[c] = s[7 + 3 * c] >> 4;
                P.vs[c] = s[7 + 3 * c] & 15;
                P.tq[c] = s[8 + 3 * c] & 3;
                if (P.hs[c] < 1 || P.hs[c] > 4 || P.vs[c] < 1 || P.vs[c] > 4)
                    return TCAM_JPEG_E_CORRUPT;
            }
            sof = true;
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return TCAM_JPEG_E_UNSUPPORTED;   // progressive / lossless / arithmetic
        } else if (m == 0xCC) {
            return TCAM_JPEG_E_UNSUPPORTED;   // arithmetic conditioning
        } else if (m == 0xC4) {
            int q = 0;
            while (q < sl) {
                if (q + 17 > sl) return TCAM_JPEG_E_CORRUPT;
                const int tc = s[q] >> 4, th = s[q] & 15;
                if (tc > 1 || th > 3) return TCAM_JPEG_E_CORRUPT;
                HSpec& t = tc ? P.ac[th] : P.dc[th];
                t.bits[0] = 0;
                int nv = 0;
                for (int l = 1; l <= 16; ++l) nv += (t.bits[l] = s[q + l]);
                if (nv > 256 || q + 17 + nv > sl) return TCAM_JPEG_E_CORRUPT;
                memcpy(t.vals, s + q + 17, nv);
                t.nv = nv;
                t.def = true;
                q += 17 + nv;
            }
        } else if (m == 0xDB) {
            int q = 0;
            while (q < sl) {
                const int pq = s[q] >> 4, tq = s[q] & 15;
                if (tq > 3) return TCAM_JPEG_E_CORRUPT;
                const int n = pq ? 129 : 65;
                if (q + n > sl) return TCAM_JPEG_E_CORRUPT;
                for (int i = 0; i < 64; ++i)
                    P.quant[tq][kZig[i]] = pq ? u16(s + q + 1 + 2 * i) : s[q + 1 + i];
                P.qdef[tq] = true;
                q += n;
            }
        } else if (m == 0xDD) {
            if (sl < 2) return TCAM_JPEG_E_CORRUPT;
            P.ri = u16(s);
        } else if (m == 0xE0) {
            if (sl >= 5 && memcmp(s, "JFIF\0", 5) == 0) P.jfif = true;
        } else if (m == 0xEE) {
            if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) P.adobe = s[11];
        } else if (m == 0xDA) {
            if (sos) return TCAM_JPEG_E_UNSUPPORTED;   // multi-scan
            if (!sof) return TCAM_JPEG_E_CORRUPT;
            const int ns = s[0];
            if (ns != P.nc || sl < 4 + 2 * ns) return TCAM_JPEG_E_UNSUPPORTED;
            for (int c = 0; c < ns; ++c) {
                if (s[1 + 2 * c] != P.cid[c]) return TCAM_JPEG_E_UNSUPPORTED;
                P.td[c] = s[2 + 2 * c] >> 4;
                P.ta[c] = s[2 + 2 * c] & 15;
                if (P.td[c] > 3 || P.ta[c] > 3) return TCAM_JPEG_E_CORRUPT;
                if (!P.dc[P.td[c]].def || !P.ac[P.ta[c]].def || !P.qdef[P.tq[c]])
                    return TCAM_JPEG_E_CORRUPT;
            }
            if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0)
                return TCAM_JPEG_E_UNSUPPORTED;
            P.ent = p + L;
            P.seg_bytes.assign(1, 0);
            size_t* cur = &P.seg_bytes.back();
            p = scan_entropy(
                d, len, P.ent, [&](const uint8_t*, size_t n) { *cur += n; },
                [&]() {
                    P.seg_bytes.push_back(0);
                    cur = &P.seg_bytes.back();
                });
            sos = true;
            continue;
        }
        p += L;
    }
    if (!sos) return TCAM_JPEG_E_CORRUPT;
    return 0;
}

struct Geo {
    int hs[3], vs[3], hmax, vmax, mx, my;
};

Geo geometry(const Parsed& P) {
    Geo g;
    if (P.nc == 1) {
        g.hs[0] = g.vs[0] = 1;
        g.hmax = g.vmax = 1;
    } else {
        g.hmax = g.vmax = 1;
        for (int c = 0; c < 3; ++c) {
            g.hs[c] = P.hs[c];
            g.vs[c] = P.vs[c];
            g.hmax = std::max(g.hmax, g.hs[c]);
            g.vmax = std::max(g.vmax, g.vs[c]);
        }
    }
    g.mx = (P.w + 8 * g.hmax - 1) / (8 * g.hmax);
    g.my = (P.h + 8 * g.vmax - 1) / (8 * g.vmax);
    return g;
}

// jdhuff.c jpeg_make_d_derived_tbl + kLutBits lookahead tables (symbol, and for AC tables
// the libjpeg-turbo-style "fast AC" entry with the extra bits already extended).
bool build_table(const HSpec& s, bool is_dc, JTab& t) {
    memset(&t, 0, sizeof(t));
    int huffsize[257], huffcode[257], p = 0;
    for (int l = 1; l <= 16; ++l)
        for (int i = 0; i < s.bits[l]; ++i) huffsize[p++] = l;
    huffsize[p] = 0;
    int code = 0, si = huffsize[0];
    p = 0;
    while (huffsize[p]) {
        while (huffsize[p] == si) {
            huffcode[p++] = code;
            ++code;
        }
        if (code >= (1 << si)) return false;   // jdhuff.c: no all-ones code (JERR_BAD_HUFF_TABLE)
        code <<= 1;
        ++si;
    }
    p = 0;
    for (int l = 1; l <= 16; ++l) {
        if (s.bits[l]) {
            t.valoff[l] = p - huffcode[p];
            p += s.bits[l];
            t.maxcode[l] = huffcode[p - 1];
        } else {
            t.maxcode[l] = -1;
        }
    }
    t.maxcode[17] = 0xFFFFF;
    p = 0;
    for (int l = 1; l <= kLutBits; ++l)
        for (int i = 0; i < s.bits[l]; ++i, ++p) {
            const int base = huffcode[p] << (kLutBits - l);
            const int sym = s.vals[p], r = sym >> 4, sz = sym & 15;
            for (int k = 0; k < (1 << (kLutBits - l)); ++k) {
                t.lut[base + k] = (uint16_t)((l << 8) | sym);
                if (is_dc) {   // DC: the symbol is the size; k advance 1, value = difference
                    if (sym == 0) {
                        t.fast[base + k] = (uint32_t)((1 << 8) | l);
                    } else if (sym <= 15 && l + sym <= kLutBits) {
                        const int extra = k >> (kLutBits - l - sym);
                        const int v = extra < (1 << (sym - 1)) ? extra - (1 << sym) + 1 : extra;
                        t.fast[base + k] = ((uint32_t)(uint16_t)(int16_t)v << 16) |
                                           (uint32_t)((1 << 8) | (l + sym));
                    }
                    continue;
                }
                if (sz == 0) {
                    t.fast[base + k] = (uint32_t)(((r == 15 ? 16 : 64) << 8) | l);
                } else if (l + sz <= kLutBits) {
                    const int extra = k >> (kLutBits - l - sz);
                    const int v = extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra;
                    t.fast[base + k] = ((uint32_t)(uint16_t)(int16_t)v << 16) |
                                       (uint32_t)((r + 1) << 8) | (uint32_t)(l + sz);
                }
            }
        }
    for (int i = 0; i < s.nv; ++i) {
        if (is_dc && s.vals[i] > 15) return false;
        t.val[i] = s.vals[i];
    }
    return true;
}

inline int64_t al16(int64_t x) { return (x + 15) & ~(int64_t)15; }

}  // namespace

// ------------------------------------------------------------------ device kernels

namespace {

// Bit reader over one segment's unstuffed bytes, starting at any bit: the 64-byte block
// being consumed sits in the lane's LDS slot, the next one is in flight in registers
// (loaded when the slot is refilled, so its latency hides behind ~512 bits of decoding),
// and the next 32-bit word is read from the slot one refill ahead.  16-byte pieces past
// the segment's end read as zeros (libjpeg's fill after a marker).
struct BitSrc {
    const uint4* src;
    int n16;                       // 16-byte pieces in the segment
    int bi;                        // 64-byte block held in q
    uint4 q0, q1, q2, q3;
    uint32_t* slot;                // 16 words in LDS
    int wi;                        // index of nextw in the slot
    uint32_t nextw;
    uint64_t buf;
    int nb;
    int pos;                       // bit position of buf's first bit in the segment
};

__device__ __forceinline__ void blk_load(BitSrc& b, int bi) {
    // blocks wholly past the end are clamped (their pieces are masked to zero anyway), so
    // a read ends < 12 pieces past the segment: inside the next segment or the blob's pad
    const int i = min(4 * bi, (b.n16 & ~3) + 8);
    b.bi = bi;
    b.q0 = b.src[i];
    b.q1 = b.src[i + 1];
    b.q2 = b.src[i + 2];
    b.q3 = b.src[i + 3];
}

__device__ __forceinline__ uint4 masked(uint4 q, bool keep) {   // no aggregate selects
    const uint32_t m = keep ? 0xffffffffu : 0u;
    return make_uint4(q.x & m, q.y & m, q.z & m, q.w & m);
}

__device__ __forceinline__ void blk_store(BitSrc& b) {   // q -> slot, zeros past the end
    const int base = 4 * b.bi;
    uint4* d = (uint4*)b.slot;
    d[0] = masked(b.q0, base + 0 < b.n16);
    d[1] = masked(b.q1, base + 1 < b.n16);
    d[2] = masked(b.q2, base + 2 < b.n16);
    d[3] = masked(b.q3, base + 3 < b.n16);
}

__device__ __forceinline__ void bits_open(BitSrc& b, const uint4* src, int n16, uint32_t* slot,
                                          int bit) {
    b.src = src;
    b.n16 = n16;
    b.slot = slot;
    blk_load(b, bit >> 9);
    blk_store(b);
    blk_load(b, (bit >> 9) + 1);
    const int wi = (bit >> 5) & 15, off = bit & 31;
    b.buf = (uint64_t)__builtin_bswap32(slot[wi]) << (32 + off);
    b.nb = 32 - off;
    b.pos = bit;
    b.wi = wi + 1;
    if (b.wi == 16) {
        b.wi = 0;
        blk_store(b);
        blk_load(b, b.bi + 1);
    }
    b.nextw = slot[b.wi];
}

__device__ __forceinline__ void refill(BitSrc& b) {
    if (b.nb <= 32) {
        b.buf |= (uint64_t)__builtin_bswap32(b.nextw) << (32 - b.nb);
        b.nb += 32;
        if (++b.wi == 16) {
            b.wi = 0;
            blk_store(b);
            blk_load(b, b.bi + 1);
        }
        b.nextw = b.slot[b.wi];
    }
}

__device__ __forceinline__ void consume(BitSrc& b, int n) {
    b.buf <<= n;
    b.nb -= n;
    b.pos += n;
}

__device__ __forceinline__ int getbits(BitSrc& b, int s) {   // 1 <= s <= 16
    const int r = (int)(b.buf >> (64 - s));
    consume(b, s);
    return r;
}

__device__ __forceinline__ int extend(int r, int s) {
    return r < (1 << (s - 1)) ? r - (1 << s) + 1 : r;
}

// One Huffman symbol (jdhuff.c jpeg_huff_decode): lookahead table, then the canonical
// maxcode search over lengths kLutBits+1 .. 16 (independent compares, first hit wins).
__device__ __forceinline__ int huff(BitSrc& b, const JTab& t) {
    const int e = t.lut[b.buf >> (64 - kLutBits)];
    int l, sym;
    if (e) {
        l = e >> 8;
        sym = e & 255;
    } else {
        l = 17;
#pragma unroll
        for (int ll = 16; ll > kLutBits; --ll)
            if ((int)(b.buf >> (64 - ll)) <= t.maxcode[ll]) l = ll;
        if (l > 16) {          // corrupt code: libjpeg substitutes a zero symbol
            l = 16;
            sym = 0;
        } else {
            sym = t.val[((int)(b.buf >> (64 - l)) + t.valoff[l]) & 255];
        }
    }
    consume(b, l);
    return sym;
}

// Decoder state at a symbol boundary: bit position, block-in-MCU j, next coefficient k
// (k == 0: a DC symbol comes next).  Packed (pos << 12) | (j << 6) | k.
__device__ __forceinline__ int64_t st_pack(int pos, int j, int k) {
    return ((int64_t)pos << 12) | (j << 6) | k;
}

// per-component fields picked with selects (a dynamic index would put the arrays in scratch)
template <class T>
__device__ __forceinline__ T sel3(int c, const T (&a)[3]) {
    return c == 0 ? a[0] : (c == 1 ? a[1] : a[2]);
}

struct SegCtx {
    const uint4* src;
    int nch16, bpm;
    uint64_t jcomp;                // block j of the MCU: component | v << 2 | h << 4, 6 bits each
    int jfirst[3];                 // first block index of each component in the MCU
    int hs[3], vs[3], bw[3], dcs[3], acs[3];
    int64_t co[3];
    int mcu0, mcus_x, total_blocks;
};

// Decode the symbols that start in [bit, end) from state (j, k).  WRITE: scatter the
// nonzero coefficients and DC differences of blocks ord, ord+1, ... (ord = ordinal of the
// block in progress, or of the next one when k == 0) into the zeroed coefficient buffer
// (blocks cut by a chunk edge get their pieces from both lanes).  One code path for DC
// and AC symbols (a DC difference is a k advance of 1 stored at natural index 0), so a
// wave's lanes stay converged.  Returns the exit state; *nstart = blocks started.
template <bool WRITE>
__device__ __forceinline__ int64_t decode_run(const SegCtx& s, const JTab* tabs,
                                              const uint8_t* nat, uint32_t* slot, int bit,
                                              int end, int j, int k, int ord, int16_t* coef,
                                              int* nstart) {
    BitSrc b;
    bits_open(b, s.src, s.nch16, slot, bit);
    int starts = 0;
    int ji = (int)((s.jcomp >> (6 * j)) & 63);
    // MCU position of block ord (write pass)
    int mx = 0, my = 0;
    int16_t* blk = coef;
    auto locate = [&]() {
        const int cc = ji & 3, v = (ji >> 2) & 3, h = ji >> 4;
        blk = coef + sel3(cc, s.co) +
              ((int64_t)(my * sel3(cc, s.vs) + v) * sel3(cc, s.bw) + mx * sel3(cc, s.hs) + h) * 64;
    };
    if (WRITE) {
        // a corrupt stream can leave a garbage parse: never address outside the segment
        if (ord < 0 || ord >= s.total_blocks) {
            *nstart = 0;
            return st_pack(bit, j, k);
        }
        const int m = s.mcu0 + ord / s.bpm;
        my = m / s.mcus_x;
        mx = m - my * s.mcus_x;
        if (k > 0) locate();
    }
    while (b.pos < end) {
        if (WRITE && k == 0 && ord >= s.total_blocks) break;   // trailing pad bits
        refill(b);
        const int cc = ji & 3;
        const JTab& tb = tabs[k == 0 ? sel3(cc, s.dcs) : sel3(cc, s.acs)];
        const uint32_t e = tb.fast[b.buf >> (64 - kLutBits)];
        int v, kadv;
        if (e) {
            consume(b, (int)(e & 31));
            kadv = (int)((e >> 8) & 127);
            v = (int)e >> 16;
        } else {
            const int sym = huff(b, tb);
            const int r = k ? sym >> 4 : 0, t = k ? sym & 15 : sym;
            v = t ? extend(getbits(b, t), t) : 0;
            kadv = t ? r + 1 : (k == 0 ? 1 : (r == 15 ? 16 : 64));
        }
        if (k == 0) {
            ++starts;
            if (WRITE) locate();
        }
        k += kadv;
        if (WRITE && v) blk[nat[k - 1]] = (int16_t)v;
        if (k >= 64) {
            k = 0;
            ++ord;
            if (++j == s.bpm) {
                j = 0;
                if (++mx == s.mcus_x) {
                    mx = 0;
                    ++my;
                }
            }
            ji = (int)((s.jcomp >> (6 * j)) & 63);
        }
    }
    *nstart = starts;
    return st_pack(b.pos, j, k);
}

// Chunk-parallel Huffman decode (self-synchronising): every chunk of a segment is decoded
// from a guessed entry state; exit states become the next chunk's entry state until no
// entry changes (the first chunk's entry is exact, so the fixpoint is the true parse),
// then block counts are prefix-summed and a final pass scatters the coefficients.
__global__ __launch_bounds__(kHuffThreads) void jpeg_huff_kernel(
    const uint8_t* __restrict__ blob, int16_t* __restrict__ coef, int* __restrict__ dbg) {
    __shared__ JTab tabs[kMaxSigTabs];
    __shared__ uint8_t nat[80];
    __shared__ uint4 slots[kHuffThreads][4];          // bit-reader blocks
    __shared__ int64_t entry[kHuffThreads + 1];
    __shared__ int nblk[kHuffThreads];
    __shared__ int changed[2];
    const JHdr* H = (const JHdr*)blob;
    const JHBlk* hbp = (const JHBlk*)(blob + H->off_hblk) + blockIdx.x;
    const int hb_ch0 = hbp->ch0, hb_nch = hbp->nch, hb_ntabs = hbp->ntabs;
    {
        const JTab* g = (const JTab*)(blob + H->off_tab);
        const int per = (int)(sizeof(JTab) / 16);
        for (int i = threadIdx.x; i < hb_ntabs * per; i += kHuffThreads) {
            const int t = i / per, kk = i - t * per;
            ((uint4*)&tabs[t])[kk] = ((const uint4*)&g[hbp->tab[t]])[kk];
        }
        if (threadIdx.x < 80) nat[threadIdx.x] = kNatural[threadIdx.x];
    }
    const int t = threadIdx.x;
    const bool live = t < hb_nch;
    JChunk ck;
    ck.seg = 0;
    ck.bit0 = ck.bit1 = 0;
    SegCtx s;
    if (live) {
        ck = ((const JChunk*)(blob + H->off_chunk))[hb_ch0 + t];
        const JSeg sg = ((const JSeg*)(blob + H->off_seg))[ck.seg];
        const JImg im = ((const JImg*)(blob + H->off_img))[sg.img];
        const JComp* cp = (const JComp*)(blob + H->off_comp) + im.comp0;
        s.src = (const uint4*)(blob + H->off_bytes + sg.byte_off);
        s.nch16 = sg.nchunks;
        s.mcu0 = sg.mcu0;
        s.mcus_x = im.mcus_x;
        s.jcomp = 0;
        int bpm = 0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int cc = c < im.ncomp ? c : 0;
            s.hs[c] = cp[cc].hs;
            s.vs[c] = cp[cc].vs;
            s.bw[c] = cp[cc].bw;
            s.dcs[c] = cp[cc].dc_slot;
            s.acs[c] = cp[cc].ac_slot;
            s.co[c] = cp[cc].coef_off;
            s.jfirst[c] = bpm;
            if (c < im.ncomp) {
                for (int v = 0; v < s.vs[c]; ++v)
                    for (int h = 0; h < s.hs[c]; ++h, ++bpm)
                        s.jcomp |= (uint64_t)(c | (v << 2) | (h << 4)) << (6 * bpm);
            }
        }
        s.bpm = bpm;
        s.total_blocks = sg.nmcu * bpm;
        // first chunk of a segment: exact entry; others: a guess at the chunk start
        entry[t] = st_pack(ck.bit0, 0, 0);
    }
    bool feeds_next = false;   // chunk t + 1 belongs to the same segment
    if (live && t + 1 < hb_nch)
        feeds_next = ((const JChunk*)(blob + H->off_chunk))[hb_ch0 + t + 1].seg == ck.seg;
    if (t == 0) changed[0] = 0;
    __syncthreads();
    const int64_t clk0 = clock64();
    // 1. fixpoint over entry states (flag double-buffered by iteration parity: the flag of
    //    iteration it + 1 is cleared after every lane has read the one of it - 1)
    int64_t exit_st = 0;
    int64_t done_from = -1;   // entry state the current exit_st was computed from
    for (int it = 0; it <= kHuffThreads; ++it) {
        if (live) {
            const int64_t e = entry[t];
            if (e != done_from) {
                int ns;
                exit_st = decode_run<false>(s, tabs, nat, (uint32_t*)slots[t], (int)(e >> 12),
                                            ck.bit1,
                                            (int)((e >> 6) & 63), (int)(e & 63), 0, coef, &ns);
                nblk[t] = ns;
                done_from = e;
            }
        }
        __syncthreads();
        if (t == 0) changed[(it + 1) & 1] = 0;
        if (feeds_next && entry[t + 1] != exit_st) {
            entry[t + 1] = exit_st;
            changed[it & 1] = 1;
        }
        __syncthreads();
        if (!changed[it & 1]) {
            if (dbg && t == 0) {   // diagnostics: rounds, cycles of the fixpoint
                dbg[4 * blockIdx.x] = it + 1;
                dbg[4 * blockIdx.x + 1] = (int)(clock64() - clk0);
            }
            break;
        }
    }
    // 2. block ordinal at each chunk's entry: exclusive prefix of block starts per segment
    //    (sequential over the workgroup's chunks: <= 256 adds by one lane)
    __shared__ int ord0[kHuffThreads];
    if (t == 0) {
        int run = 0, seg = -1;
        for (int i = 0; i < hb_nch; ++i) {
            const int sgi = ((const JChunk*)(blob + H->off_chunk))[hb_ch0 + i].seg;
            if (sgi != seg) {
                seg = sgi;
                run = 0;
            }
            ord0[i] = run;
            run += nblk[i];
        }
    }
    __syncthreads();
    // 3. write pass from the exact entry states
    if (live) {
        const int64_t e = entry[t];
        const int k = (int)(e & 63);
        const int ord = ord0[t] - (k > 0 ? 1 : 0);
        int ns;
        const int64_t c1 = clock64();
        decode_run<true>(s, tabs, nat, (uint32_t*)slots[t], (int)(e >> 12), ck.bit1,
                         (int)((e >> 6) & 63), k, ord, coef, &ns);
        if (dbg && t == 0) {   // diagnostics: cycles and blocks of lane 0's write pass
            dbg[4 * blockIdx.x + 2] = (int)(clock64() - c1);
            dbg[4 * blockIdx.x + 3] = ns;
        }
    }
}

// DC prediction (jdhuff.c last_dc_val): per (segment, component), the decoded DC
// differences become running sums in MCU order, reset at every restart interval.
__global__ __launch_bounds__(256) void jpeg_dc_kernel(const uint8_t* __restrict__ blob,
                                                      int16_t* __restrict__ coef) {
    __shared__ int part[256];
    const JHdr* H = (const JHdr*)blob;
    const int task = blockIdx.x;
    const int segi = task / 3, c = task - segi * 3;
    const JSeg sg = ((const JSeg*)(blob + H->off_seg))[segi];
    const JImg im = ((const JImg*)(blob + H->off_img))[sg.img];
    if (c >= im.ncomp) return;
    const JComp cp = ((const JComp*)(blob + H->off_comp))[im.comp0 + c];
    const int per_mcu = cp.hs * cp.vs;
    const int count = sg.nmcu * per_mcu;
    const int per = (count + 255) / 256;
    const int i0 = min(count, (int)threadIdx.x * per), i1 = min(count, i0 + per);
    auto addr = [&](int i) -> int16_t* {
        const int m = i / per_mcu, r = i - m * per_mcu;
        const int v = r / cp.hs, h = r - v * cp.hs;
        const int mcu = sg.mcu0 + m;
        const int my = mcu / im.mcus_x, mx = mcu - my * im.mcus_x;
        return coef + cp.coef_off + ((int64_t)(my * cp.vs + v) * cp.bw + mx * cp.hs + h) * 64;
    };
    int sum = 0;
    for (int i = i0; i < i1; ++i) sum += *addr(i);
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int i = 0; i < 256; ++i) {
            const int v = part[i];
            part[i] = run;
            run += v;
        }
    }
    __syncthreads();
    int run = part[threadIdx.x];
    for (int i = i0; i < i1; ++i) {
        int16_t* p = addr(i);
        run += *p;
        *p = (int16_t)run;
    }
}

// jidctint.c jpeg_idct_islow constants (CONST_BITS 13)
#define F0298 2446
#define F0390 3196
#define F0541 4433
#define F0765 6270
#define F0899 7373
#define F1175 9633
#define F1501 12299
#define F1847 15137
#define F1961 16069
#define F2053 16819
#define F2562 20995
#define F3072 25172

__device__ __forceinline__ void idct8(const int* v, int* o, int shift) {
    const int rnd = 1 << (shift - 1);
    int z2 = v[2], z3 = v[6];
    int z1 = (z2 + z3) * F0541;
    const int tmp2e = z1 + z3 * (-F1847);
    const int tmp3e = z1 + z2 * F0765;
    const int t0 = (v[0] + v[4]) * (1 << 13);
    const int t1 = (v[0] - v[4]) * (1 << 13);
    const int t10 = t0 + tmp3e, t13 = t0 - tmp3e, t11 = t1 + tmp2e, t12 = t1 - tmp2e;
    int tmp0 = v[7], tmp1 = v[5], tmp2 = v[3], tmp3 = v[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 = z3 * (-F1961) + z5;
    z4 = z4 * (-F0390) + z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = (t10 + tmp3 + rnd) >> shift;
    o[7] = (t10 - tmp3 + rnd) >> shift;
    o[1] = (t11 + tmp2 + rnd) >> shift;
    o[6] = (t11 - tmp2 + rnd) >> shift;
    o[2] = (t12 + tmp1 + rnd) >> shift;
    o[5] = (t12 - tmp1 + rnd) >> shift;
    o[3] = (t13 + tmp0 + rnd) >> shift;
    o[4] = (t13 - tmp0 + rnd) >> shift;
}

// jdmaster.c prepare_range_limit_table as read by the IDCT (index & RANGE_MASK)
__device__ __forceinline__ uint32_t range_limit(int x) {
    const int i = x & 1023;
    return (uint32_t)(i < 128 ? i + 128 : i < 512 ? 255 : i < 896 ? 0 : i - 896);
}

// last index i with first(a[i]) <= key over an ascending array
#define FIND_LAST_LE(a, n, key, field)            \
    ({                                            \
        int lo_ = 0, hi_ = (n) - 1;               \
        while (lo_ < hi_) {                       \
            const int mid_ = (lo_ + hi_ + 1) >> 1; \
            if ((int64_t)(a)[mid_].field <= (key)) \
                lo_ = mid_;                       \
            else                                  \
                hi_ = mid_ - 1;                   \
        }                                         \
        lo_;                                      \
    })

constexpr int kIdctBlocks = 32;   // blocks per 256-thread workgroup

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const uint8_t* __restrict__ blob,
                                                        const int16_t* __restrict__ coef,
                                                        uint8_t* __restrict__ planes) {
    __shared__ int dq[kIdctBlocks][8][9];   // dequantised coefficients, row-major
    __shared__ int ws[kIdctBlocks][8][9];   // column-pass output
    __shared__ int s_comp;
    const JHdr* H = (const JHdr*)blob;
    const int lb = threadIdx.x >> 3, c = threadIdx.x & 7;
    const int g0 = blockIdx.x * kIdctBlocks;
    const int g = g0 + lb;
    const int total = H->total_blocks;
    const bool live = g < total;
    const JComp* comps = (const JComp*)(blob + H->off_comp);
    // the workgroup's 32 blocks nearly always lie in one component: search once
    if (threadIdx.x == 0) {
        const int ci0 = FIND_LAST_LE(comps, H->ncomp_desc, (int64_t)g0, first_block);
        const int gl = min(g0 + kIdctBlocks, total) - 1;
        const int ci1 = FIND_LAST_LE(comps, H->ncomp_desc, (int64_t)gl, first_block);
        s_comp = ci0 == ci1 ? ci0 : -1;
    }
    __syncthreads();
    const int ci = s_comp >= 0 ? s_comp
                               : (live ? FIND_LAST_LE(comps, H->ncomp_desc, (int64_t)g, first_block) : 0);
    const JComp cp = comps[ci];
    const int b = g - cp.first_block;
    if (live) {   // lane c: row c of the block, one 16-B load + its quantiser row
        const int4 raw = *(const int4*)(coef + cp.coef_off + (int64_t)b * 64 + 8 * c);
        const int4* q4 = (const int4*)((const int*)(blob + H->off_q) + cp.qoff + 8 * c);
        const int4 qa = q4[0], qb = q4[1];
        const uint32_t w[4] = {(uint32_t)raw.x, (uint32_t)raw.y, (uint32_t)raw.z, (uint32_t)raw.w};
        const int qq[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int16_t v = (int16_t)((k & 1) ? (w[k >> 1] >> 16) : (w[k >> 1] & 0xffffu));
            dq[lb][c][k] = (int)v * qq[k];
        }
    }
    __syncthreads();
    if (live) {   // column pass: lane c = column c
        int v[8], o[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = dq[lb][r][c];
        idct8(v, o, 11);   // CONST_BITS - PASS1_BITS
#pragma unroll
        for (int r = 0; r < 8; ++r) ws[lb][r][c] = o[r];
    }
    __syncthreads();
    if (!live) return;
    int v[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ws[lb][c][k];
    idct8(v, o, 18);       // CONST_BITS + PASS1_BITS + 3
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lo |= range_limit(o[k]) << (8 * k);
        hi |= range_limit(o[k + 4]) << (8 * k);
    }
    const int by = b / cp.bw, bx = b - by * cp.bw;
    uint2* dst = (uint2*)(planes + cp.plane_off + (int64_t)(by * 8 + c) * cp.stride + bx * 8);
    *dst = make_uint2(lo, hi);
}

struct CompView {
    const uint8_t* p;
    int stride, rh, rv, dsw, dsh;
};

__device__ __forceinline__ int px(const CompView& v, int y, int x) { return v.p[y * v.stride + x]; }

// jdsample.c for one output sample (y, x) of a component
__device__ __forceinline__ int upsample(const CompView& v, int y, int x) {
    if (v.rh == 1 && v.rv == 1) return px(v, y, x);
    if (v.rh == 2 && v.rv == 1 && v.dsw > 2) {          // h2v1_fancy_upsample
        const int ix = x >> 1, cur = px(v, y, ix);
        if (!(x & 1)) return ix == 0 ? cur : (3 * cur + px(v, y, ix - 1) + 1) >> 2;
        return ix == v.dsw - 1 ? cur : (3 * cur + px(v, y, ix + 1) + 2) >> 2;
    }
    if (v.rh == 1 && v.rv == 2) {                       // h1v2_fancy_upsample
        const int iy = y >> 1;
        const int ny = (y & 1) ? min(iy + 1, v.dsh - 1) : max(iy - 1, 0);
        return (3 * px(v, iy, x) + px(v, ny, x) + ((y & 1) ? 2 : 1)) >> 2;
    }
    if (v.rh == 2 && v.rv == 2 && v.dsw > 2) {          // h2v2_fancy_upsample
        const int iy = y >> 1;
        const int ny = (y & 1) ? min(iy + 1, v.dsh - 1) : max(iy - 1, 0);
        const int ix = x >> 1;
        const int cs = 3 * px(v, iy, ix) + px(v, ny, ix);
        if (!(x & 1)) {
            if (ix == 0) return (cs * 4 + 8) >> 4;
            return (3 * cs + 3 * px(v, iy, ix - 1) + px(v, ny, ix - 1) + 8) >> 4;
        }
        if (ix == v.dsw - 1) return (cs * 4 + 7) >> 4;
        return (3 * cs + 3 * px(v, iy, ix + 1) + px(v, ny, ix + 1) + 7) >> 4;
    }
    return px(v, y / v.rv, x / v.rh);                   // int_upsample / box
}

__device__ __forceinline__ int clamp255(int x) { return min(max(x, 0), 255); }

__device__ __forceinline__ uint32_t ycc_rgb(int y, int cb, int cr, int cs) {
    int r, g, bl;
    if (cs == 0) {
        r = g = bl = y;
    } else if (cs == 2) {
        r = y;
        g = cb;
        bl = cr;
    } else {   // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert, SCALEBITS 16
        cb -= 128;
        cr -= 128;
        const int crr = (91881 * cr + 32768) >> 16;
        const int cbb = (116130 * cb + 32768) >> 16;
        const int gg = ((-22554 * cb + 32768) + (-46802 * cr)) >> 16;
        r = clamp255(y + crr);
        g = clamp255(y + gg);
        bl = clamp255(y + cbb);
    }
    return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)bl << 16);
}

constexpr int kColorPx = 4;   // output pixels of one row per lane

// blockIdx.y = image (its descriptors are wave-uniform scalar loads), blockIdx.x * 256 +
// lane = a run of 4 pixels of one row; 12 output bytes as three 4-byte stores when aligned.
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ blob,
                                                         const uint8_t* __restrict__ planes,
                                                         uint8_t* __restrict__ out) {
    const JHdr* H = (const JHdr*)blob;
    const JImg im = ((const JImg*)(blob + H->off_img))[blockIdx.y];
    const int qpr = (im.w + kColorPx - 1) / kColorPx;   // runs per row
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= qpr * im.h) return;
    const int y = q / qpr, x0 = (q - y * qpr) * kColorPx;
    const JComp* cp = (const JComp*)(blob + H->off_comp) + im.comp0;
    int smp[3][kColorPx];
    // 4:2:0 fast path (image-uniform): the 4 pixels share chroma columns ix0-1 .. ix0+2 of
    // rows iy and its context row, loaded once per component; the same h2v2 arithmetic
    const bool f420 = im.ncomp == 3 && im.hmax == 2 && im.vmax == 2 && cp[0].hs == 2 &&
                      cp[0].vs == 2 && cp[1].hs == 1 && cp[1].vs == 1 && cp[2].hs == 1 &&
                      cp[2].vs == 1 && cp[1].dsw > 2 && cp[2].dsw > 2;
    if (f420) {
        const uint8_t* yp = planes + cp[0].plane_off + (int64_t)y * cp[0].stride + x0;
        const uint32_t yw = *(const uint32_t*)yp;   // x0 % 4 == 0, stride % 8 == 0
#pragma unroll
        for (int i = 0; i < kColorPx; ++i) smp[0][i] = (yw >> (8 * i)) & 255;
#pragma unroll
        for (int c = 1; c < 3; ++c) {
            const int dsw = cp[c].dsw, dsh = cp[c].dsh, st = cp[c].stride;
            const uint8_t* pl = planes + cp[c].plane_off;
            const int iy = y >> 1, ny = (y & 1) ? min(iy + 1, dsh - 1) : max(iy - 1, 0);
            const int ix0 = x0 >> 1;
            int cs[4];   // column sums 3 * row iy + row ny at ix0-1 .. ix0+2 (clamped)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ix = min(max(ix0 - 1 + j, 0), dsw - 1);
                cs[j] = 3 * pl[iy * st + ix] + pl[ny * st + ix];
            }
            // x0 (even, ix0), x0+1 (odd, ix0), x0+2 (even, ix0+1), x0+3 (odd, ix0+1)
            smp[c][0] = ix0 == 0 ? (cs[1] * 4 + 8) >> 4 : (3 * cs[1] + cs[0] + 8) >> 4;
            smp[c][1] = ix0 == dsw - 1 ? (cs[1] * 4 + 7) >> 4 : (3 * cs[1] + cs[2] + 7) >> 4;
            smp[c][2] = (3 * cs[2] + cs[1] + 8) >> 4;
            smp[c][3] = ix0 + 1 == dsw - 1 ? (cs[2] * 4 + 7) >> 4 : (3 * cs[2] + cs[3] + 7) >> 4;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (f420 || c >= im.ncomp) break;
        CompView v;
        v.p = planes + cp[c].plane_off;
        v.stride = cp[c].stride;
        v.rh = im.hmax / cp[c].hs;
        v.rv = im.vmax / cp[c].vs;
        v.dsw = cp[c].dsw;
        v.dsh = cp[c].dsh;
#pragma unroll
        for (int i = 0; i < kColorPx; ++i) smp[c][i] = upsample(v, y, min(x0 + i, im.w - 1));
    }
    uint32_t px[kColorPx];
#pragma unroll
    for (int i = 0; i < kColorPx; ++i)
        px[i] = im.ncomp == 1 ? ycc_rgb(smp[0][i], 0, 0, 0)
                              : ycc_rgb(smp[0][i], smp[1][i], smp[2][i], im.cs);
    uint8_t* o = out + im.out_off + ((int64_t)y * im.w + x0) * 3;
    if (x0 + kColorPx <= im.w && (((uintptr_t)o) & 3) == 0) {
        uint32_t* o4 = (uint32_t*)o;
        o4[0] = px[0] | (px[1] << 24);
        o4[1] = (px[1] >> 8) | (px[2] << 16);
        o4[2] = (px[2] >> 16) | (px[3] << 8);
    } else {
#pragma unroll
        for (int i = 0; i < kColorPx; ++i) {
            if (x0 + i >= im.w) break;
            o[3 * i] = (uint8_t)px[i];
            o[3 * i + 1] = (uint8_t)(px[i] >> 8);
            o[3 * i + 2] = (uint8_t)(px[i] >> 16);
        }
    }
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" int tcam_jpeg_pack(const uint8_t* const* data, const size_t* len, int n, void* blob,
                              size_t cap, int64_t* sizes, int* dims) {
    if (n < 0 || (n > 0 && (!data || !len)) || !sizes) return TCAM_E_ARG;
    std::vector<Parsed> P(n);
    int err = 0;
    for (int i = 0; i < n; ++i) {
        int e = data[i] ? parse(data[i], len[i], P[i]) : TCAM_JPEG_E_NOTJPEG;
        if (!e) {   // restart segments must match the interval
            const Geo g = geometry(P[i]);
            const int64_t total = (int64_t)g.mx * g.my;
            const int64_t ri = P[i].ri ? P[i].ri : total;
            if ((int64_t)P[i].seg_bytes.size() != (total + ri - 1) / ri) e = TCAM_JPEG_E_CORRUPT;
            if (P[i].nc == 3)
                for (int c = 0; c < 3; ++c)
                    if (g.hmax % g.hs[c] || g.vmax % g.vs[c]) e = TCAM_JPEG_E_UNSUPPORTED;
        }
        if (dims) {
            dims[3 * i + 0] = e ? 0 : P[i].h;
            dims[3 * i + 1] = e ? 0 : P[i].w;
            dims[3 * i + 2] = e;
        }
        if (e && !err) err = e;
    }
    if (err) return err;

    // Huffman tables deduplicated by content; one signature (ordered table list) per image
    std::map<std::string, int> tab_id;
    std::vector<JTab> tabs;
    std::map<std::vector<int>, int> sig_id;
    std::vector<std::vector<int>> sigs;
    std::vector<int> img_sig(n);
    std::vector<std::array<int, 6>> img_slots(n);
    for (int i = 0; i < n; ++i) {
        std::vector<int> sig;
        auto slot_of = [&](const HSpec& s, bool dc) -> int {
            std::string key(1, dc ? 'D' : 'A');
            key.append((const char*)s.bits + 1, 16);
            key.append((const char*)s.vals, s.nv);
            auto it = tab_id.find(key);
            int id;
            if (it == tab_id.end()) {
                JTab t;
                if (!build_table(s, dc, t)) return -1;
                id = (int)tabs.size();
                tabs.push_back(t);
                tab_id[key] = id;
            } else {
                id = it->second;
            }
            for (size_t k = 0; k < sig.size(); ++k)
                if (sig[k] == id) return (int)k;
            sig.push_back(id);
            return (int)sig.size() - 1;
        };
        for (int c = 0; c < P[i].nc; ++c) {
            const int d = slot_of(P[i].dc[P[i].td[c]], true);
            const int a = slot_of(P[i].ac[P[i].ta[c]], false);
            if (d < 0 || a < 0) {
                if (dims) dims[3 * i + 2] = TCAM_JPEG_E_CORRUPT;
                return TCAM_JPEG_E_CORRUPT;
            }
            img_slots[i][2 * c] = d;
            img_slots[i][2 * c + 1] = a;
        }
        auto it = sig_id.find(sig);
        if (it == sig_id.end()) {
            img_sig[i] = (int)sigs.size();
            sig_id[sig] = img_sig[i];
            sigs.push_back(sig);
        } else {
            img_sig[i] = it->second;
        }
    }

    // sizes
    int ncd = 0, nseg = 0;
    int64_t total_blocks = 0, total_pix = 0, coef = 0, plane = 0, out = 0, bytes = 0;
    std::vector<Geo> G(n);
    for (int i = 0; i < n; ++i) {
        G[i] = geometry(P[i]);
        ncd += P[i].nc;
        nseg += (int)P[i].seg_bytes.size();
        for (int c = 0; c < P[i].nc; ++c) {
            const int64_t nb = (int64_t)G[i].mx * G[i].hs[c] * G[i].my * G[i].vs[c];
            total_blocks += nb;
            coef += nb * 64;
            plane += al16(nb * 64);
        }
        for (size_t s : P[i].seg_bytes) bytes += al16((int64_t)s);
        total_pix += (int64_t)P[i].w * P[i].h;
        out += (int64_t)P[i].w * P[i].h * 3;
    }
    if (total_blocks > 0x7fffffff) return TCAM_E_ARG;
    for (int i = 0; i < n; ++i)   // chunk bit positions are int
        for (size_t sb : P[i].seg_bytes)
            if (sb > ((size_t)1 << 27)) return TCAM_E_ARG;
    // Huffman workgroups: the chunks of whole segments of one signature, <= 256 per group
    auto seg_nchunks = [](size_t bytes) -> int {
        const int64_t bits = (int64_t)bytes * 8;
        return (int)std::max<int64_t>(1, std::min<int64_t>(kHuffThreads,
                                                           (bits + kChunkBits - 1) / kChunkBits));
    };
    std::vector<std::vector<int>> sig_imgs(sigs.size());
    for (int i = 0; i < n; ++i) sig_imgs[img_sig[i]].push_back(i);
    int nhblk = 0, nchunk = 0;
    for (size_t s = 0; s < sigs.size(); ++s) {
        int fill = kHuffThreads;
        for (int i : sig_imgs[s])
            for (size_t sb : P[i].seg_bytes) {
                const int c = seg_nchunks(sb);
                if (fill + c > kHuffThreads) {
                    ++nhblk;
                    fill = 0;
                }
                fill += c;
                nchunk += c;
            }
    }

    JHdr h;
    memset(&h, 0, sizeof(h));
    h.magic = kMagic;
    h.n = n;
    h.ncomp_desc = ncd;
    h.nseg = nseg;
    h.nhblk = nhblk;
    h.nchunk = nchunk;
    for (int i = 0; i < n; ++i)
        h.max_runs = std::max(h.max_runs, P[i].h * ((P[i].w + 3) / 4));
    h.ntab = (int)tabs.size();
    h.total_blocks = (int)total_blocks;
    h.total_pixels = total_pix;
    int64_t off = al16(sizeof(JHdr));
    h.off_img = off;
    off = al16(off + (int64_t)n * sizeof(JImg));
    h.off_comp = off;
    off = al16(off + (int64_t)ncd * sizeof(JComp));
    h.off_seg = off;
    off = al16(off + (int64_t)nseg * sizeof(JSeg));
    h.off_hblk = off;
    off = al16(off + (int64_t)nhblk * sizeof(JHBlk));
    h.off_chunk = off;
    off = al16(off + (int64_t)nchunk * sizeof(JChunk));
    h.off_tab = off;
    off = al16(off + (int64_t)tabs.size() * sizeof(JTab));
    h.off_q = off;
    off = al16(off + (int64_t)ncd * 64 * 4);
    h.off_bytes = off;
    off = al16(off + bytes + 256);   // bit-reader blocks over-read < 192 bytes
    h.blob_bytes = off;
    h.coef_bytes = coef * 2;
    h.plane_bytes = plane;
    h.out_bytes = out;
    sizes[0] = h.blob_bytes;
    sizes[1] = al16(h.coef_bytes) + h.plane_bytes;   // device workspace
    sizes[2] = h.out_bytes;
    sizes[3] = total_blocks;
    if (!blob) return 0;
    if (cap < (size_t)h.blob_bytes) return TCAM_E_NOMEM;

    uint8_t* B = (uint8_t*)blob;
    memset(B, 0, h.off_bytes);
    memcpy(B, &h, sizeof(h));
    JImg* imgs = (JImg*)(B + h.off_img);
    JComp* comps = (JComp*)(B + h.off_comp);
    JSeg* segs = (JSeg*)(B + h.off_seg);
    JHBlk* hbs = (JHBlk*)(B + h.off_hblk);
    JChunk* chs = (JChunk*)(B + h.off_chunk);
    memcpy(B + h.off_tab, tabs.data(), tabs.size() * sizeof(JTab));
    int* qs = (int*)(B + h.off_q);

    int cd = 0;
    int64_t fb = 0, co = 0, po = 0, oo = 0, pf = 0;
    std::vector<int64_t> seg_off_img(n);
    int64_t bo = 0;
    for (int i = 0; i < n; ++i) {
        const Parsed& p = P[i];
        const Geo& g = G[i];
        JImg& im = imgs[i];
        im.w = p.w;
        im.h = p.h;
        im.ncomp = p.nc;
        if (p.nc == 1) {
            im.cs = 0;
        } else if (p.jfif) {
            im.cs = 1;
        } else if (p.adobe >= 0) {
            im.cs = p.adobe == 0 ? 2 : 1;
        } else {
            im.cs = (p.cid[0] == 82 && p.cid[1] == 71 && p.cid[2] == 66) ? 2 : 1;
        }
        im.hmax = g.hmax;
        im.vmax = g.vmax;
        im.mcus_x = g.mx;
        im.mcus_y = g.my;
        im.comp0 = cd;
        im.out_off = oo;
        im.pix_first = pf;
        oo += (int64_t)p.w * p.h * 3;
        pf += (int64_t)p.w * p.h;
        for (int c = 0; c < p.nc; ++c, ++cd) {
            JComp& k = comps[cd];
            k.img = i;
            k.hs = g.hs[c];
            k.vs = g.vs[c];
            k.bw = g.mx * g.hs[c];
            k.bh = g.my * g.vs[c];
            k.dsw = (int)(((int64_t)p.w * g.hs[c] + g.hmax - 1) / g.hmax);
            k.dsh = (int)(((int64_t)p.h * g.vs[c] + g.vmax - 1) / g.vmax);
            k.first_block = (int)fb;
            k.qoff = cd * 64;
            k.dc_slot = img_slots[i][2 * c];
            k.ac_slot = img_slots[i][2 * c + 1];
            k.stride = k.bw * 8;
            k.coef_off = co;
            k.plane_off = po;
            const int64_t nb = (int64_t)k.bw * k.bh;
            fb += nb;
            co += nb * 64;
            po += al16(nb * 64);
            for (int z = 0; z < 64; ++z) qs[cd * 64 + z] = p.quant[p.tq[c]][z];
        }
        // copy + unstuff the entropy bytes, one 16-byte-aligned run per segment
        seg_off_img[i] = bo;
        uint8_t* dst = B + h.off_bytes;
        int64_t cur = bo;
        std::vector<int64_t> starts(1, bo);
        scan_entropy(
            data[i], len[i], p.ent,
            [&](const uint8_t* s, size_t m) {
                memcpy(dst + cur, s, m);
                cur += (int64_t)m;
            },
            [&]() {
                const int64_t e = al16(cur);
                memset(dst + cur, 0, e - cur);
                cur = e;
                starts.push_back(cur);
            });
        const int64_t e = al16(cur);
        memset(dst + cur, 0, e - cur);
        bo = e;
    }
    memset(B + h.off_bytes + bo, 0, h.blob_bytes - h.off_bytes - bo);

    // segments ordered by signature, split into chunks; workgroups of whole segments
    int si = 0, hi = -1, ci = 0;
    for (size_t s = 0; s < sigs.size(); ++s) {
        int fill = kHuffThreads;
        for (int i : sig_imgs[s]) {
            const Parsed& p = P[i];
            const Geo& g = G[i];
            const int64_t total = (int64_t)g.mx * g.my;
            const int64_t ri = p.ri ? p.ri : total;
            int64_t o = seg_off_img[i];
            for (size_t k = 0; k < p.seg_bytes.size(); ++k) {
                JSeg& sg = segs[si];
                sg.img = i;
                sg.mcu0 = (int)(k * ri);
                sg.nmcu = (int)std::min<int64_t>(ri, total - (int64_t)k * ri);
                sg.nchunks = (int)(al16((int64_t)p.seg_bytes[k]) / 16);
                sg.byte_off = o;
                o += al16((int64_t)p.seg_bytes[k]);
                const int nc = seg_nchunks(p.seg_bytes[k]);
                if (fill + nc > kHuffThreads) {
                    JHBlk& hb = hbs[++hi];
                    hb.ch0 = ci;
                    hb.nch = 0;
                    hb.ntabs = (int)sigs[s].size();
                    for (size_t t = 0; t < sigs[s].size(); ++t) hb.tab[t] = sigs[s][t];
                    fill = 0;
                }
                const int bits = (int)(p.seg_bytes[k] * 8);
                const int step = (bits + nc - 1) / nc;
                for (int c = 0; c < nc; ++c, ++ci) {
                    chs[ci].seg = si;
                    chs[ci].bit0 = std::min(bits, c * step);
                    chs[ci].bit1 = c == nc - 1 ? bits : std::min(bits, (c + 1) * step);
                }
                hbs[hi].nch += nc;
                fill += nc;
                ++si;
            }
        }
    }
    return 0;
}

static int* g_jpeg_dbg = nullptr;

// Diagnostics: the next decodes write per Huffman workgroup 4 ints: fixpoint rounds, their clock cycles, write-pass cycles and blocks of lane 0,
// into dev_rounds[0 .. number of workgroups) (NULL turns it off).  Returns the workgroup
// count of the packed blob host_blob (or 0).
extern "C" int tcam_jpeg_debug_rounds(const void* host_blob, int* dev_rounds) {
    g_jpeg_dbg = dev_rounds;
    const JHdr* h = (const JHdr*)host_blob;
    return (h && h->magic == kMagic) ? h->nhblk : 0;
}

extern "C" int tcam_jpeg_decode(const void* host_blob, const void* dev_blob, void* ws,
                                size_t ws_bytes, uint8_t* out, void* stream) {
    const JHdr* h = (const JHdr*)host_blob;
    if (!h || h->magic != kMagic || !dev_blob) return TCAM_E_ARG;
    if (h->n == 0) return 0;
    if (!ws || !out) return TCAM_E_ARG;
    const int64_t need = al16(h->coef_bytes) + h->plane_bytes;
    if ((int64_t)ws_bytes < need) return TCAM_E_NOMEM;
    hipStream_t st = as_stream(stream);
    int16_t* coef = (int16_t*)ws;
    uint8_t* planes = (uint8_t*)ws + al16(h->coef_bytes);
    hipError_t e = hipMemsetAsync(coef, 0, h->coef_bytes, st);
    if (e != hipSuccess) return (int)e;
    const uint8_t* b = (const uint8_t*)dev_blob;
    hipLaunchKernelGGL(jpeg_huff_kernel, dim3(h->nhblk), dim3(kHuffThreads), 0, st, b, coef,
                       g_jpeg_dbg);
    TCAM_CHECK_LAUNCH();
    hipLaunchKernelGGL(jpeg_dc_kernel, dim3(h->nseg * 3), dim3(256), 0, st, b, coef);
    TCAM_CHECK_LAUNCH();
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3(cdiv(h->total_blocks, kIdctBlocks)), dim3(256),
                       0, st, b, (const int16_t*)coef, planes);
    TCAM_CHECK_LAUNCH();
    hipLaunchKernelGGL(jpeg_color_kernel, dim3(cdiv(h->max_runs, 256), h->n), dim3(256), 0, st,
                       b, (const uint8_t*)planes, out);
    TCAM_CHECK_LAUNCH();
    return 0;
}
