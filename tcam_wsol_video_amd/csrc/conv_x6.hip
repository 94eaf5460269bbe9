// Implicit-GEMM convolution at fp32 accuracy on the bf16 MFMA pipe (gfx950).
//
// Every fp32 value x is carried as three bf16 parts x = hi + mid + lo
// (hi = rne(x), mid = rne(x - hi), lo = x - hi - mid; the decomposition is
// exact: 8 + 8 + 8 significand bits cover fp32's 24).  A product a*b keeps
// the six cross terms of order <= 2
//     ah*bh + ah*bm + am*bh + ah*bl + am*bm + al*bh
// (the dropped terms are below 2^-24 |a b|), each an exact bf16 x bf16
// product accumulated in fp32 by v_mfma_f32_32x32x16_bf16.  Six of those
// (6 x 32 cycles for 32x32x16) replace eight v_mfma_f32_32x32x2_f32
// (8 x 64 cycles), so the ceiling is 2.67x the fp32 MFMA peak:
// 2.5 PF / 6 = 417 TF fp32-equivalent.
//
// Activations ("S3" layout, see include/tcam_hip.h): NHWC with channels in
// groups of 8, each group stored as [hi x8][mid x8][lo x8] bf16 = 48 bytes,
// i.e. a (B, H, W, C/8, 3, 8) bf16 array.  A 16-byte load is one part of one
// group: exactly the 8 consecutive k of one lane's MFMA operand.  The epilogue
// writes its output in the same form (split once per element here instead
// of once per consumer re-read).
//
// GEMM: out[n, m] = act(sum_k W[k, m] X[k, n] + bias[m] (+ res[n, m])),
// n = (frame, oh, ow), m = Cout, k = tap * Ctot + c (tap-major; c over the
// concatenated sources, every source C % 8 == 0 so a group of 8 k is one tap
// of one source).  Weights pre-split and packed (Kpad/32, 4, 3, Mpad, 8) bf16:
// element [kt][g][p][m][e] = part p of W[32 kt + 8 g + e][m].
//
// Block tile BM x BN, K-step 32 (4 groups), waves WM x WN each owning
// (BM/WM) x (BN/WN) as 32x32 subtiles.  One LDS stage + register prefetch of
// the next K-step (two barriers per step; several blocks per CU hide them), or
// two stages and one barrier.
//
// Scheduling: a plain grid (one block per tile) when the tile count fills the
// chip in whole waves; otherwise stream-K — a persistent grid of exactly the
// resident block count splits the flattened (tile, K-step) iteration space
// evenly; a tile cut between blocks has its fp32 partial sums reduced in fixed
// block order (deterministic) by whichever block arrives last, which then runs
// the epilogue.
#include <vector>

#include "common.h"
#include "s3_util.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BK = 32;
constexpr uint32_t OOB = 0x80000000u;
constexpr int SC1 = 16;  // buffer cache-policy bit: write-through store / coherent load

struct SrcX {
    int C, H, W, stride, up2, G;  // G = C / 8
};

struct ConvX {
    const void* sp[2];
    uint32_t sbytes[2];
    SrcX s[2];
    int c0, Ctot;
    const void* wt;
    uint32_t wbytes;
    int Mpad;
    const float* bias;
    const float* wscale;  // FmtF16: per-output-channel weight scale (power of two)
    int* oflow;           // FmtF16: set to 1 when an output leaves the S2 range (or null)
    const void* res;
    void* out;
    int Cout, Gout, Hout, Wout, pad_h, pad_w, relu, KH, KW;
    int out_gs, out_go;  // output: groups per pixel (>= Gout) and this conv's group offset
    // grouped launch (tcam_conv2d_x6_multi, 16x16x32 tiles only): output groups
    // [dg1, dg2) go to out1 (out1_gs, out1_go), [dg2, Gout) to out2; dg1 = dg2 = Gout
    // when everything goes to out
    void* out1;
    void* out2;
    int out1_gs, out1_go, out2_gs, out2_go, dg1, dg2;
    int K, N, HWo, nk;
    int mtiles, ntiles_total, nblocks;
    // stream-K (sk_grid > 0): workspace of 2 partial slots per block + one
    // arrival counter per tile (counters are left at 0 after every launch)
    int sk_grid;
    float* sk_part;
    int* sk_cnt;
    long sk_part_bytes;
    int corder;  // LDS-DMA tiles: K-steps in (32-channel chunk, tap) order (see segment)
    int sk_req;  // (A/B, TCAM_CONV_TILE_MAP "...s<grid>") stream-K over this grid
    int ntres;   // residual read with the non-temporal policy (LDS-DMA tiles: the residual
                 // stream would evict the weight and input slices the next tiles re-read)
    int gm;   // tile order: bands of gm m-tiles (gm divides mtiles; 0/1 = n-major, below)
    int dbg;  // timing experiments only (tcam_conv_x6_debug): 1 = B from pixel 0, 2 = no
              // global loads in the K loop after the first step, 4 = tap-major K order,
              // 8 = no epilogue (no residual loads, no stores), 16 = no residual prefetch
              // before the last K-step, 32 = Cout <= 16 thin layers on the 32-row kernel,
              // 64 = non-temporal residual loads, 128 = non-temporal output stores (16x16
              // tiles' LDS-staged epilogue), 256 = m-major tile order
};

// stream-K workspace: [arrival counters, SK_CNT_BYTES][partial slots]
constexpr long SK_CNT_BYTES = 1L << 20;
constexpr long SK_WS_BYTES = SK_CNT_BYTES + (96L << 20);

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
constexpr int NT = 2;     // buffer cache-policy bit: non-temporal (streaming) access
__device__ __forceinline__ uint4 bload16_nt(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, NT));
}

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

// x = hi + mid + lo exactly; returns the three parts' bit patterns.
__device__ __forceinline__ void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
    const __bf16 bh = (__bf16)x;
    h = __builtin_bit_cast(uint16_t, bh);
    const float r1 = x - bf2f(h);
    const __bf16 bm = (__bf16)r1;
    m = __builtin_bit_cast(uint16_t, bm);
    const float r2 = r1 - bf2f(m);
    l = __builtin_bit_cast(uint16_t, (__bf16)r2);
}

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// Operand formats.  FmtX6: three bf16 parts (S3 activations, the x6 product: six cross
// terms).  FmtF16: two fp16 parts (S2 activations, x = h + l, 22 significand bits; the
// packed weights carry a per-output-channel power-of-two scale that the epilogue undoes;
// three cross terms al*bh + ah*bl + ah*bh on the fp16 MFMA, which runs at the bf16 rate).
struct FmtX6 {
    using Out = FmtX6;                  // output (and residual) format: see FmtF16S3
    static constexpr int NP = 3;        // parts per value
    static constexpr int NTERM = 6;     // MFMA products per K-step and subtile pair
    static constexpr int PL = 4 * NP;   // 16-B planes per 32-deep K-step (4 groups x parts)
    static constexpr int GB = 16 * NP;  // bytes per 8-channel group
    static constexpr bool SCALED = false;
    using V8 = bf16x8;
    // term t multiplies A part ta(t) by B part tb(t): small terms first, hi*hi last
    static constexpr int ta(int t) { return t == 0 ? 2 : (t == 2 || t == 3) ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 2 : (t == 2 || t == 4) ? 1 : 0; }
    static __device__ __forceinline__ floatx4 mfma16(V8 a, V8 b, floatx4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ void split(float y, uint32_t (&pt)[NP]) {
        split3(y, pt[0], pt[1], pt[2]);
    }
    // element (2k + hi16) of a group from its parts' 32-bit words k
    static __device__ __forceinline__ float join(const uint32_t (&w)[NP], int hi16) {
        const int sh = hi16 ? 16 : 0;
        return (bf2f((w[0] >> sh) & 0xffffu) + bf2f((w[1] >> sh) & 0xffffu)) +
               bf2f((w[2] >> sh) & 0xffffu);
    }
};
struct FmtF16 {
    using Out = FmtF16;
    static constexpr int NP = 2;
    static constexpr int NTERM = 3;
    static constexpr int PL = 4 * NP;
    static constexpr int GB = 16 * NP;
    static constexpr bool SCALED = true;
    using V8 = halfx8;
    static constexpr int ta(int t) { return t == 0 ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 1 : 0; }
    static __device__ __forceinline__ floatx4 mfma16(V8 a, V8 b, floatx4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ void split(float y, uint32_t (&pt)[NP]) {
        s2::split2(y, pt[0], pt[1]);
    }
    static __device__ __forceinline__ float join(const uint32_t (&w)[NP], int hi16) {
        return hi16 ? s2::h_hi(w[0]) + s2::h_hi(w[1]) : s2::h_lo(w[0]) + s2::h_lo(w[1]);
    }
};

// FmtH1: ONE fp16 part (S1 activations, autocast's fp16 operand: the AMP training path),
// one product ah*bh per K-step on the fp16 MFMA, accumulated in fp32; the output is rounded
// to fp16 (beyond 65504 -> inf, as an fp16 conv output under torch.cuda.amp.autocast).
struct FmtH1 {
    using Out = FmtH1;
    static constexpr int NP = 1;
    static constexpr int NTERM = 1;
    static constexpr int PL = 4 * NP;
    static constexpr int GB = 16 * NP;
    static constexpr bool SCALED = false;
    using V8 = halfx8;
    static constexpr int ta(int) { return 0; }
    static constexpr int tb(int) { return 0; }
    static __device__ __forceinline__ floatx4 mfma16(V8 a, V8 b, floatx4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ void split(float y, uint32_t (&pt)[NP]) {
        pt[0] = s2::hbits(y);
    }
    static __device__ __forceinline__ float join(const uint32_t (&w)[NP], int hi16) {
        return hi16 ? s2::h_hi(w[0]) : s2::h_lo(w[0]);
    }
};

// FmtF16 operands with an S3 output (the x6 split): the f16x3 data gradient of the
// fp32-accurate training step, whose input dy is a per-channel power-of-two scaled S2 copy
// (the packed weights divide the scales out exactly) and whose output — an activation
// gradient, ~1e-7 — must not be stored in fp16 parts.
struct FmtF16S3 : FmtF16 {
    using Out = FmtX6;
};

// The S2 representable range: |y| > 65504 has no fp16 hi part (the epilogue flags it).
__device__ __forceinline__ bool f16_overflow(float y) { return fabsf(y) > 65504.f; }



// ---- 16x16x32 MFMA helpers shared by both tile families (M16 = true) ----
// A wave owns (WTM/16) x (WTN/16) 16x16 subtiles.  The A rows of each 32-row
// block are read in the order that makes lane (q = lane/16) of the pair of
// M-subtiles (2t, 2t+1) hold the 8 channels of group q: MFMA row 4q + e of
// subtile 2t + s is channel 8q + 4s + e, so the epilogue needs no lane
// exchange.  A planes are offset by APAD x 16 B per K-group so this permuted
// ds_read_b128 pattern is free of bank conflicts.
struct NoHook {
    __device__ void operator()(int) const {}
};

// This wave's fragments of one K-step (A rows in the channel-grouped order above).
template <class F, int BM, int BN, int WM, int WN, int APAD>
__device__ __forceinline__ void frag16(const uint4* As, const uint4* Bs,
                                       typename F::V8 (&fa)[BM / WM / 16][F::NP],
                                       typename F::V8 (&fb)[BN / WN / 16][F::NP]) {
    using V8 = typename F::V8;
    constexpr int WTM = BM / WM, WTN = BN / WN, T16M = WTM / 16, T16N = WTN / 16;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int q = lane >> 4, c16 = lane & 15;
    const int arow = 8 * (c16 >> 2) + (c16 & 3);
#pragma unroll
    for (int i = 0; i < T16M; ++i)
#pragma unroll
        for (int pp = 0; pp < F::NP; ++pp)
            fa[i][pp] = __builtin_bit_cast(
                V8, As[(q * F::NP + pp) * BM + q * APAD + wm * WTM + 32 * (i >> 1) + 4 * (i & 1) +
                       arow]);
#pragma unroll
    for (int j = 0; j < T16N; ++j)
#pragma unroll
        for (int pp = 0; pp < F::NP; ++pp)
            fb[j][pp] = __builtin_bit_cast(V8, Bs[(q * F::NP + pp) * BN + wn * WTN + j * 16 + c16]);
}

// The F::NTERM cross terms of one K-step on 16x16x32: term-major (T16M x T16N independent
// accumulators between dependent MFMAs); small terms first, hi*hi last.
// hook(t) runs after the MFMAs of term t (sched_barrier-fenced when a hook is given).
template <class F, int T16M, int T16N, class Hook = NoHook>
__device__ __forceinline__ void mfma6(const typename F::V8 (&fa)[T16M][F::NP],
                                      const typename F::V8 (&fb)[T16N][F::NP],
                                      floatx4 (&acc)[T16M][T16N], Hook hook = Hook()) {
#pragma unroll
    for (int t = 0; t < F::NTERM; ++t) {
#pragma unroll
        for (int i = 0; i < T16M; ++i)
#pragma unroll
            for (int j = 0; j < T16N; ++j)
                acc[i][j] = F::mfma16(fa[i][F::ta(t)], fb[j][F::tb(t)], acc[i][j]);
        if constexpr (!std::is_same<Hook, NoHook>::value) {
            __builtin_amdgcn_sched_barrier(0);
            hook(t);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <class F, int BM, int BN, int WM, int WN, int APAD, class Hook = NoHook>
__device__ __forceinline__ void mma16(const uint4* As, const uint4* Bs,
                                      floatx4 (&acc)[BM / WM / 16][BN / WN / 16],
                                      Hook hook = Hook()) {
    constexpr int T16M = BM / WM / 16, T16N = BN / WN / 16;
    typename F::V8 fa[T16M][F::NP], fb[T16N][F::NP];
    frag16<F, BM, BN, WM, WN, APAD>(As, Bs, fa, fb);
    mfma6<F, T16M, T16N>(fa, fb, acc, hook);
}

// The 32x32x16 form: lane (r32, h) reads the A rows / B columns of K-group 2 cc + h (APAD 0).
template <class F, int BM, int BN, int WM, int WN>
__device__ __forceinline__ void mma32(const uint4* As, const uint4* Bs,
                                      floatx16 (&acc)[BM / WM / 32][BN / WN / 32], int h) {
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32, NP = F::NP;
    using V8 = typename F::V8;
    const int r32 = threadIdx.x & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WN, wn = wave % WN;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
        const int g = 2 * cc + h;
        V8 fa[TM][NP], fb[TN][NP];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int pp = 0; pp < NP; ++pp)
                fa[i][pp] = __builtin_bit_cast(V8, As[(g * NP + pp) * BM + wm * WTM + i * 32 + r32]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int pp = 0; pp < NP; ++pp)
                fb[j][pp] = __builtin_bit_cast(V8, Bs[(g * NP + pp) * BN + wn * WTN + j * 32 + r32]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                floatx16 a = acc[i][j];
#pragma unroll
                for (int t = 0; t < F::NTERM; ++t) a = F::mfma32(fa[i][F::ta(t)], fb[j][F::tb(t)], a);
                acc[i][j] = a;
            }
    }
}

// Lane (q, c16) holds, for each 32-row block t of its wave tile, the 8 channels
// of group 4t + q at pixel column c16: subtile 2t gives channels 0..3, 2t+1 4..7.
//
// The epilogue goes through LDS (the K loop's ring is free once every wave has passed the
// barrier below).  Per 32-row block, a wave's 4 output groups of one pixel are 192
// contiguous bytes of the S3 tensor; the wave stages its WTN pixels as LDS rows of those
// 192 B, so the residual is read and the output written as whole pixel rows (one wave
// instruction covers 5.3 rows) instead of 16-B pieces of 16 pixels at a 48-B stride, the
// shape that kept the wide 1x1 layers' epilogues far below HBM rate.  Rows are padded to
// 13 x 16 B where LDS allows (the lanes' 48-B group reads then fall in distinct banks).
// The arithmetic (bias, residual, ReLU, split) is the register epilogue's, bit for bit.
// 16-pixel subtiles per staged chunk: the most that fit the tile's LDS (whole wave tile on
// the tiles in use; two chunks on the register-staged 64x128)
// Epilogue arithmetic shared by every tile: bias (+ the FmtF16 weight scale), residual,
// ReLU, split into the output format's parts (one uint4 per part of an 8-channel group).
template <class F>
__device__ __forceinline__ void load_bias_scale(const ConvX& p, int g, float (&bb)[8],
                                                float (&sc)[8]) {
    const float4 b0 = *reinterpret_cast<const float4*>(p.bias + 8 * g);
    const float4 b1 = *reinterpret_cast<const float4*>(p.bias + 8 * g + 4);
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
    bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    if constexpr (F::SCALED) {
        const float4 s0 = *reinterpret_cast<const float4*>(p.wscale + 8 * g);
        const float4 s1 = *reinterpret_cast<const float4*>(p.wscale + 8 * g + 4);
        sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
        sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) sc[e] = 1.f;
    }
}

// acc * scale + bias (FmtX6: acc + bias, the x6 epilogue's arithmetic bit for bit; the
// FmtF16 scale is a power of two, so acc * scale is exact)
template <class F>
__device__ __forceinline__ float epi_val(float acc, float sc, float b) {
    if constexpr (F::SCALED) return acc * sc + b;
    else return acc + b;
}

// x += the residual group held in its parts' 16-B pieces
template <class F>
__device__ __forceinline__ void add_group(float (&x)[8], const uint4 (&r)[F::NP]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t w[F::NP];
#pragma unroll
        for (int pp = 0; pp < F::NP; ++pp)
            w[pp] = k == 0 ? r[pp].x : k == 1 ? r[pp].y : k == 2 ? r[pp].z : r[pp].w;
        x[2 * k] += F::join(w, 0);
        x[2 * k + 1] += F::join(w, 1);
    }
}

// ReLU (NaN-propagating) + split of 8 channels into the parts' 16-B pieces of the OUTPUT
// format F (= the tile format's Out); S2 outputs flag values beyond the S2 range
template <class F>
__device__ __forceinline__ void split_group(const ConvX& p, const float (&x)[8],
                                            uint4 (&o)[F::NP]) {
    uint32_t pt[8][F::NP];
    bool bad = false;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float y = p.relu ? relu_nan(x[e]) : x[e];
        if constexpr (F::SCALED) bad |= f16_overflow(y);
        F::split(y, pt[e]);
    }
#pragma unroll
    for (int pp = 0; pp < F::NP; ++pp)
        o[pp] = make_uint4(pt[0][pp] | (pt[1][pp] << 16), pt[2][pp] | (pt[3][pp] << 16),
                           pt[4][pp] | (pt[5][pp] << 16), pt[6][pp] | (pt[7][pp] << 16));
    if constexpr (F::SCALED) {
        if (bad && p.oflow) *p.oflow = 1;
    }
}

constexpr int epi_chunk(int t16n, int nw, int cap, int pl) {
    for (int jc = t16n; jc > 1; --jc)
        if (t16n % jc == 0 && nw * jc * 16 * pl <= cap) return jc;
    return 1;
}

template <class F, int BM, int BN, int WM, int WN, int LDS_CAP>
struct Epi16 {
    static constexpr int WTM = BM / WM, WTN = BN / WN, T16M = WTM / 16, T16N = WTN / 16;
    static constexpr int NTB = T16M / 2 > 0 ? T16M / 2 : 1;  // 32-row blocks per wave
    static constexpr int NW = WM * WN;
    using O = typename F::Out;                    // the output / residual format
    static constexpr int PL = O::PL, NP = O::NP;  // 16-B pieces per pixel of a 32-row block
    static constexpr int JC = epi_chunk(T16N, NW, LDS_CAP, PL);  // 16-pixel subtiles per chunk
    static constexpr int CPX = 16 * JC;                          // pixels per chunk
    // LDS row pitch (16-B units): one pad piece where LDS allows
    static constexpr int RP = (NW * CPX * (PL + 1) <= LDS_CAP) ? PL + 1 : PL;
    static constexpr int NI = CPX * PL / 64;  // wave instructions per row sweep
    static constexpr int NCH = NTB * (T16N / JC);  // staged chunks per wave
    // Residual pieces of the first NPF chunks are loaded into registers ahead of the
    // epilogue (issued before the tile's last K-step, so their HBM latency hides under its
    // MFMAs); a wave keeps at most PF_CAP x 16 B of them (more spills the deep tiles
    // during their last K-step).  Later chunks load in place.
    static constexpr int PF_CAP = 12;
    static constexpr int NPF = (NCH * NI <= PF_CAP) ? NCH : (PF_CAP / NI > 0 ? PF_CAP / NI : 1);
    struct Res {
        uint4 v[NPF][NI];
    };

    // residual pieces of chunk tc of this wave (16-B piece k = c % PL of pixel c / PL,
    // c = 64 i + lane)
    static __device__ __forceinline__ void chunk_load(const ConvX& p, int m0, int n0, int tc,
                                                      uint4 (&rv)[NI]) {
        const int lane = threadIdx.x & 63;
        const int wave = threadIdx.x >> 6;
        const int wm = wave / WN, wn = wave % WN;
        const int t = tc / (T16N / JC), jc = tc % (T16N / JC);
        const int g0 = (m0 + wm * WTM + 32 * t) / 8;
        const int nc0 = n0 + wn * WTN + jc * CPX;
        const rsrc_t rr = make_rsrc(p.res, p.res ? (uint32_t)p.N * p.Gout * O::GB : 0u);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = 64 * i + lane, pl = c / PL, k = c - PL * pl;
            const int n = nc0 + pl;
            const bool ok = n < p.N && g0 + k / NP < p.Gout;
            const uint32_t off = ok ? (uint32_t)((n * p.Gout + g0) * O::GB + 16 * k) : OOB;
            rv[i] = (p.ntres || (p.dbg & 64)) ? bload16_nt(rr, off) : bload16(rr, off);
        }
    }

    static __device__ __forceinline__ void res_load(const ConvX& p, int m0, int n0, Res& rv) {
        if (!p.res || (p.dbg & (8 | 16))) return;
#pragma unroll
        for (int tc = 0; tc < NPF; ++tc) chunk_load(p, m0, n0, tc, rv.v[tc]);
    }

    // rv: res_load's pieces (loaded by the caller before the last K-step); PRE = false:
    // rv is not used, every chunk loads its residual here (the stream-K kernel: there the
    // prefetched registers spill)
    template <bool PRE>
    static __device__ __forceinline__ void run(const ConvX& p, int m0, int n0,
                                               const floatx4 (&acc)[T16M][T16N], uint4* lds,
                                               const Res& rv) {
        static_assert(T16M % 2 == 0, "16x16 tiles hold whole 32-row blocks");
        static_assert(NW * CPX * RP <= LDS_CAP, "epilogue staging must fit the tile's LDS");
        if (p.dbg & 8) return;   // timing experiments only: no epilogue traffic
        const int tid = threadIdx.x;
        const int lane = tid & 63;
        const int wave = tid >> 6;
        const int wm = wave / WN, wn = wave % WN;
        const int q = lane >> 4, c16 = lane & 15;
        const int nw0 = n0 + wn * WTN;  // the wave's first pixel
        uint4* wl = lds + wave * (CPX * RP);
        uint8_t* outb = reinterpret_cast<uint8_t*>(p.out);
        __syncthreads();  // every wave has read its last K-step from the ring
#pragma unroll
        for (int tc = 0; tc < NCH; ++tc) {
            const int t = tc / (T16N / JC), jc = tc % (T16N / JC);
            const int g0 = (m0 + wm * WTM + 32 * t) / 8;  // the wave's 4 groups of this block
            // (no early break: the loop must unroll so rv is indexed at compile time)
            if (g0 >= p.Gout) continue;
            const int nc0 = nw0 + jc * CPX;  // the chunk's first pixel
            if (p.res) {
                // dbg 16 (A/B timing only): no prefetch, every chunk loads here
                // (two separate stores: a select between the two register arrays is
                // lowered to a select of their addresses, i.e. both go to scratch)
                if (!PRE || tc >= NPF || (p.dbg & 16)) {
                    uint4 rl[NI];
                    chunk_load(p, m0, n0, tc, rl);
#pragma unroll
                    for (int i = 0; i < NI; ++i) {
                        const int c = 64 * i + lane, pl = c / PL;
                        wl[pl * RP + (c - PL * pl)] = rl[i];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < NI; ++i) {
                        const int c = 64 * i + lane, pl = c / PL;
                        wl[pl * RP + (c - PL * pl)] = rv.v[tc < NPF ? tc : 0][i];
                    }
                }
            }
            const int g = g0 + q;
            if (g < p.Gout) {
                float bb[8], sc[8];
                load_bias_scale<F>(p, g, bb, sc);
#pragma unroll
                for (int jj = 0; jj < JC; ++jj) {
                    const int j = jc * JC + jj;
                    uint4* row = wl + (jj * 16 + c16) * RP + NP * q;
                    float x[8];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        x[e] = epi_val<F>(acc[2 * t][j][e], sc[e], bb[e]);
                        x[4 + e] = epi_val<F>(acc[2 * t + 1][j][e], sc[4 + e], bb[4 + e]);
                    }
                    if (p.res) {
                        uint4 rr[NP];
#pragma unroll
                        for (int pp = 0; pp < NP; ++pp) rr[pp] = row[pp];
                        add_group<O>(x, rr);
                    }
                    uint4 outp[NP];
                    split_group<O>(p, x, outp);
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp) row[pp] = outp[pp];
                }
            }
            // (LDS accesses of one wave execute in order: the sweep below reads what the
            // other lanes of this wave wrote above)
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int c = 64 * i + lane, pl = c / PL, k = c - PL * pl;
                const int n = nc0 + pl;
                const int g2 = g0 + k / NP;
                if (n < p.N && g2 < p.Gout) {
                    // destination of group g2 (one tensor unless this is a grouped launch)
                    uint8_t* ob = outb;
                    int gs = p.out_gs, go = p.out_go + g2;
                    if (g2 >= p.dg1) {
                        const bool two = g2 >= p.dg2;
                        ob = reinterpret_cast<uint8_t*>(two ? p.out2 : p.out1);
                        gs = two ? p.out2_gs : p.out1_gs;
                        go = two ? p.out2_go + g2 - p.dg2 : p.out1_go + g2 - p.dg1;
                    }
                    uint4* dst = reinterpret_cast<uint4*>(ob + (uint32_t)((n * gs + go) * O::GB +
                                                                        16 * (k % NP)));
                    if (p.dbg & 128) {
                        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, wl[pl * RP + k]),
                                                    reinterpret_cast<u32x4*>(dst));
                    } else {
                        *dst = wl[pl * RP + k];
                    }
                }
            }
        }
    }
};

// Flat view of a tile's accumulators (index r in [0, T::ACC), compile-time after
// unrolling): stream-K slabs and zeroing work on either MFMA shape.
template <class T>
__device__ __forceinline__ float acc_get(const typename T::Acc& a, int r) {
    if constexpr (T::M16_) {
        constexpr int TN16 = T::WTN / 16;
        return a[r / (TN16 * 4)][(r / 4) % TN16][r % 4];
    } else {
        return a[r / (T::TN * 16)][(r / 16) % T::TN][r % 16];
    }
}
template <class T>
__device__ __forceinline__ void acc_set(typename T::Acc& a, int r, float v) {
    if constexpr (T::M16_) {
        constexpr int TN16 = T::WTN / 16;
        a[r / (TN16 * 4)][(r / 4) % TN16][r % 4] = v;
    } else {
        a[r / (T::TN * 16)][(r / 16) % T::TN][r % 16] = v;
    }
}
template <class T>
__device__ __forceinline__ void acc_zero(typename T::Acc& a) {
#pragma unroll
    for (int r = 0; r < T::ACC; ++r) acc_set<T>(a, r, 0.f);
}

template <class F, int BM, int BN, int WM, int WN, int STAGES, bool M16 = false>
struct ConvTile {
    static constexpr int BM_ = BM, BN_ = BN;
    static constexpr int NP = F::NP, PL = F::PL;
    using V8 = typename F::V8;
    static constexpr bool M16_ = M16;
    static constexpr int APAD = M16 ? 4 : 0;  // see mma16
    static constexpr bool AUTO_SK = true;
    static constexpr int MIN_WAVES = 2;
    static constexpr int NT = 64 * WM * WN;
    static constexpr int WTM = BM / WM, WTN = BN / WN;
    static constexpr int TM = WTM / 32, TN = WTN / 32;
    static constexpr int A_CHUNKS = PL * BM;  // 16-B chunks per K-step
    static constexpr int A_PER = (A_CHUNKS + NT - 1) / NT;
    static constexpr int B_ITEMS = 4 * BN;    // (group, pixel) items, F::GB bytes each
    static_assert(B_ITEMS % NT == 0, "B items must divide evenly");
    static_assert(BN % 64 == 0, "a wave's items share one group");
    static constexpr int B_PER = B_ITEMS / NT;
    static constexpr int ACC = TM * TN * 16;  // accumulator floats per lane (either shape)
    using Acc = typename std::conditional<M16, floatx4[WTM / 16][WTN / 16],
                                          floatx16[TM][TN]>::type;
    static constexpr int A_UINT4 = PL * BM + 4 * APAD;  // one stage of A planes
    static constexpr int LDS_UINT4 = STAGES * (A_UINT4 + PL * BN);
    using Epi = Epi16<F, BM, BN, WM, WN, LDS_UINT4>;
    using Res = typename Epi::Res;
    static __device__ __forceinline__ void res_load(const ConvX& p, int m0, int n0, Res& rv) {
        if constexpr (M16) Epi::res_load(p, m0, n0, rv);
    }

    // Accumulate K-steps [kb, ke) of tile (m0, n0) into acc (zeroed here).  (No residual
    // prefetch hook here: its registers would cost these tiles a wave per SIMD; the epilogue
    // issues all of its residual loads up front instead.)
    static constexpr bool PREFETCH = false;
    template <class Pre>
    static __device__ __forceinline__ void segment(const ConvX& p, int m0, int n0, int kb,
                                                   int ke, Acc& acc, uint4* lds, Pre) {
        auto As_ = reinterpret_cast<uint4(*)[A_UINT4]>(lds);
        auto Bs_ = reinterpret_cast<uint4(*)[PL * BN]>(lds + STAGES * A_UINT4);
        const int tid = threadIdx.x;
        const int lane = tid & 63;
        const int wave = tid >> 6;
        const int wm = wave / WN, wn = wave % WN;
        const int r32 = lane & 31, h = lane >> 5;

        const rsrc_t rs0 = make_rsrc(p.sp[0], p.sbytes[0]);
        const rsrc_t rs1 = make_rsrc(p.sp[1], p.sbytes[1]);
        const rsrc_t rw = make_rsrc(p.wt, p.wbytes);

        // per-item B-loader state: the item's pixel and its group's (tap, c)
        int it_img[B_PER], it_oy[B_PER], it_ox[B_PER];
        bool it_nv[B_PER];
        int g_tap[B_PER], g_c[B_PER], g_kh[B_PER], g_kw[B_PER];
#pragma unroll
        for (int j = 0; j < B_PER; ++j) {
            const int it = tid + j * NT;
            const int n = n0 + it % BN;
            it_nv[j] = n < p.N;
            const int nn = it_nv[j] ? n : 0;
            it_img[j] = nn / p.HWo;
            const int hw = nn - it_img[j] * p.HWo;
            it_oy[j] = hw / p.Wout;
            it_ox[j] = hw - it_oy[j] * p.Wout;
            const int g = __builtin_amdgcn_readfirstlane(it / BN);  // wave-uniform
            const int k = kb * BK + 8 * g;
            const int tap = k / p.Ctot;
            g_c[j] = k - tap * p.Ctot;
            g_tap[j] = tap;
            g_kh[j] = tap / p.KW;
            g_kw[j] = tap - g_kh[j] * p.KW;
        }

        uint4 ra[A_PER];
        uint4 rb[B_PER][NP];

        auto gload = [&](int kt) {
#pragma unroll
            for (int j = 0; j < A_PER; ++j) {
                const int q = tid + j * NT;
                if (A_CHUNKS % NT == 0 || q < A_CHUNKS) {
                    const int gp = q / BM, m = q % BM;
                    const uint32_t off = (uint32_t)(((kt * PL + gp) * p.Mpad + m0 + m) * 16);
                    ra[j] = bload16(rw, off);
                }
            }
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int k = g_tap[j] * p.Ctot + g_c[j];
                const int si = g_c[j] >= p.c0 ? 1 : 0;
                const int c = si ? g_c[j] - p.c0 : g_c[j];
                const SrcX& s = p.s[si];
                const int iy = it_oy[j] * s.stride - p.pad_h + g_kh[j];
                const int ix = it_ox[j] * s.stride - p.pad_w + g_kw[j];
                const bool ok = it_nv[j] && k < p.K && (unsigned)iy < (unsigned)(s.H << s.up2) &&
                                (unsigned)ix < (unsigned)(s.W << s.up2);
                const uint32_t off = (p.dbg & 1) ? (uint32_t)(c >> 3) * F::GB :
                    ok ? (uint32_t)((((it_img[j] * s.H + (iy >> s.up2)) * s.W + (ix >> s.up2)) *
                                         s.G +
                                     (c >> 3)) *
                                    F::GB)
                       : OOB;
                const rsrc_t r = si ? rs1 : rs0;
                rb[j][0] = bload16(r, off);
#pragma unroll
                for (int pp = 1; pp < NP; ++pp) rb[j][pp] = bload16(r, ok ? off + 16u * pp : OOB);
                // advance this item's group to the next K-step
                int cc = g_c[j] + BK;
                while (cc >= p.Ctot) {
                    cc -= p.Ctot;
                    if (++g_kw[j] == p.KW) {
                        g_kw[j] = 0;
                        ++g_kh[j];
                    }
                    ++g_tap[j];
                }
                g_c[j] = cc;
            }
        };

        auto lstore = [&](int st) {
            uint4* As = As_[st];
            uint4* Bs = Bs_[st];
#pragma unroll
            for (int j = 0; j < A_PER; ++j) {
                const int q = tid + j * NT;
                if (A_CHUNKS % NT == 0 || q < A_CHUNKS) As[q + (q / (NP * BM)) * APAD] = ra[j];
            }
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int it = tid + j * NT;
                const int g = it / BN, n = it % BN;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp) Bs[(g * NP + pp) * BN + n] = rb[j][pp];
            }
        };

        auto compute = [&](int st) {
            const uint4* As = As_[st];
            const uint4* Bs = Bs_[st];
            if constexpr (M16) {
                mma16<F, BM, BN, WM, WN, APAD>(As, Bs, acc);
            } else {
                mma32<F, BM, BN, WM, WN>(As, Bs, acc, h);
            }
        };

        acc_zero<ConvTile>(acc);

        gload(kb);
        if constexpr (STAGES == 1) {
            for (int kt = kb; kt < ke; ++kt) {
                __syncthreads();
                lstore(0);
                __syncthreads();
                if (kt + 1 < ke && !(p.dbg & 2)) gload(kt + 1);
                compute(0);
            }
            __syncthreads();  // LDS free for the next segment
        } else {
            // stage (kt - kb) & 1 holds step kt; step kt + 1 is written into the
            // other stage after computing kt, which every wave finished reading
            // at kt - 1 (ordered by the barrier ending that step).
            __syncthreads();
            lstore(0);
            __syncthreads();
            for (int kt = kb; kt < ke; ++kt) {
                const int st = (kt - kb) & 1;
                if (kt + 1 < ke && !(p.dbg & 2)) gload(kt + 1);
                compute(st);
                if (kt + 1 < ke) lstore(st ^ 1);
                __syncthreads();
            }
        }
    }

    // Epilogue.  In subtile (i, j) lane (r32, h) holds pixel n = column r32 and
    // channels 8q + 4h + (0..3), q = 0..3 (acc[4q + e]).  Two v_permlane32_swap
    // per register pair hand each lane two whole 8-channel groups: lane h = 0
    // gets groups 0, 1 and lane h = 1 groups 2, 3 of the subtile, so a lane
    // reads its residual and writes its output as 96 contiguous bytes
    // (6 x 16 B) and a lane pair covers the pixel's 192 B of the subtile.
    template <bool PRE>
    static __device__ __forceinline__ void epilogue(const ConvX& p, int m0, int n0,
                                                    const Acc& acc, uint4* lds, const Res& rv) {
        if constexpr (M16) {
            Epi::template run<PRE>(p, m0, n0, acc, lds, rv);
        } else {
            epilogue32(p, m0, n0, acc);
        }
    }

    static __device__ __forceinline__ void epilogue32(const ConvX& p, int m0, int n0,
                                                      const floatx16 (&acc)[TM][TN]) {
        if (p.dbg & 8) return;   // timing experiments only: no epilogue traffic
        const int tid = threadIdx.x;
        const int lane = tid & 63;
        const int wave = tid >> 6;
        const int wm = wave / WN, wn = wave % WN;
        const int r32 = lane & 31, h = lane >> 5;
        using O = typename F::Out;
        constexpr int ONP = O::NP;
        const rsrc_t rr = make_rsrc(p.res, p.res ? (uint32_t)p.N * p.Gout * O::GB : 0u);
        uint8_t* outb = reinterpret_cast<uint8_t*>(p.out);
        // All residual loads first (one batch in flight; the store stream
        // below may alias from the compiler's view, which would otherwise
        // serialise each load behind the previous group's stores).
        uint4 rv[TM][TN][2][ONP];
        if (p.res) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WTN + j * 32 + r32;
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int g0 = (m0 + wm * WTM + i * 32) / 8 + 2 * h;
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const bool ok = n < p.N && g0 + t < p.Gout;
                        const uint32_t off = ok ? (uint32_t)((n * p.Gout + g0 + t) * O::GB) : OOB;
#pragma unroll
                        for (int pp = 0; pp < ONP; ++pp)
                            rv[i][j][t][pp] = bload16(rr, ok ? off + 16u * pp : OOB);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WTN + j * 32 + r32;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                float v[16];  // v[8t + e]: channel e of group t (t = 0, 1) of this lane
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // pair (q0, q2): lo lanes keep q0's channel e and receive 4 + e;
                    // hi lanes receive q2's channel 16 + e and keep 20 + e.
                    const auto s02 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(acc[i][j][e]), __float_as_uint(acc[i][j][8 + e]), false,
                        false);
                    const auto s13 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(acc[i][j][4 + e]), __float_as_uint(acc[i][j][12 + e]),
                        false, false);
                    v[e] = __uint_as_float(s02[0]);
                    v[4 + e] = __uint_as_float(s02[1]);
                    v[8 + e] = __uint_as_float(s13[0]);
                    v[12 + e] = __uint_as_float(s13[1]);
                }
                if (n >= p.N) continue;
                const int g0 = (m0 + wm * WTM + i * 32) / 8 + 2 * h;  // this lane's first group
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int g = g0 + t;
                    if (g >= p.Gout) continue;
                    float bb[8], sc[8];
                    load_bias_scale<F>(p, g, bb, sc);
                    float x[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) x[e] = epi_val<F>(v[8 * t + e], sc[e], bb[e]);
                    const uint32_t off = (uint32_t)((n * p.out_gs + p.out_go + g) * O::GB);
                    if (p.res) add_group<O>(x, rv[i][j][t]);
                    uint4 o[ONP];
                    split_group<O>(p, x, o);
#pragma unroll
                    for (int pp = 0; pp < ONP; ++pp)
                        *reinterpret_cast<uint4*>(outb + off + 16 * pp) = o[pp];
                }
            }
        }
    }
};

// LDS-DMA pipelined tile for "aligned" convolutions (every source C % 32 == 0,
// so each 32-deep K-step is 32 consecutive channels of ONE tap of ONE source:
// 192 contiguous bytes per pixel).  Loads go global -> LDS by
// buffer_load_dwordx4 ... lds (no VGPR staging, no ds_write; out-of-range
// offsets read 0, which implements the padding), into a STAGES-deep ring
// issued STAGES-1 steps ahead; one barrier per K-step, waited with a counted
// vmcnt so the younger steps stay in flight across it.  All LDS is one array
// (cdna_hip_programming.md §5 'Pipelining across barriers').
//
// M16 = true: the same pipeline on v_mfma_f32_16x16x32_bf16 (one instruction
// covers the whole 32-deep K-step; the 16x16 shape holds a higher clock on
// random data than 32x32x16 at equal cycles per FLOP, MI355X_MICROARCH.md
// 'DVFS give-back').  A wave owns (WTM/16) x (WTN/16) 16x16 subtiles.  The A
// rows of each 32-row block are read in the order that makes lane (q = lane/16)
// of the pair of M-subtiles (2t, 2t+1) hold the 8 channels of group q: MFMA row
// 4q' + e of subtile 2t + s is channel 8q' + 4s + e.  The A planes are offset
// by 4 x 16 B per K-group so that this permuted ds_read_b128 pattern stays
// free of bank conflicts.
struct KPos {
    int c, kh, kw;  // K-step position: first channel, tap row, tap column
};

template <class F, int BM, int BN, int WM, int WN, int STAGES, bool M16 = false,
          bool IL = false, bool LW = false, bool PP = false, bool FP = false>
struct ConvTileG {
    static constexpr int BM_ = BM, BN_ = BN;
    static constexpr int NP = F::NP, PL = F::PL;
    static constexpr bool M16_ = M16;
    static constexpr int APAD = M16 ? 4 : 0;    // uint4 offset per K-group plane (A)
    static constexpr int T16M = BM / WM / 16, T16N = BN / WN / 16;
    static constexpr bool AUTO_SK = false;  // slower with stream-K on full waves (pipeline
                                            // restarts); see launch_t for the under-filled case
    static constexpr int MIN_WAVES = 2;
    static constexpr int NT = 64 * WM * WN;
    static constexpr int NW = WM * WN;
    static constexpr int WTM = BM / WM, WTN = BN / WN;
    static constexpr int TM = WTM / 32, TN = WTN / 32;
    static constexpr int ACC = TM * TN * 16;
    static constexpr int A_INS = PL * BM / 64;  // 1-KiB LDS-DMA pieces per K-step
    static constexpr int B_INS = PL * BN / 64;
    static_assert(A_INS % NW == 0 && B_INS % NW == 0, "pieces split evenly over waves");
    static constexpr int A_PW = A_INS / NW, B_PW = B_INS / NW;
    static constexpr int PW = A_PW + B_PW;      // pieces per wave per K-step
    // LW: only the first half of the waves issue the LDS-DMA pieces (twice as many each):
    // waves w and w + NW/2 share a SIMD, so one of them issues while the other runs MFMAs
    // instead of both stalling on the issue burst after the barrier
    static constexpr int LWN = LW ? NW / 2 : NW;  // issuing waves
    static constexpr int A_PWI = A_INS / LWN, B_PWI = B_INS / LWN, PWI = A_PWI + B_PWI;
    static_assert(A_INS % LWN == 0 && B_INS % LWN == 0, "pieces split evenly");
    static constexpr int STAGE_UINT4 = PL * (BM + BN) + 4 * APAD;
    static constexpr int B_OFF = PL * BM + 4 * APAD;  // B planes after the (padded) A planes
    static constexpr int LDS_UINT4 = STAGES * STAGE_UINT4;
    static constexpr int BH = BN / 64;          // pixel slots per lane (one per 64-pixel half)
    // accumulators: 32x32 subtiles (floatx16) or 16x16 subtiles (floatx4)
    using Acc = typename std::conditional<M16, floatx4[T16M][T16N], floatx16[TM][TN]>::type;
    static constexpr bool PREFETCH = true;   // residual loads issued before the last K-step
    using Epi = Epi16<F, BM, BN, WM, WN, LDS_UINT4>;
    using Res = typename Epi::Res;
    static __device__ __forceinline__ void res_load(const ConvX& p, int m0, int n0, Res& rv) {
        if constexpr (M16) Epi::res_load(p, m0, n0, rv);
    }

    static __device__ __forceinline__ void wait_vm(int outstanding_steps) {
        // vmcnt = pieces of the younger steps still allowed in flight (an issuing wave's
        // count; the other waves of an LW tile have none outstanding)
        if constexpr (STAGES >= 5) {
            if (outstanding_steps >= 4) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 * PWI) : "memory"); return; }
        }
        if constexpr (STAGES >= 4) {
            if (outstanding_steps >= 3) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * PWI) : "memory"); return; }
        }
        if constexpr (STAGES >= 3) {
            if (outstanding_steps >= 2) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PWI) : "memory"); return; }
        }
        if (outstanding_steps >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PWI) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

    template <class Pre>
    static __device__ __forceinline__ void segment(const ConvX& p, int m0, int n0, int kb,
                                                   int ke, Acc& acc, uint4* lds, Pre pre_last) {
        const int tid = threadIdx.x;
        const int lane = tid & 63;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int wm = wave / WN, wn = wave % WN;
        const int r32 = lane & 31, h = lane >> 5;

        const rsrc_t rs0 = make_rsrc(p.sp[0], p.sbytes[0]);
        const rsrc_t rs1 = make_rsrc(p.sp[1], p.sbytes[1]);
        const rsrc_t rw = make_rsrc(p.wt, p.wbytes);

        // this lane's pixels (one per 64-pixel half of the tile)
        int px_img[BH], px_oy[BH], px_ox[BH];
        bool px_ok[BH];
#pragma unroll
        for (int q = 0; q < BH; ++q) {
            const int n = n0 + q * 64 + lane;
            px_ok[q] = n < p.N;
            const int nn = px_ok[q] ? n : 0;
            px_img[q] = nn / p.HWo;
            const int hw = nn - px_img[q] * p.HWo;
            px_oy[q] = hw / p.Wout;
            px_ox[q] = hw - px_oy[q] * p.Wout;
        }
        // running (tap -> kh, kw; channel c) of the K-step being issued (block-uniform).
        // K-step order: with several taps (p.corder), 32-channel chunk outer and tap inner —
        // the KH*KW steps of one chunk read the same 32 channels of overlapping pixel
        // windows back to back, so the shifted re-reads hit L2 instead of coming from
        // beyond it (tap-major order re-reads each input Ctot/32 steps later).  The packed
        // weights stay tap-major: step (chunk, tap) reads 32-row block tap*Ctot/32 + chunk.
        const int KHW = p.KH * p.KW, CT = p.Ctot / BK;
        // The position is a value carried by the K loop (never captured by reference:
        // an address-taken position was kept in scratch and re-loaded every K-step).
        KPos pos;
        {
            int tap;
            if (p.corder) {
                tap = kb % KHW;
                pos.c = (kb / KHW) * BK;
            } else {
                const int k = kb * BK;
                tap = k / p.Ctot;
                pos.c = k - tap * p.Ctot;
            }
            pos.kh = tap / p.KW;
            pos.kw = tap - pos.kh * p.KW;
        }
        auto next = [&p](KPos q) {
            if (p.corder) {
                if (++q.kw == p.KW) {
                    q.kw = 0;
                    if (++q.kh == p.KH) {
                        q.kh = 0;
                        q.c += BK;
                    }
                }
            } else {
                q.c += BK;
                if (q.c >= p.Ctot) {
                    q.c -= p.Ctot;
                    if (++q.kw == p.KW) {
                        q.kw = 0;
                        ++q.kh;
                    }
                }
            }
            return q;
        };

        // pieces [lo, hi) of this wave's PW LDS-DMA pieces of one K-step (A: 0 .. A_PW-1,
        // B: A_PW .. PW-1); lo / hi are compile-time after inlining
        auto issue_parts = [&](int kt, int stage, const KPos ps, int lo, int hi) {
            if (LW && wave >= LWN) return;
            const int c_is = ps.c, kh_is = ps.kh, kw_is = ps.kw;
            uint4* st = lds + stage * STAGE_UINT4;
            // A: weights, planes (g, p) x BM rows
#pragma unroll
            for (int i = 0; i < A_PWI; ++i) {
                if (i < lo || i >= hi) continue;
                const int idx = wave * A_PWI + i;
                const int plane = idx / (BM / 64), part = idx % (BM / 64);
                const int kblk = p.corder ? (kh_is * p.KW + kw_is) * CT + (c_is >> 5) : kt;
                const uint32_t off =
                    (uint32_t)(((kblk * PL + plane) * p.Mpad + m0 + part * 64 + lane) * 16);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rw,
                    (__attribute__((address_space(3))) void*)(st + plane * BM + (plane / NP) * APAD +
                                                              part * 64),
                    16, off, 0, 0, 0);
            }
            // B: activations, planes (g, p) x BN pixels; K-step = one tap of one source.
            // The source's fields are scalar selects between the two kernel-argument
            // copies: indexing p.s[si] with a runtime si would copy the struct to scratch
            // and put scratch loads (waited with vmcnt, i.e. behind the in-flight LDS-DMA
            // pieces) into the K loop.
            const bool s1 = __builtin_amdgcn_readfirstlane(c_is) >= p.c0;
            const int sH = s1 ? p.s[1].H : p.s[0].H, sW = s1 ? p.s[1].W : p.s[0].W;
            const int sst = s1 ? p.s[1].stride : p.s[0].stride;
            const int sup = s1 ? p.s[1].up2 : p.s[0].up2, sG = s1 ? p.s[1].G : p.s[0].G;
            const int cg = (s1 ? c_is - p.c0 : c_is) >> 3;
            const bool kin = kt * BK < p.K;
            uint32_t pix_off[BH];
#pragma unroll
            for (int q = 0; q < BH; ++q) {
                const int iy = px_oy[q] * sst - p.pad_h + kh_is;
                const int ix = px_ox[q] * sst - p.pad_w + kw_is;
                const bool ok = px_ok[q] && kin && (unsigned)iy < (unsigned)(sH << sup) &&
                                (unsigned)ix < (unsigned)(sW << sup);
                // computed unconditionally (no exec-masked branch around the multiplies)
                const uint32_t off = (uint32_t)((((px_img[q] * sH + (iy >> sup)) * sW +
                                                  (ix >> sup)) * sG + cg) * F::GB);
                pix_off[q] = ok ? off : OOB;
            }
            const rsrc_t rb = s1 ? rs1 : rs0;
            uint4* bst = st + B_OFF;
#pragma unroll
            for (int i = 0; i < B_PWI; ++i) {
                if (A_PWI + i < lo || A_PWI + i >= hi) continue;
                const int idx = wave * B_PWI + i;
                const int plane = idx / BH, q = idx % BH;
                const int g = plane / NP, pp = plane % NP;
                // q depends on the (runtime) wave index: pick with compile-time indices
                // (a runtime-indexed register array is placed in scratch)
                uint32_t po = pix_off[0];
#pragma unroll
                for (int qq = 1; qq < BH; ++qq)
                    if (q == qq) po = pix_off[qq];
                const uint32_t off = po == OOB ? OOB : po + g * F::GB + pp * 16;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rb, (__attribute__((address_space(3))) void*)(bst + plane * BN + q * 64), 16,
                    off, 0, 0, 0);
            }
        };
        auto issue = [&](int kt, int stage, const KPos ps) { issue_parts(kt, stage, ps, 0, PWI); };

        auto compute = [&](int stage) {
            const uint4* As = lds + stage * STAGE_UINT4;
            if constexpr (M16) {
                mma16<F, BM, BN, WM, WN, APAD>(As, As + B_OFF, acc);
            } else {
                mma32<F, BM, BN, WM, WN>(As, As + PL * BM, acc, h);
            }
        };

        acc_zero<ConvTileG>(acc);

        if constexpr (PP) {
            // Ping-pong: group 0 = waves 0 .. NW/2-1 (one per SIMD, the LDS-DMA issuers), group
            // 1 = the other wave of every SIMD, one phase behind.  A K-step is two phases
            // separated by workgroup barriers: R (ds_read this step's fragments; group 0 also
            // issues the next step's LDS-DMA pieces) and M (the 6 x T16M x T16N MFMAs).  Between
            // barriers 2k and 2k+1 group 0 reads step k while group 1 runs step k-1's MFMAs;
            // between 2k+1 and 2k+2 group 0 runs step k's MFMAs while group 1 reads step k —
            // so every SIMD's MFMA pipe has one wave feeding it while the other reads LDS.
            // Ring (2 stages): DMA(k+1) is issued in group 0's R(k), into the stage both groups
            // finished reading (lgkmcnt(0) before the barriers 2k-1 / 2k), and retired by group
            // 0's vmcnt(0) before barrier 2k+2, after which both groups read it.
            static_assert(M16 && LW && STAGES == 2 && NW % 2 == 0, "ping-pong tile");
            const bool g1 = wave >= NW / 2;
            __syncthreads();   // the previous segment's readers are done with the ring
            issue(kb, 0, pos);  // group 1 returns at once (LW)
            pos = next(pos);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (g1) __builtin_amdgcn_s_barrier();   // group 1 starts one phase behind
            int st = 0;
            for (int kt = kb; kt < ke; ++kt) {
                const uint4* As = lds + st * STAGE_UINT4;
                if (kt + 1 < ke && !(p.dbg & 2)) {
                    issue(kt + 1, st ^ 1, pos);
                    pos = next(pos);
                }
                typename F::V8 fa[T16M][NP], fb[T16N][NP];
                frag16<F, BM, BN, WM, WN, APAD>(As, As + B_OFF, fa, fb);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
                mfma6<F, T16M, T16N>(fa, fb, acc);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // group 0: DMA(kt+1) landed
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                st ^= 1;
            }
            if (!g1) __builtin_amdgcn_s_barrier();  // pair group 1's last barrier
            pre_last();
            __syncthreads();
            return;
        }

        if constexpr (FP && NP == 1) {
            // Fragment prefetch on one-part operands (AMP, round 5): one MFMA product per
            // fragment, so a step's LDS reads weigh 3x more against its MFMAs than in f16x3.
            // Step kt+1's fragments are read in place as registers free up: B in two halves,
            // each after the MFMAs that read it, A after the last ones (any double buffer
            // spills at the 256 registers of two waves per SIMD).  The slot of
            // step kt (read during step kt-1) takes step kt+STAGES right after the barrier:
            // STAGES-1 steps of LDS-DMA in flight.  Per step: [my reads retired + my pieces of
            // kt+1 landed] -> barrier -> issue kt+STAGES into slot kt -> MFMAs (kt, B half 0)
            // -> read B half 0 (kt+1) || MFMAs (kt, B half 1) -> read A, B half 1 (kt+1).
            // Same MFMA order and operands as the base ring: bit-identical.
            static_assert(M16 && !IL && !PP && F::NTERM == 1 && T16N % 2 == 0,
                          "fragment prefetch (1 part)");
            using V8 = typename F::V8;
            constexpr int HN = T16N / 2;
            const int q = lane >> 4, c16 = lane & 15;
            const int arow = 8 * (c16 >> 2) + (c16 & 3);
            auto rd_a = [&](const uint4* S, V8 (&a)[T16M]) {
#pragma unroll
                for (int i = 0; i < T16M; ++i)
                    a[i] = __builtin_bit_cast(V8, S[q * BM + q * APAD + wm * WTM + 32 * (i >> 1) +
                                                    4 * (i & 1) + arow]);
            };
            auto rd_b = [&](const uint4* S, V8 (&b)[T16N], int h) {
#pragma unroll
                for (int j = h * HN; j < (h + 1) * HN; ++j)
                    b[j] = __builtin_bit_cast(V8, S[B_OFF + q * BN + wn * WTN + j * 16 + c16]);
            };
            auto mm = [&](const V8 (&a)[T16M], const V8 (&b)[T16N], int h) {
#pragma unroll
                for (int i = 0; i < T16M; ++i)
#pragma unroll
                    for (int j = h * HN; j < (h + 1) * HN; ++j)
                        acc[i][j] = F::mfma16(a[i], b[j], acc[i][j]);
            };
            V8 af[T16M], bf[T16N];
            __syncthreads();  // the previous segment's readers are done with the ring
#pragma unroll
            for (int d = 0; d < STAGES; ++d)
                if (kb + d < ke) {
                    issue(kb + d, d, pos);
                    pos = next(pos);
                }
            wait_vm(min(ke - 1 - kb, STAGES - 1));   // step kb landed
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            rd_a(lds, af);
            rd_b(lds, bf, 0);
            rd_b(lds, bf, 1);
            int stage = 0;   // the slot of step kt
            for (int kt = kb; kt + 1 < ke; ++kt) {
                wait_vm(min(STAGES - 2, ke - 2 - kt));   // my pieces of kt+1 landed
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // my reads of slot kt
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                if (kt + STAGES < ke && !(p.dbg & 2)) {
                    issue(kt + STAGES, stage, pos);
                    pos = next(pos);
                }
                int ns = stage + 1;
                if (ns == STAGES) ns = 0;
                const uint4* Ns = lds + ns * STAGE_UINT4;
                mm(af, bf, 0);
                __builtin_amdgcn_sched_barrier(0);
                rd_b(Ns, bf, 0);
                __builtin_amdgcn_sched_barrier(0);
                mm(af, bf, 1);
                __builtin_amdgcn_sched_barrier(0);
                rd_a(Ns, af);
                rd_b(Ns, bf, 1);
                __builtin_amdgcn_sched_barrier(0);
                stage = ns;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            pre_last();
            __builtin_amdgcn_sched_barrier(0);
            mm(af, bf, 0);
            mm(af, bf, 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __syncthreads();
            return;
        } else if constexpr (FP) {
            // Fragment prefetch (round 5).  The base ring reads a step's fragments right after
            // its barrier and then runs its MFMAs, so every wave of the CU waits on its LDS
            // reads (8 waves x 16 ds_read_b128 = 512 LDS cycles a step) before the matrix
            // pipe starts: ~1/3 of the 1536 MFMA cycles exposed.  Here the fragments of step
            // kt+1 are read UNDER the MFMAs of step kt, group by group as registers free up:
            // the hi parts (used by two terms) are double-buffered, the lo parts reloaded in
            // place after the one term that reads them (96 fragment VGPRs instead of 2 x 64).
            // Per step: [my reads of slot kt retired (lgkmcnt 0) + my pieces of kt+1 landed
            // (counted vmcnt)] -> barrier (every wave: kt+1 landed, slot kt read) -> issue
            // kt+3 into slot kt (two steps of LDS-DMA in flight) -> read hi(kt+1) || term 0
            // (al bh) -> read al(kt+1) || term 1 (ah bl) -> read bl(kt+1) || term 2 (ah bh).
            // Same MFMA order and operands as the base ring: bit-identical results.
            static_assert(M16 && STAGES == 3 && !IL && !PP && NP == 2 && F::NTERM == 3,
                          "fragment prefetch: 3-stage 16x16x32 f16x3 ring");
            using V8 = typename F::V8;
            const int q = lane >> 4, c16 = lane & 15;
            const int arow = 8 * (c16 >> 2) + (c16 & 3);
            auto rd_a = [&](const uint4* As, int pp, V8 (&d)[T16M]) {
#pragma unroll
                for (int i = 0; i < T16M; ++i)
                    d[i] = __builtin_bit_cast(V8, As[(q * NP + pp) * BM + q * APAD + wm * WTM +
                                                     32 * (i >> 1) + 4 * (i & 1) + arow]);
            };
            auto rd_b = [&](const uint4* Bs, int pp, V8 (&d)[T16N]) {
#pragma unroll
                for (int j = 0; j < T16N; ++j)
                    d[j] = __builtin_bit_cast(V8, Bs[(q * NP + pp) * BN + wn * WTN + j * 16 + c16]);
            };
            auto mm = [&](const V8 (&a)[T16M], const V8 (&b)[T16N]) {
#pragma unroll
                for (int i = 0; i < T16M; ++i)
#pragma unroll
                    for (int j = 0; j < T16N; ++j) acc[i][j] = F::mfma16(a[i], b[j], acc[i][j]);
            };
            V8 a0x[T16M], a0y[T16M], a1[T16M], b0x[T16N], b0y[T16N], b1[T16N];
            // (debug 512, A/B: static priority for the younger half of the waves — the
            // non-loader waves 4-7, MI355X_MICROARCH.md "Two waves per SIMD" item 4)
            const bool prio = (p.dbg & 512) && wave >= NW / 2;
            if (prio) __builtin_amdgcn_s_setprio(1);
            __syncthreads();  // the previous segment's readers are done with the ring
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (kb + d < ke) {
                    issue(kb + d, d, pos);
                    pos = next(pos);
                }
            wait_vm(min(ke - 1 - kb, 2));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            rd_a(lds, 0, a0x);
            rd_b(lds + B_OFF, 0, b0x);
            rd_a(lds, 1, a1);
            rd_b(lds + B_OFF, 1, b1);
            int stage = 0;   // the slot of step kt
            // a step with a successor (no data-dependent branch inside: the register sets
            // stay fixed across the unrolled pair)
            auto step = [&](int kt, V8 (&ca0)[T16M], V8 (&cb0)[T16N], V8 (&na0)[T16M],
                            V8 (&nb0)[T16N]) {
                wait_vm(kt + 2 < ke ? 1 : 0);    // my pieces of kt+1 landed
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // my reads of slot kt
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                if (kt + 3 < ke && !(p.dbg & 2)) {
                    issue(kt + 3, stage, pos);
                    pos = next(pos);
                }
                int ns = stage + 1;
                if (ns == STAGES) ns = 0;
                const uint4* Ns = lds + ns * STAGE_UINT4;
                rd_a(Ns, 0, na0);
                rd_b(Ns + B_OFF, 0, nb0);
                __builtin_amdgcn_sched_barrier(0);
                mm(a1, cb0);                     // term 0: al * bh
                __builtin_amdgcn_sched_barrier(0);
                rd_a(Ns, 1, a1);
                __builtin_amdgcn_sched_barrier(0);
                mm(ca0, b1);                     // term 1: ah * bl
                __builtin_amdgcn_sched_barrier(0);
                rd_b(Ns + B_OFF, 1, b1);
                __builtin_amdgcn_sched_barrier(0);
                mm(ca0, cb0);                    // term 2: ah * bh
                __builtin_amdgcn_sched_barrier(0);
                stage = ns;
            };
            // the last step: no successor; the residual loads go out before its MFMAs
            auto last = [&](V8 (&ca0)[T16M], V8 (&cb0)[T16N]) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                pre_last();
                __builtin_amdgcn_sched_barrier(0);
                mm(a1, cb0);
                mm(ca0, b1);
                mm(ca0, cb0);
            };
            int kt = kb;
            for (; kt + 2 < ke; kt += 2) {
                step(kt, a0x, b0x, a0y, b0y);
                step(kt + 1, a0y, b0y, a0x, b0x);
            }
            if (kt + 1 < ke) {
                step(kt, a0x, b0x, a0y, b0y);
                last(a0y, b0y);
            } else {
                last(a0x, b0x);
            }
            if (prio) __builtin_amdgcn_s_setprio(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __syncthreads();
            return;
        }

        // prologue: the first STAGES-1 steps in flight
        __syncthreads();  // the previous segment's readers are done with the ring
#pragma unroll
        for (int d = 0; d < STAGES - 1; ++d)
            if (kb + d < ke) {
                issue(kb + d, d, pos);
                pos = next(pos);
            }
        int stage = 0;
        if constexpr (IL) {
            static_assert(M16 && STAGES == 2, "interleaved issue: 16x16 tiles, two stages");
            // the next step's LDS-DMA pieces are issued between the MFMA terms of this one
            // instead of in a burst after the barrier (a burst holds both waves of a SIMD
            // off the MFMA pipe while they issue)
            for (int kt = kb; kt < ke; ++kt) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                const uint4* As = lds + stage * STAGE_UINT4;
                if (kt + 1 < ke && !(p.dbg & 2)) {
                    const KPos ps = pos;
                    // spread over the first two terms: the pieces still get most of the
                    // step to land before the next barrier's vmcnt(0)
                    mma16<F, BM, BN, WM, WN, APAD>(As, As + B_OFF, acc, [&](int t) {
                        if (t < 2)
                            issue_parts(kt + 1, stage ^ 1, ps, PWI * t / 2, PWI * (t + 1) / 2);
                    });
                    pos = next(pos);
                } else {
                    mma16<F, BM, BN, WM, WN, APAD>(As, As + B_OFF, acc);
                }
                stage ^= 1;
            }
            pre_last();   // (after the loop: inside it the residual registers spill)
        } else {
        for (int kt = kb; kt < ke - 1; ++kt) {
            // step kt landed (this wave's pieces); younger steps may stay in flight
            const int younger = min(ke - 1 - kt, STAGES - 2);
            wait_vm(younger);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave's pieces of kt landed; kt-1 fully read
            if (kt + STAGES - 1 < ke && !(p.dbg & 2)) {
                int st2 = stage + STAGES - 1;
                if (st2 >= STAGES) st2 -= STAGES;
                issue(kt + STAGES - 1, st2, pos);
                pos = next(pos);
            }
            compute(stage);
            if (++stage == STAGES) stage = 0;
        }
        // the last step, peeled: the residual loads go out between its barrier and its
        // MFMAs (inside the loop their registers would be live across every step)
        wait_vm(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        pre_last();
        compute(stage);
        }
        // (the last step's wait_vm(0) retired every LDS-DMA piece; only pre_last's residual
        // loads may still be in flight, and the epilogue's uses wait for them)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }

    template <bool PRE>
    static __device__ __forceinline__ void epilogue(const ConvX& p, int m0, int n0,
                                                    const Acc& acc, uint4* lds, const Res& rv) {
        if constexpr (!M16) {
            ConvTile<F, BM, BN, WM, WN, 1>::epilogue32(p, m0, n0, acc);
        } else {
            Epi::template run<PRE>(p, m0, n0, acc, lds, rv);
        }
    }
};

// first iteration of stream-K block b: floor(b * I / G)
__device__ __forceinline__ long sk_start(long b, long I, long G) { return b * I / G; }

__device__ __forceinline__ long sk_block_of(long x, long I, long G) {
    long b = x * G / I;
    while (b + 1 < G && sk_start(b + 1, I, G) <= x) ++b;
    while (b > 0 && sk_start(b, I, G) > x) --b;
    return b;
}

template <class T, bool SK>
__global__ __launch_bounds__(T::NT) __attribute__((amdgpu_waves_per_eu(T::MIN_WAVES)))
void conv_x6_kernel(ConvX p) {
    constexpr int BM = T::BM_, BN = T::BN_;
    __shared__ uint4 lds[T::LDS_UINT4];
    typename T::Acc acc;

    if constexpr (!SK) {
        const int lb = xcd_remap(blockIdx.x, p.nblocks);
        // (debug 256, A/B only: m-major tile order, so an XCD's run of tiles shares one
        // weight slice instead of one input slice)
        const int ntn = p.nblocks / p.mtiles;
        int mi, ni;
        if (p.gm > 1) {
            // bands of gm m-tiles (round 5): xcd_remap gives each XCD a contiguous run of lb,
            // so an XCD works in ONE band — its resident blocks share gm weight slices (L2
            // keeps them) and each input tile is read by gm blocks side by side.  The n-major
            // order (gm = mtiles) has every XCD stream all the weight slices per round of
            // tiles, which for l4.c3 (4 MB of weights) is more than its L2 holds.
            const int per = p.gm * ntn, g = lb / per, r = lb - g * per;
            mi = g * p.gm + r % p.gm;
            ni = r / p.gm;
        } else {
            mi = (p.dbg & 256) ? lb / ntn : lb % p.mtiles;
            ni = (p.dbg & 256) ? lb % ntn : lb / p.mtiles;
        }
        const int m0 = mi * BM, n0 = ni * BN;
        typename T::Res rv;
        T::segment(p, m0, n0, 0, p.nk, acc, lds, [&]() { T::res_load(p, m0, n0, rv); });
        if constexpr (!T::PREFETCH) T::res_load(p, m0, n0, rv);
        T::template epilogue<true>(p, m0, n0, acc, lds, rv);
        return;
    } else {

    // ---- stream-K ----
    __shared__ int s_old;
    const long G = p.sk_grid;
    const long I = (long)p.ntiles_total * p.nk;
    const long b = xcd_remap(blockIdx.x, p.sk_grid);
    const long it0 = sk_start(b, I, G), it1 = sk_start(b + 1, I, G);
    const int tid = threadIdx.x;
    for (long it = it0; it < it1;) {
        const int t = (int)(it / p.nk);
        const int kb = (int)(it - (long)t * p.nk);
        const int ke = (int)min<long>((long)p.nk, kb + (it1 - it));
        const int m0 = (t % p.mtiles) * BM;
        const int n0 = (t / p.mtiles) * BN;
        typename T::Res rv;
        T::segment(p, m0, n0, kb, ke, acc, lds, [] {});
        if (kb == 0 && ke == p.nk) {
            T::template epilogue<false>(p, m0, n0, acc, lds, rv);
            __syncthreads();   // the next segment refills the ring the epilogue staged in
        } else {
            // Publish this segment's partial sums (lane-major per register) with
            // write-through (sc1) stores, drain, then one relaxed agent-scope
            // ticket per block; the block drawing the last ticket acquires once
            // and reads every slab (cdna_hip_programming.md Guideline 16): no
            // __threadfence (an L2 writeback per thread across 8 XCDs).
            const int which = (it == it0) ? 0 : 1;
            const long slot_off = (b * 2 + which) * (long)(T::ACC * T::NT) * 4;
            const rsrc_t rp = make_rsrc(p.sk_part, 0x7fffffff);
#pragma unroll
            for (int r = 0; r < T::ACC; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(
                    __float_as_uint(acc_get<T>(acc, r)), rp,
                    (int)(slot_off + (r * T::NT + tid) * 4), 0, SC1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const long tb = (long)t * p.nk;
            const long b_lo = sk_block_of(tb, I, G), b_hi = sk_block_of(tb + p.nk - 1, I, G);
            if (tid == 0)
                s_old = __hip_atomic_fetch_add(p.sk_cnt + t, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (s_old == (int)(b_hi - b_lo)) {
                // last arrival: one agent-scope acquire (drops this XCD's stale
                // L1/L2 lines, e.g. of the workspace's zero fill), then reduce all
                // segments (its own slot included) in block order, so the sum
                // does not depend on arrival order
                if (tid == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __syncthreads();
                acc_zero<T>(acc);
                for (long bb = b_lo; bb <= b_hi; ++bb) {
                    const int wh = (sk_start(bb, I, G) >= tb) ? 0 : 1;
                    const long so = (bb * 2 + wh) * (long)(T::ACC * T::NT) * 4;
#pragma unroll
                    for (int r = 0; r < T::ACC; ++r) {
                        acc_set<T>(acc, r,
                                   acc_get<T>(acc, r) +
                                       __builtin_bit_cast(
                                           float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rp, (int)(so + (r * T::NT + tid) * 4), 0,
                                                      SC1)));
                        if (r % 16 == 15) asm volatile("" ::: "memory");  // bound live loads
                    }
                }
                if (tid == 0)
                    __hip_atomic_store(p.sk_cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                T::template epilogue<false>(p, m0, n0, acc, lds, rv);
            }
            __syncthreads();   // the next segment refills the ring
        }
        it += ke - kb;
    }
    }
}


// ---- heterogeneous grouped launch (tcam_conv2d_group): up to kMaxGroup independent
// convolutions of one tile shape (any source / K / output geometry each) in ONE grid.  An
// 8-frame InceptionV3 shard's branch convs have 86-172 tiles each (a third to two thirds of
// the 256 CUs); launched together the branches of a block fill the chip and share one ramp
// and one tail.  Member i owns grid blocks [bstart[i], bstart[i] + nblocks_i); bstart is a
// multiple of 8, so a member's block t runs on XCD t % 8 and xcd_remap keeps the member's
// tiles that share input pixels on one XCD's L2, as in a launch of its own.
constexpr int kMaxGroup = 4;
struct ConvXG {
    ConvX p[kMaxGroup];
    int bstart[kMaxGroup + 1];
    int n;
};

template <class T>
__global__ __launch_bounds__(T::NT) __attribute__((amdgpu_waves_per_eu(T::MIN_WAVES)))
void conv_x6_group_kernel(ConvXG g) {
    constexpr int BM = T::BM_, BN = T::BN_;
    __shared__ uint4 lds[T::LDS_UINT4];
    typename T::Acc acc;
    const int b = blockIdx.x;
    int i = 0;
#pragma unroll
    for (int j = 1; j < kMaxGroup; ++j) i += (j < g.n && b >= g.bstart[j]) ? 1 : 0;
    const ConvX& p = g.p[i];
    const int t = b - g.bstart[i];
    if (t >= p.nblocks) return;   // the member's padding to a multiple of 8 blocks
    const int lb = xcd_remap(t, p.nblocks);
    const int m0 = (lb % p.mtiles) * BM;
    const int n0 = (lb / p.mtiles) * BN;
    typename T::Res rv;
    T::segment(p, m0, n0, 0, p.nk, acc, lds, [&]() { T::res_load(p, m0, n0, rv); });
    if constexpr (!T::PREFETCH) T::res_load(p, m0, n0, rv);
    T::template epilogue<true>(p, m0, n0, acc, lds, rv);
}

// ---- thin 3x3 convolutions (Cout <= 64, stride 1, pad 1: the decoder blocks at 56^2 ..
// 224^2, layer1's 3x3).  These are input-bandwidth bound: the implicit-GEMM tiles re-fetch each
// input pixel for every tap through L2.  Here a block owns a 16x16 output tile of one
// frame and stages its 18x18 halo (32 channels at a time, S3 parts as [part][group][pixel]
// 16-B rows) in LDS once; all nine taps read it shifted.  Wave w computes output rows
// 4w..4w+3 (four 16-pixel subtiles) x 32 MB output channels on v_mfma_f32_16x16x32_bf16 with
// the six x6 terms; A fragments (the packed weights, L2-resident) are loaded per K-step
// straight into registers in mma16's channel-grouped row order.
constexpr int TH_T = 16, TH_H = TH_T + 2, TH_PX = TH_H * TH_H;  // tile, halo side, halo px

// MB: 32-row blocks of output channels (Cout <= 32 MB), in mma16's channel-grouped row order;
// MB = 0: Cout <= 16 on ONE 16-row subtile in the natural row order (MFMA row r = channel r),
// so the last decoder block's 16 channels do not pay for 32 MFMA rows: lane (q, c16) then
// holds channels 4q .. 4q+3, half of one 8-channel group, and stores 8-byte pieces.
// GCM: 8-channel groups of one staged chunk (4; 2 when Ctot == 16: half the LDS, so more
// blocks per CU hide the halo loads of the 224^2 layer)
template <class F, int MB, int GCM = 4>
__global__ __launch_bounds__(256) void conv3x3_thin_kernel(ConvX p) {
    constexpr int TM = MB == 0 ? 1 : 2 * MB;   // 16-row M subtiles
    constexpr int NP = F::NP, PL = F::PL;
    using V8 = typename F::V8;
    __shared__ uint4 hs[NP * GCM * TH_PX];   // [part][group][halo pixel]
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = (p.Wout + TH_T - 1) / TH_T, ty = (p.Hout + TH_T - 1) / TH_T;
    const int bid = blockIdx.x;
    const int b = bid / (tx * ty);
    const int rr = bid - b * tx * ty;
    const int oy0 = (rr / tx) * TH_T, ox0 = (rr % tx) * TH_T;
    const int q = lane >> 4, c16 = lane & 15;
    const int arow = 8 * (c16 >> 2) + (c16 & 3);
    const rsrc_t rw = make_rsrc(p.wt, p.wbytes);
    const rsrc_t rs0 = make_rsrc(p.sp[0], p.sbytes[0]);
    const rsrc_t rs1 = make_rsrc(p.sp[1], p.sbytes[1]);
    floatx4 acc[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int CC = p.Ctot < 32 ? p.Ctot : 32;     // channels per chunk (16 or 32)
    const int GC = CC / 8;
    const int nchunk = p.Ctot / CC;
    // The halo of a chunk (channels [c0, c0 + CC): items (pixel, group), F::GB bytes each) is
    // loaded into registers, every item of the thread at once, then stored to LDS: one memory
    // latency per chunk (round 6: d2.c1 0.151 -> 0.134 ms, d3.c1 0.117 -> 0.100; a load-store
    // loop waited on each load before its LDS store).  PF: the next chunk's loads issued before
    // this chunk's K-steps (measured on the 32-channel layers: no gain, off).
    constexpr bool PF = false;
    constexpr int HIT = (TH_PX * GCM + 255) / 256;   // items per thread, at most
    uint4 hv[HIT][NP];
    auto issue = [&](int ch) {
        const int c0 = ch * CC;
        const bool s1 = c0 >= p.c0;   // a chunk lies within one source (thin_ok)
        const int sH = s1 ? p.s[1].H : p.s[0].H, sW = s1 ? p.s[1].W : p.s[0].W;
        const int sup = s1 ? p.s[1].up2 : p.s[0].up2, sG = s1 ? p.s[1].G : p.s[0].G;
        const rsrc_t r = s1 ? rs1 : rs0;
#pragma unroll
        for (int u = 0; u < HIT; ++u) {
            const int it = u * 256 + tid;
            const int g = it % GC, hp = it / GC;
            const int hy = hp / TH_H, hx = hp - hy * TH_H;
            const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
            const int cl = (s1 ? c0 - p.c0 : c0) + 8 * g;
            const bool ok = it < TH_PX * GC && (unsigned)iy < (unsigned)p.Hout &&
                            (unsigned)ix < (unsigned)p.Wout;
            const uint32_t off = ok ? (uint32_t)((((b * sH + (iy >> sup)) * sW +
                                                   (ix >> sup)) * sG + (cl >> 3)) * F::GB)
                                    : OOB;
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) hv[u][pp] = bload16(r, ok ? off + 16u * pp : OOB);
        }
    };
    if (PF) issue(0);
    for (int ch = 0; ch < nchunk; ++ch) {
        const int c0 = ch * CC;
        if (!PF) issue(ch);
        __syncthreads();   // the previous chunk's readers are done with the halo
#pragma unroll
        for (int u = 0; u < HIT; ++u) {
            const int it = u * 256 + tid;
            if (it < TH_PX * GC) {
                const int g = it % GC, hp = it / GC;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp) hs[(pp * GCM + g) * TH_PX + hp] = hv[u][pp];
            }
        }
        __syncthreads();
        if (PF && ch + 1 < nchunk) issue(ch + 1);
        // K-steps of this chunk: Ctot % 32 == 0 -> (tap, chunk) blocks tap * Ctot/32 + ch;
        // Ctot == 16 -> the five 32-deep blocks of the tap-major packing (2 taps each)
        const int nks = p.Ctot % 32 == 0 ? 9 : p.nk;
        for (int ks = 0; ks < nks; ++ks) {
            const int kb = p.Ctot % 32 == 0 ? ks * (p.Ctot / 32) + ch : ks;
            // this lane's group: k = 32 kb + 8 q -> (tap, channel)
            const int k = 32 * kb + 8 * q;
            const int tap = k / p.Ctot, cg = ((k - tap * p.Ctot) - c0) >> 3;
            const int kh = tap / 3, kw = tap - kh * 3;
            const bool kin = tap < 9;
            V8 fa[TM][NP], fb[4][NP];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    fa[i][pp] = __builtin_bit_cast(
                        V8, bload16(rw, (uint32_t)(((kb * PL + q * NP + pp) * p.Mpad +
                                                        (MB == 0 ? c16 : 32 * (i >> 1) +
                                                         4 * (i & 1) + arow)) *
                                                       16)));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int hp = (4 * w + j + kh) * TH_H + c16 + kw;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp) {
                    const uint4 v = kin ? hs[(pp * GCM + cg) * TH_PX + hp] : make_uint4(0, 0, 0, 0);
                    fb[j][pp] = __builtin_bit_cast(V8, v);
                }
            }
#pragma unroll
            for (int t = 0; t < F::NTERM; ++t)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = F::mfma16(fa[i][F::ta(t)], fb[j][F::tb(t)], acc[i][j]);
        }
    }
    uint8_t* outb = reinterpret_cast<uint8_t*>(p.out);
    using O = typename F::Out;   // output format
    constexpr int ONP = O::NP;
    if constexpr (MB == 0) {
        // lane (q, c16) holds channels 4q .. 4q+3 (half h = q & 1 of group q >> 1) of pixel
        // (row 4w + j, column c16)
        const int g = q >> 1, h = q & 1;
        if (g >= p.Gout) return;
        const float4 b4 = *reinterpret_cast<const float4*>(p.bias + 4 * q);
        const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
        float sc[4] = {1.f, 1.f, 1.f, 1.f};
        if constexpr (F::SCALED) {
            const float4 s4 = *reinterpret_cast<const float4*>(p.wscale + 4 * q);
            sc[0] = s4.x; sc[1] = s4.y; sc[2] = s4.z; sc[3] = s4.w;
        }
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int oy = oy0 + 4 * w + j, ox = ox0 + c16;
            if (oy >= p.Hout || ox >= p.Wout) continue;
            const int n = (b * p.Hout + oy) * p.Wout + ox;
            const floatx4 a = acc[0][j];
            uint32_t pt[4][ONP];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = epi_val<F>(a[e], sc[e], bb[e]);
                const float y = p.relu ? relu_nan(x) : x;
                if constexpr (O::SCALED) bad |= f16_overflow(y);
                O::split(y, pt[e]);
            }
            const uint32_t off = (uint32_t)((n * p.out_gs + p.out_go + g) * O::GB + 8 * h);
#pragma unroll
            for (int pp = 0; pp < ONP; ++pp)
                *reinterpret_cast<uint2*>(outb + off + 16 * pp) =
                    make_uint2(pt[0][pp] | (pt[1][pp] << 16), pt[2][pp] | (pt[3][pp] << 16));
        }
        if constexpr (O::SCALED) {
            if (bad && p.oflow) *p.oflow = 1;
        }
        return;
    }
    // epilogue: lane (q, c16) holds channels 8q .. 8q+7 of each 32-row block tb for
    // pixel (row 4w + j, column c16)
#pragma unroll
    for (int tb = 0; tb < MB; ++tb) {
    const int g = 4 * tb + q;
    if (g >= p.Gout) continue;
    float bb[8], sc[8];
    load_bias_scale<F>(p, g, bb, sc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int oy = oy0 + 4 * w + j, ox = ox0 + c16;
        if (oy >= p.Hout || ox >= p.Wout) continue;
        const int n = (b * p.Hout + oy) * p.Wout + ox;
        const floatx4 a0 = acc[2 * tb][j], a1 = acc[2 * tb + 1][j];
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            x[e] = epi_val<F>(a0[e], sc[e], bb[e]);
            x[4 + e] = epi_val<F>(a1[e], sc[4 + e], bb[4 + e]);
        }
        uint4 o[ONP];
        split_group<O>(p, x, o);
        const uint32_t off = (uint32_t)((n * p.out_gs + p.out_go + g) * O::GB);
#pragma unroll
        for (int pp = 0; pp < ONP; ++pp) *reinterpret_cast<uint4*>(outb + off + 16 * pp) = o[pp];
    }
    }
}

// ---- fused layer-1 bottleneck (f16x3, round 5): conv1 (1x1, Cin -> 64) + BN + ReLU, conv2
// (3x3, 64 -> 64) + BN + ReLU, conv3 (1x1, 64 -> 256) + BN + the residual (or, in the first
// block, the K-concat projection shortcut of the input) + ReLU — encoders/resnet.py:175-232's
// Bottleneck on the 56^2 stage — in ONE launch.  Unfused, the stage moves its 256-channel
// tensors through HBM three times per block (conv1 reads x, conv3 reads the residual x and
// writes the output) plus the 64-channel intermediates twice each; here a block owns a 14x14
// output tile of one frame, computes conv1 over the 16x16 halo (zero outside the image: the
// 3x3's padding), keeps both intermediates in LDS as S2 and reads x once more only for the
// residual (L2).  The arithmetic is the unfused path's bit for bit: the same packed weights,
// 32-deep K-steps in the same order (conv1 channel chunks; conv2 chunk-outer / tap-inner as
// conv3x3_thin_kernel; conv3 the conv2 output then the shortcut input), the three f16x3 terms
// per K-step in mfma6's order, and the same epilogue (acc * scale + bias, + residual, ReLU,
// split with the overflow check).
constexpr int BK_T = 14, BK_H = 16;   // output tile width, halo row width

struct BneckConv {      // one folded conv: packed S2 weights, power-of-two scales, bias
    const void* wt;
    const float* wscale;
    const float* bias;
    uint32_t wbytes;
    int Mpad;
};

struct BneckArgs {
    const void* x;      // block input, S2 (B, H, W, Cin)
    void* out;          // block output, S2 (B, H, W, 256)
    int* oflow;
    uint32_t xbytes;
    int B, H, W, Cin;   // Cin 64 (with ds: the first block) or 256
    int ds;             // conv3 carries the projection shortcut (K = 64 + Cin)
    int tx, ty;         // tiles per frame along x / y
    BneckConv c1, c2, c3;
    unsigned long long* dbg;   // (profiling) per-block phase stamps, 4 per block, or null
    int xcd;                   // map consecutive tiles to one XCD
};

// ReLU + split + overflow check of 8 channels (split_group's arithmetic without a ConvX)
template <class F>
__device__ __forceinline__ void bk_split(const float (&x)[8], bool& bad, uint4 (&o)[F::NP]) {
    uint32_t pt[8][F::NP];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float y = relu_nan(x[e]);
        if constexpr (F::SCALED) bad |= f16_overflow(y);
        F::split(y, pt[e]);
    }
#pragma unroll
    for (int pp = 0; pp < F::NP; ++pp)
        o[pp] = make_uint4(pt[0][pp] | (pt[1][pp] << 16), pt[2][pp] | (pt[3][pp] << 16),
                           pt[4][pp] | (pt[5][pp] << 16), pt[6][pp] | (pt[7][pp] << 16));
}

template <class F>
__device__ __forceinline__ void bk_bias_scale(const BneckConv& c, int g, float (&bb)[8],
                                              float (&sc)[8]) {
    const float4 b0 = *reinterpret_cast<const float4*>(c.bias + 8 * g);
    const float4 b1 = *reinterpret_cast<const float4*>(c.bias + 8 * g + 4);
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
    bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    if constexpr (F::SCALED) {
        const float4 s0 = *reinterpret_cast<const float4*>(c.wscale + 8 * g);
        const float4 s1 = *reinterpret_cast<const float4*>(c.wscale + 8 * g + 4);
        sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
        sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) sc[e] = 1.f;
    }
}

// A fragments of one 32-row block (rows r0 .. r0+31, mma16's channel-grouped order) of packed
// weight block kb
template <class F>
__device__ __forceinline__ void bk_frag_a(rsrc_t rw, int Mpad, int kb, int r0, int q, int arow,
                                          halfx8 (&fa)[2][F::NP]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pp = 0; pp < F::NP; ++pp)
            fa[i][pp] = __builtin_bit_cast(
                halfx8, bload16(rw, (uint32_t)(((kb * F::PL + q * F::NP + pp) * Mpad + r0 +
                                                4 * i + arow) * 16)));
}

template <class F>
__device__ __forceinline__ void bk_mma(const halfx8 (&fa)[2][F::NP], const halfx8 (&fb)[F::NP],
                                       floatx4& a0, floatx4& a1) {
#pragma unroll
    for (int t = 0; t < F::NTERM; ++t) {
        a0 = F::mfma16(fa[0][F::ta(t)], fb[F::tb(t)], a0);
        a1 = F::mfma16(fa[1][F::ta(t)], fb[F::tb(t)], a1);
    }
}

// TR: output rows per tile (the tile is 14 wide; the halo TR + 2 rows of 16 px); NWV: waves.
// <14, 8>: one 14x14 tile per 512-thread block (128 KB LDS, one block per CU); <7, 4>: a 14x7
// tile per 256-thread block (72 KB, two blocks per CU, so one block's HBM phases overlap the
// other's MFMA phases).  Each 32-deep K-step runs the f16x3 terms in mfma6's order.
template <class F, int TR, int NWV, int XB>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(8 / NWV)))
void bottleneck_f16x3_kernel(BneckArgs a) {
    constexpr int NP = F::NP, GB = F::GB;          // parts per value, bytes per 8-ch group
    constexpr int NT = 64 * NWV;
    constexpr int HP = (TR + 2) * BK_H;            // halo pixels (conv1's N)
    constexpr int N1S = HP / 16;                   // conv1 subtiles
    constexpr int VALID = TR * BK_T;               // tile pixels
    constexpr int N2S = (VALID + 15) / 16;         // conv2 / conv3 subtiles
    constexpr int N2 = 16 * N2S;
    constexpr int WN = NWV / 2;                    // conv1 / conv2: 2 row blocks x WN
    constexpr int J1 = (N1S + WN - 1) / WN, J2 = (N2S + WN - 1) / WN;
    constexpr int RB = 8 / NWV;                    // conv3: 32-row blocks per wave
    constexpr int SIT = (HP * 4 + NT - 1) / NT;    // conv1 staging items per thread
    static_assert(HP % 16 == 0 && NWV % 2 == 0 && 8 % NWV == 0 && XB == 2, "bottleneck geometry");
    // LDS: y1 = conv1 output [16 planes (group, part)][HP], which conv2's output [16 planes]
    // [N2] overwrites once conv2's K loop is done; then conv1's input K-steps [8 planes][HP]
    // in XB = 2 buffers
    __shared__ uint4 lds[8 * NP * HP + XB * 4 * NP * HP];
    static_assert(N2 <= HP, "conv2 output fits over conv1's");
    uint4* y1 = lds;
    uint4* xs = lds + 8 * NP * HP;
    uint4* y2 = y1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, c16 = lane & 15;
    const int arow = 8 * (c16 >> 2) + (c16 & 3);
    const int per = a.tx * a.ty;
    // consecutive tiles (vertical neighbours share two halo rows) on one XCD's L2
    // (TCAM_BNECK_XCD=0: blocks in dispatch order)
    const int lb = a.xcd ? xcd_remap((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int b = lb / per, rr = lb - b * per;
    const int oy0 = (rr / a.tx) * TR, ox0 = (rr % a.tx) * BK_T;
    const int G = a.Cin / 8;
    const rsrc_t rx = make_rsrc(a.x, a.xbytes);
    bool bad = false;
    auto stamp = [&](int k) {
        if (a.dbg && tid == 0) a.dbg[blockIdx.x * 4 + k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // ---- conv1: M 64 x N HP halo px x K Cin.  Wave (wm, wn): rows 32 wm .., subtiles
    // wn + WN jj
    {
        const int wm = wave / WN, wn = wave % WN;
        const rsrc_t rw = make_rsrc(a.c1.wt, a.c1.wbytes);
        const int nk = a.Cin / 32;
        // the input K-steps are staged through two LDS buffers from a two-deep register
        // ring (step kb+2's loads are in flight while step kb computes), the weight
        // fragments from a two-deep ring as well; nk (2 or 8) is even
        auto stage_load = [&](int kb, uint4 (&v)[SIT][NP]) {
#pragma unroll
            for (int u = 0; u < SIT; ++u) {
                const int it = tid + NT * u;
                const int g = it & 3, hp = it >> 2;
                const int iy = oy0 - 1 + (hp >> 4), ix = ox0 - 1 + (hp & 15);
                const bool ok = it < HP * 4 && (unsigned)iy < (unsigned)a.H &&
                                (unsigned)ix < (unsigned)a.W;
                const uint32_t off =
                    ok ? (uint32_t)((((b * a.H + iy) * a.W + ix) * G + kb * 4 + g) * GB) : OOB;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp) v[u][pp] = bload16(rx, ok ? off + 16u * pp : OOB);
            }
        };
        auto stage_store = [&](int buf, const uint4 (&v)[SIT][NP]) {
#pragma unroll
            for (int u = 0; u < SIT; ++u) {
                const int it = tid + NT * u;
                if (it < HP * 4) {
                    const int g = it & 3, hp = it >> 2;
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        xs[buf * 4 * NP * HP + (g * NP + pp) * HP + hp] = v[u][pp];
                }
            }
        };
        floatx4 acc[2][J1];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < J1; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        auto compute = [&](int buf, const halfx8 (&fa)[2][NP]) {
            const uint4* B0 = xs + buf * 4 * NP * HP;
#pragma unroll
            for (int jj = 0; jj < J1; ++jj) {
                const int j = wn + WN * jj;
                if (j < N1S) {
                    const int px = 16 * j + c16;
                    halfx8 fb[NP];
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        fb[pp] = __builtin_bit_cast(halfx8, B0[(q * NP + pp) * HP + px]);
                    bk_mma<F>(fa, fb, acc[0][jj], acc[1][jj]);
                }
            }
        };
        uint4 sv[2][SIT][NP];
        halfx8 fr[2][2][NP];
        stage_load(0, sv[0]);
        bk_frag_a<F>(rw, a.c1.Mpad, 0, 32 * wm, q, arow, fr[0]);
        stage_load(1, sv[1]);
        bk_frag_a<F>(rw, a.c1.Mpad, 1, 32 * wm, q, arow, fr[1]);
        stage_store(0, sv[0]);
        __syncthreads();
        if (nk > 2) stage_load(2, sv[0]);
        for (int kb = 0; kb < nk; kb += 2) {
            // step kb: buffer 0 holds it, sv[1] step kb+1, sv[0] step kb+2 (in flight)
            compute(0, fr[0]);
            if (kb + 2 < nk) bk_frag_a<F>(rw, a.c1.Mpad, kb + 2, 32 * wm, q, arow, fr[0]);
            stage_store(1, sv[1]);   // buffer 1 was last read by step kb-1
            __syncthreads();
            if (kb + 3 < nk) stage_load(kb + 3, sv[1]);
            // step kb+1: buffer 1 holds it, sv[0] step kb+2, sv[1] step kb+3 (in flight)
            compute(1, fr[1]);
            if (kb + 3 < nk) bk_frag_a<F>(rw, a.c1.Mpad, kb + 3, 32 * wm, q, arow, fr[1]);
            if (kb + 2 < nk) stage_store(0, sv[0]);
            __syncthreads();
            if (kb + 4 < nk) stage_load(kb + 4, sv[0]);
        }
        // epilogue: group 4 wm + q of this wave's halo px; zero outside the image (conv2's
        // padding)
        const int g = 4 * wm + q;
        float bb[8], sc[8];
        bk_bias_scale<F>(a.c1, g, bb, sc);
#pragma unroll
        for (int jj = 0; jj < J1; ++jj) {
            const int j = wn + WN * jj;
            if (j >= N1S) continue;
            const int px = 16 * j + c16;
            const int iy = oy0 - 1 + (px >> 4), ix = ox0 - 1 + (px & 15);
            uint4 o[NP];
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) o[pp] = make_uint4(0, 0, 0, 0);
            if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
                float x[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    x[e] = epi_val<F>(acc[0][jj][e], sc[e], bb[e]);
                    x[4 + e] = epi_val<F>(acc[1][jj][e], sc[4 + e], bb[4 + e]);
                }
                bk_split<F>(x, bad, o);
            }
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) y1[(g * NP + pp) * HP + px] = o[pp];
        }
    }
    __syncthreads();   // y1 complete
    stamp(1);

    // ---- conv2: M 64 x N N2 (VALID) x K 576: chunk ch outer, tap inner (packed block
    // tap * 2 + ch).  Wave (wm, wn): rows 32 wm .., subtiles wn + WN jj
    {
        const int wm = wave / WN, wn = wave % WN;
        const rsrc_t rw = make_rsrc(a.c2.wt, a.c2.wbytes);
        floatx4 acc[2][J2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < J2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // this lane's output pixel per subtile -> its halo pixel at tap (0, 0)
        int hp0[J2];
#pragma unroll
        for (int jj = 0; jj < J2; ++jj) {
            const int n = 16 * (wn + WN * jj) + c16;
            const int oy = n / BK_T, ox = n - oy * BK_T;
            hp0[jj] = n < VALID ? oy * BK_H + ox : 0;
        }
        // the weight fragments (L2) run AR steps ahead in a register ring: a K-step's MFMAs
        // (a few hundred cycles) are far shorter than an L2 round trip under load
        constexpr int AR = 3;   // 18 = 6 x AR
        halfx8 fr[AR][2][NP];
        auto ld = [&](int ks, halfx8 (&f)[2][NP]) {
            const int ch = ks / 9, tap = ks - 9 * ch;
            bk_frag_a<F>(rw, a.c2.Mpad, tap * 2 + ch, 32 * wm, q, arow, f);
        };
#pragma unroll
        for (int r = 0; r < AR; ++r) ld(r, fr[r]);
        for (int k0 = 0; k0 < 18; k0 += AR) {
#pragma unroll
            for (int r = 0; r < AR; ++r) {
                const int ks = k0 + r;
                const int ch = ks / 9, tap = ks - 9 * ch;
                const int kh = tap / 3, kw = tap - 3 * kh;
                const int sh = kh * BK_H + kw;
#pragma unroll
                for (int jj = 0; jj < J2; ++jj) {
                    if (wn + WN * jj < N2S) {
                        halfx8 fb[NP];
#pragma unroll
                        for (int pp = 0; pp < NP; ++pp)
                            fb[pp] = __builtin_bit_cast(
                                halfx8, y1[((4 * ch + q) * NP + pp) * HP + hp0[jj] + sh]);
                        bk_mma<F>(fr[r], fb, acc[0][jj], acc[1][jj]);
                    }
                }
                if (ks + AR < 18) ld(ks + AR, fr[r]);
            }
        }
        __syncthreads();   // every wave is done reading y1: conv2's output goes over it
        const int g = 4 * wm + q;
        float bb[8], sc[8];
        bk_bias_scale<F>(a.c2, g, bb, sc);
#pragma unroll
        for (int jj = 0; jj < J2; ++jj) {
            const int j = wn + WN * jj;
            if (j >= N2S) continue;
            const int n = 16 * j + c16;
            uint4 o[NP];
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) o[pp] = make_uint4(0, 0, 0, 0);
            if (n < VALID) {
                float x[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    x[e] = epi_val<F>(acc[0][jj][e], sc[e], bb[e]);
                    x[4 + e] = epi_val<F>(acc[1][jj][e], sc[4 + e], bb[4 + e]);
                }
                // (a tile pixel outside the image computes from zero padding only: finite,
                // never stored by conv3)
                bk_split<F>(x, bad, o);
            }
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) y2[(g * NP + pp) * N2 + n] = o[pp];
        }
    }
    __syncthreads();   // y2 complete
    stamp(2);

    // ---- conv3: M 256 x N N2 x K 64 (+ Cin of the shortcut).  Wave w: rows 32 RB w .., all
    // subtiles; epilogue + residual + ReLU straight to the output
    {
        const rsrc_t rw = make_rsrc(a.c3.wt, a.c3.wbytes);
        floatx4 acc[RB][2][N2S];
#pragma unroll
        for (int t = 0; t < RB; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < N2S; ++j) acc[t][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // this lane's global pixel per subtile (-1: not stored)
        int gp[N2S];
#pragma unroll
        for (int j = 0; j < N2S; ++j) {
            const int n = 16 * j + c16;
            const int oy = n / BK_T, ox = n - oy * BK_T;
            const int gy = oy0 + oy, gx = ox0 + ox;
            gp[j] = (n < VALID && gy < a.H && gx < a.W) ? (b * a.H + gy) * a.W + gx : -1;
        }
        // residual pieces in batches of BJ subtiles: the first batch goes out before the K loop
        // (its latency hides under conv3's MFMAs), each later one right before its use, so a
        // wave waits on a residual load once per batch instead of once per subtile (the
        // output stores between them keep later loads from being hoisted)
        constexpr int BJ = N2S > 7 ? 7 : N2S, NBJ = (N2S + BJ - 1) / BJ;
        uint4 rres[BJ][NP];
        auto res_issue = [&](int t, int j0) {
            const int g = 4 * (RB * wave + t) + q;
#pragma unroll
            for (int jj = 0; jj < BJ; ++jj) {
                const int j = j0 + jj;
                if (j < N2S) {
                    const bool ok = !a.ds && gp[j] >= 0;
                    const uint32_t off = ok ? (uint32_t)((gp[j] * G + g) * GB) : OOB;
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        rres[jj][pp] = bload16(rx, ok ? off + 16u * pp : OOB);
                }
            }
        };
        res_issue(0, 0);
        const int nk = 2 + (a.ds ? a.Cin / 32 : 0);
        for (int kb = 0; kb < nk; ++kb) {
            halfx8 fa[RB][2][NP];
#pragma unroll
            for (int t = 0; t < RB; ++t)
                bk_frag_a<F>(rw, a.c3.Mpad, kb, 32 * (RB * wave + t), q, arow, fa[t]);
#pragma unroll
            for (int j = 0; j < N2S; ++j) {
                halfx8 fb[NP];
                if (kb < 2) {
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        fb[pp] = __builtin_bit_cast(
                            halfx8, y2[((4 * kb + q) * NP + pp) * N2 + 16 * j + c16]);
                } else {
                    // the shortcut's input channels 32 (kb - 2) + 8 q .. of this pixel
                    const uint32_t off =
                        gp[j] >= 0 ? (uint32_t)((gp[j] * G + 4 * (kb - 2) + q) * GB) : OOB;
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        fb[pp] = __builtin_bit_cast(halfx8,
                                                    bload16(rx, gp[j] >= 0 ? off + 16u * pp : OOB));
                }
#pragma unroll
                for (int t = 0; t < RB; ++t) bk_mma<F>(fa[t], fb, acc[t][0][j], acc[t][1][j]);
            }
        }
        uint8_t* outb = reinterpret_cast<uint8_t*>(a.out);
#pragma unroll
        for (int t = 0; t < RB; ++t) {
            const int g = 4 * (RB * wave + t) + q;   // output group (32 groups)
            float bb[8], sc[8];
            bk_bias_scale<F>(a.c3, g, bb, sc);
#pragma unroll
            for (int k = 0; k < NBJ; ++k) {
                if (t > 0 || k > 0) res_issue(t, k * BJ);
#pragma unroll
                for (int jj = 0; jj < BJ; ++jj) {
                    const int j = k * BJ + jj;
                    if (j >= N2S || gp[j] < 0) continue;
                    float x[8];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        x[e] = epi_val<F>(acc[t][0][j][e], sc[e], bb[e]);
                        x[4 + e] = epi_val<F>(acc[t][1][j][e], sc[4 + e], bb[4 + e]);
                    }
                    // residual: the block input, 256 channels = the output's groups
                    if (!a.ds) add_group<F>(x, rres[jj]);
                    uint4 o[NP];
                    bk_split<F>(x, bad, o);
                    const long ob = ((long)gp[j] * 32 + g) * GB;
#pragma unroll
                    for (int pp = 0; pp < NP; ++pp)
                        *reinterpret_cast<uint4*>(outb + ob + 16 * pp) = o[pp];
                }
            }
        }
    }
    // one store per wave that saw an out-of-range value (the flag only goes 0 -> 1)
    const unsigned long long msk = __ballot(bad);
    if (msk && a.oflow && lane == __builtin_ctzll(msk)) *a.oflow = 1;
    stamp(3);
}

int g_force_sk = -1;  // -1 auto, 0 off, > 0 forced stream-K grid (tests)
// (TCAM_X6_DEBUG sets the initial flags: A/B runs of a whole bench, e.g. 64 | 128)
int g_dbg = getenv("TCAM_X6_DEBUG") ? atoi(getenv("TCAM_X6_DEBUG")) : 0;

template <class F>
void launch_thin(const ConvX& p, long blocks, int Cout, hipStream_t st) {
    const dim3 grid((unsigned)blocks), block(256);
    if (Cout <= 16 && p.Ctot == 16 && !(g_dbg & 32))
        timed_launch(conv3x3_thin_kernel<F, 0, 2>, grid, block, st, p);
    else if (Cout <= 16 && !(g_dbg & 32))
        timed_launch(conv3x3_thin_kernel<F, 0>, grid, block, st, p);
    else if (Cout <= 32) timed_launch(conv3x3_thin_kernel<F, 1>, grid, block, st, p);
    else timed_launch(conv3x3_thin_kernel<F, 2>, grid, block, st, p);
}

bool thin_ok(const ConvX& p, const tcam_conv_src* srcs, int nsrc, bool has_res) {
    if (p.KH != 3 || p.KW != 3 || p.pad_h != 1 || p.pad_w != 1 || p.Cout > 64 || has_res)
        return false;
    if (!(p.Ctot == 16 || p.Ctot % 32 == 0)) return false;
    for (int i = 0; i < nsrc; ++i) {
        if (srcs[i].stride != 1) return false;
        const int h = srcs[i].up2 ? 2 * srcs[i].H : srcs[i].H;
        const int w = srcs[i].up2 ? 2 * srcs[i].W : srcs[i].W;
        if (h != p.Hout || w != p.Wout) return false;
        if (nsrc == 2 && srcs[0].C % 32) return false;   // a chunk within one source
    }
    return true;
}


// m-tile band of the tile order (conv_x6_kernel): TCAM_CONV_GM=g (A/B) uses bands of g
// m-tiles on every launch whose mtiles it divides; 0 (default) keeps the n-major order
int tile_band(const ConvX& p) {
    static const int g = [] {
        const char* e = getenv("TCAM_CONV_GM");
        return e ? atoi(e) : 0;
    }();
    if (g > 1 && p.mtiles > g && p.mtiles % g == 0) return g;
    return 0;
}

template <class T>
int launch_t(ConvX& p, hipStream_t st) {
    constexpr int BM = T::BM_, BN = T::BN_;
    p.mtiles = (p.Cout + BM - 1) / BM;
    const int ntiles = (p.N + BN - 1) / BN;
    p.ntiles_total = p.mtiles * ntiles;
    p.nblocks = p.ntiles_total;
    auto kern = conv_x6_kernel<T, false>;
    auto kern_sk = conv_x6_kernel<T, true>;
    // resident blocks of the stream-K instantiation (queried once)
    static int resident = -1;
    if (resident < 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern_sk, T::NT, 0) !=
                hipSuccess)
            return TCAM_E_ARG;
        // the occupancy API can report one block/CU too many (MI355X_MICROARCH.md,
        // correctness boundaries); bound it by LDS (160 KiB per CU) as well
        const int by_lds = (160 * 1024) / (int)(T::LDS_UINT4 * sizeof(uint4) + 16);
        resident = min(per_cu, by_lds) * cus;
    }
    p.sk_grid = 0;
    p.gm = tile_band(p);
    const long iters = (long)p.ntiles_total * p.nk;
    const int fsk = g_force_sk > 0 ? g_force_sk : p.sk_req;
    if (p.sk_part && fsk > 0) {
        // test hook: stream-K over a forced grid (>= 1 iteration per block)
        const long needed = (long)fsk * 2 * T::ACC * T::NT * 4;
        if (needed <= p.sk_part_bytes && (long)p.ntiles_total * 4 <= SK_CNT_BYTES)
            p.sk_grid = (int)(fsk < iters ? fsk : iters);
    } else if (p.sk_part && g_force_sk < 0 && T::AUTO_SK && resident > 0 &&
               iters >= 2L * resident) {
        // stream-K when whole waves of tiles would leave >= 8 % of the slots idle
        const int waves = (p.ntiles_total + resident - 1) / resident;
        const double eff = (double)p.ntiles_total / ((double)waves * resident);
        const long needed = (long)resident * 2 * T::ACC * T::NT * 4;
        if (eff < 0.8 && p.nk >= 32 && needed <= p.sk_part_bytes &&
            (long)p.ntiles_total * 4 <= SK_CNT_BYTES)
            p.sk_grid = resident;
    } else if (p.sk_part && g_force_sk < 0 && !T::AUTO_SK && resident > 0 && p.nk >= 64 &&
               getenv("TCAM_X6_SK_G") &&
               (long)p.ntiles_total * 5 <= (long)resident * 3) {
        // LDS-DMA tiles, opt-in (TCAM_X6_SK_G=1): stream-K when one partial wave of tiles
        // would leave >= 40 % of the CUs idle on a deep K.  In isolation it takes such a
        // launch (96 tiles, d0.c1 at 16 frames) from 120 to 208 TF
        // (profiles/round2_tune_x6_sk.txt), but in the pipelined forward the other stream
        // fills those CUs and the fix-up costs more: InceptionV3 1286 vs 1305 frames/s.
        // >= 8 K-steps per block (every block of a stream-K grid needs >= 1)
        const long grid = std::min<long>(resident, iters / 8);
        const long needed = grid * 2 * T::ACC * T::NT * 4;
        if (grid >= 2L * p.ntiles_total && needed <= p.sk_part_bytes &&
            (long)p.ntiles_total * 4 <= SK_CNT_BYTES)
            p.sk_grid = (int)grid;
    }
    if (p.sk_grid) {
        timed_launch(kern_sk, dim3(p.sk_grid), dim3(T::NT), st, p);
    } else {
        timed_launch(kern, dim3(p.nblocks), dim3(T::NT), st, p);
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class T>
int launch_group_t(ConvX* ps, int n, hipStream_t st) {
    constexpr int BM = T::BM_, BN = T::BN_;
    ConvXG g{};
    int b = 0;
    for (int i = 0; i < n; ++i) {
        ConvX& p = ps[i];
        p.mtiles = (p.Cout + BM - 1) / BM;
        p.ntiles_total = p.mtiles * ((p.N + BN - 1) / BN);
        p.nblocks = p.ntiles_total;
        p.sk_grid = 0;
        g.p[i] = p;
        g.bstart[i] = b;
        b += (p.nblocks + 7) / 8 * 8;
    }
    g.bstart[n] = b;
    g.n = n;
    timed_launch(conv_x6_group_kernel<T>, dim3(b), dim3(T::NT), st, g);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class F, int BM, int BN, int WM, int WN, int STAGES = 1>
int launch(ConvX& p, hipStream_t st) {
    return launch_t<ConvTile<F, BM, BN, WM, WN, STAGES>>(p, st);
}

// ids 0 .. 34 (27 = conv3x3_thin_kernel, not in launch_tile; 30 .. 34 exist for FmtF16 only:
// their stages need the 2-part operands' smaller LDS footprint)
constexpr int kNumTiles = 42;
constexpr int kThinTile = 27;  // forced-tile id of conv3x3_thin_kernel
int g_force_tile = -1;

bool is_g_tile(int id);

template <class F>
int launch_tile(int id, ConvX& p, hipStream_t st) {
    if constexpr (!std::is_same<typename F::Out, F>::value) {
        // FmtF16S3 (the f16x3 data gradients of training): the tiles the chooser picks on
        // those shapes; any other id maps to the nearest of them
        switch (id) {
            case 3: return launch<F, 128, 64, 2, 2>(p, st);
            case 15: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true>>(p, st);
            case 17: return launch_t<ConvTile<F, 64, 64, 2, 2, 1, true>>(p, st);
            case 18: return launch_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(p, st);
            case 20: return launch_t<ConvTile<F, 64, 128, 2, 2, 1, true>>(p, st);
            case 26: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true, false, true>>(p, st);
            case 30: return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, true, false, true>>(p, st);
            default: break;
        }
        if (!is_g_tile(id)) return launch_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(p, st);
        return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, true, false, true>>(p, st);
    } else if constexpr (F::NP == 1) {
        // FmtH1 (AMP training): the tiles the chooser picks; any other id maps to the nearest
        // of them (LDS-DMA or register-staged)
        switch (id) {
            case 2: return launch_t<ConvTile<F, 32, 256, 1, 4, 1, true>>(p, st);
            case 3: return launch<F, 128, 64, 2, 2>(p, st);
            case 6: return launch<F, 256, 128, 4, 2, 2>(p, st);
            case 15: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true>>(p, st);
            case 17: return launch_t<ConvTile<F, 64, 64, 2, 2, 1, true>>(p, st);
            case 18: return launch_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(p, st);
            case 20: return launch_t<ConvTile<F, 64, 128, 2, 2, 1, true>>(p, st);
            case 26: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true, false, true>>(p, st);
            // one-part operands: 256x256 / 128x256 LDS-DMA on 32x32x16 with loader waves,
            // three stages in 96 KB (per K-step 2x the FLOPs of 256x128 for 1.33x the bytes)
            case 31: return launch_t<ConvTileG<F, 256, 256, 4, 2, 3, false, false, true>>(p, st);
            case 32: return launch_t<ConvTileG<F, 128, 256, 2, 4, 3, false, false, true>>(p, st);
            // round 5: deeper rings for the one-part operands (one MFMA product per fragment:
            // the K loop waits on L2 / HBM latency, so more steps in flight): 256x256 with four
            // stages (128 KB, three steps in flight) on 32x32x16 / 16x16x32 (five stages exceed the
            // LDS by the kernel's own 4-byte word)
            case 38: return launch_t<ConvTileG<F, 256, 256, 4, 2, 4, false, false, true>>(p, st);
            case 39: return launch_t<ConvTileG<F, 256, 256, 4, 2, 4, true, false, true>>(p, st);
            // the 16x16x32 forms with fragment prefetch (FP), four and three stages
            case 40: return launch_t<ConvTileG<F, 256, 256, 4, 2, 4, true, false, true, false,
                                               true>>(p, st);
            case 41: return launch_t<ConvTileG<F, 256, 256, 4, 2, 3, true, false, true, false,
                                               true>>(p, st);
            default: break;
        }
        if (!is_g_tile(id)) return launch_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(p, st);
        return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, true, false, true>>(p, st);
    } else {
    switch (id) {
        case 0: return launch<F, 128, 128, 2, 2>(p, st);
        case 1: return launch<F, 64, 128, 2, 2>(p, st);
        case 2: return launch<F, 32, 256, 1, 4>(p, st);
        case 3: return launch<F, 128, 64, 2, 2>(p, st);
        case 4: return launch<F, 64, 64, 2, 2>(p, st);
        case 5: return launch<F, 256, 128, 4, 2>(p, st);
        case 6: return launch<F, 256, 128, 4, 2, 2>(p, st);
        case 7: return launch<F, 128, 128, 2, 2, 2>(p, st);
        case 8: return launch<F, 128, 64, 2, 2, 2>(p, st);
        case 9: return launch<F, 64, 64, 2, 2, 2>(p, st);
        // LDS-DMA pipelined tiles (aligned convolutions only)
        case 10: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3>>(p, st);
        case 11: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2>>(p, st);
        case 12: return launch_t<ConvTileG<F, 128, 128, 2, 2, 3>>(p, st);
        case 13: return launch_t<ConvTileG<F, 64, 128, 2, 2, 3>>(p, st);
        // the same LDS-DMA pipelines on the 16x16x32 MFMA
        case 14: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true>>(p, st);
        case 15: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true>>(p, st);
        case 16: return launch_t<ConvTileG<F, 128, 128, 2, 2, 3, true>>(p, st);
        // register-staged tiles on the 16x16x32 MFMA
        case 17: return launch_t<ConvTile<F, 64, 64, 2, 2, 1, true>>(p, st);
        case 18: return launch_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(p, st);
        case 19: return launch_t<ConvTile<F, 128, 128, 2, 2, 1, true>>(p, st);
        case 20: return launch_t<ConvTile<F, 64, 128, 2, 2, 1, true>>(p, st);
        case 21: return launch_t<ConvTile<F, 32, 256, 1, 4, 1, true>>(p, st);
        // 256x128 LDS-DMA, 16x16x32, next step's pieces interleaved with the MFMA terms
        case 22: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true, true>>(p, st);
        // ... with the pieces issued by half of the waves (loader waves)
        case 23: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true, false, true>>(p, st);
        case 24: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true, true, true>>(p, st);
        case 25: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, false, false, true>>(p, st);
        case 26: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true, false, true>>(p, st);
        // ping-pong wave groups (one phase apart: one wave of each SIMD on the MFMA pipe while
        // the other reads LDS)
        case 28: return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true, false, true, true>>(p, st);
        case 29: return launch_t<ConvTileG<F, 128, 128, 4, 2, 2, true, false, true, true>>(p, st);
        default: break;
    }
    if constexpr (F::NP == 2) {
        switch (id) {
            // 256x128 LDS-DMA, 16x16x32, loader waves, THREE stages (147 KB with 2 parts)
            case 30: return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, true, false, true>>(p, st);
            // 256x256 LDS-DMA on 32x32x16 (a wave owns 64x128: 1.33x the FLOP per LDS byte of
            // 256x128), loader waves, two stages (131 KB)
            case 31: return launch_t<ConvTileG<F, 256, 256, 4, 2, 2, false, false, true>>(p, st);
            // 128x256 LDS-DMA on 32x32x16, loader waves, three stages (147 KB)
            case 32: return launch_t<ConvTileG<F, 128, 256, 2, 4, 3, false, false, true>>(p, st);
            // 256x128 LDS-DMA on 32x32x16, loader waves, three stages
            case 33: return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, false, false, true>>(p, st);
            // 128x128 LDS-DMA, 16x16x32, loader waves, TWO stages (64 KB with 2 parts): two
            // blocks per CU, so one block's epilogue overlaps the other's K loop (the residual
            // 1x1 layers, whose epilogue traffic otherwise idles the MFMAs of every CU at once)
            case 34: return launch_t<ConvTileG<F, 128, 128, 4, 2, 2, true, false, true>>(p, st);
            // tiles 30 / 26 with fragment prefetch (FP): the next step's LDS fragments read
            // under this step's MFMAs, two steps of LDS-DMA in flight
            case 35: return launch_t<ConvTileG<F, 256, 128, 4, 2, 3, true, false, true, false,
                                               true>>(p, st);
            case 36: return launch_t<ConvTileG<F, 128, 128, 4, 2, 3, true, false, true, false,
                                               true>>(p, st);
            // 256x192 LDS-DMA, 16x16x32, loader waves, two stages (115 KB): a launch whose
            // 192-pixel tiles make exactly one round where 128 makes two and 256 leaves CUs
            // idle (InceptionV3's SPG heads at 8 x 39^2: 256 tiles on 256 CUs)
            case 37: return launch_t<ConvTileG<F, 256, 192, 4, 2, 2, true, false, true>>(p, st);
            default: break;
        }
    }
    return launch_t<ConvTileG<F, 256, 128, 4, 2, 2, true, false, true>>(p, st);
    }
}

// The tiles of a grouped launch (16x16x32 forms: the per-group destinations of their
// epilogue): 15 / 26 = 128x128 LDS-DMA (26 with loader waves; aligned members only),
// 17 = 64x64, 18 = 128x64, 20 = 64x128 register-staged.
template <class F>
int launch_group_tile(int id, ConvX* ps, int n, hipStream_t st) {
    switch (id) {
        case 15: return launch_group_t<ConvTileG<F, 128, 128, 4, 2, 3, true>>(ps, n, st);
        case 26: return launch_group_t<ConvTileG<F, 128, 128, 4, 2, 3, true, false, true>>(ps, n, st);
        case 17: return launch_group_t<ConvTile<F, 64, 64, 2, 2, 1, true>>(ps, n, st);
        case 20: return launch_group_t<ConvTile<F, 64, 128, 2, 2, 1, true>>(ps, n, st);
        default: return launch_group_t<ConvTile<F, 128, 64, 2, 2, 1, true>>(ps, n, st);
    }
}
bool is_group_tile(int id) { return id == 15 || id == 26 || id == 17 || id == 18 || id == 20; }

// Per-shape choice from scripts/tune_conv_x6.py on MI355X (ResNet50-TCAM,
// batch 32, profiles/round1_tune_x6*.txt).  `aligned`: every source C % 32 == 0
// (the LDS-DMA tiles need it).
bool is_g_tile(int id) { return (id >= 10 && id <= 16) || (id >= 22 && id <= 26) || id >= 28; }
bool is_f16_only_tile(int id) { return id >= 30; }
// tiles on v_mfma_f32_16x16x32_bf16 (epilogue16)
bool is_m16_tile(int id) { return (id >= 14 && id <= 24) || id == 26 || (id >= 28 && id <= 30) || (id >= 34 && id <= 37) || id >= 39; }

int choose_tile_x6(const ConvX& p, bool aligned) {
    // 16x16x32-MFMA forms where they measured ahead (profiles/round1_tune_x6_m16*.txt: the
    // 256x128 LDS-DMA tile +0-4 % on deep-K layers, the register-staged 128x64 +3-13 % on
    // the wide 1x1 c3 layers, 64x64 +0-6 % on Cout 32/64)
    // 256x128 LDS-DMA on 16x16x32 with loader waves (profiles/round1_tune_x6_lw*.txt: +3-17 %
    // over the same tile with every wave issuing)
    static const int nolw = getenv("TCAM_X6_NOLW") ? atoi(getenv("TCAM_X6_NOLW")) : 0;
    const bool tap3 = p.KH * p.KW > 1;
    // A deep-K launch whose LDS-DMA tiles (one 148 KB block per CU, no stream-K) would give
    // fewer than half of the CUs a tile goes to the register-staged tile of the same shape,
    // which splits its (tile, K-step) iterations over every CU (stream-K, launch_t):
    // SPG-InceptionV3's decoder block 0 at 8 frames (96 tiles) 120 -> 189 TF, block 1 92 ->
    // 137 TF (profiles/round2_tune_x6_inception.txt).  The ResNet50 / VGG16 layers at 32
    // frames have >= 196 tiles and keep the LDS-DMA tiles.
    // (tcam_conv_x6_force_streamk(0): no stream-K and no fill-dependent choice, so every
    // frame's result is independent of how the frames are batched)
    const long ntn = (p.N + 127) / 128;
    const bool deep = p.K >= 32 * 32 && g_force_sk != 0;
    if (aligned && p.Cout >= 256 && p.K >= 1024) {
        if (deep && (long)((p.Cout + 255) / 256) * ntn * 2 < 256) return 6;
        return (nolw & 1) ? (tap3 ? 22 : 14) : 23;
    }
    if (aligned && p.Cout >= 2048 && p.K >= 512) return (nolw & 1) ? 14 : 23;  // layer4 c3
    // 128x128 LDS-DMA: 3x3 on 16x16x32 with loader waves (+10 %), 1x1 on 16x16x32 (+10 %
    // over the 32x32x16 form since the LDS-staged epilogue, profiles/round2_tune_x6_epi.txt)
    if (aligned && p.Cout == 128) {
        if (deep && tap3 && ntn * 2 < 256) return 3;
        return tap3 ? ((nolw & 2) ? 10 : 26) : 15;
    }
    // Cout between 128 and 256 (InceptionV3's 160 / 192-channel 1x7 / 7x1 / 1x1 convs): the
    // 128x128 LDS-DMA tiles (+28 % on the 1x7 / 7x1 layers, +14 % on the 1x1, over the
    // register-staged 128x64)
    if (aligned && p.Cout > 128 && p.Cout < 256) return tap3 ? 26 : 15;
    if (p.Cout >= 512 && p.K <= 128) return 17;              // l2.c3: 64x64 (+6 %)
    if (p.Cout >= 256) return 18;                             // wide 1x1 (c3) layers
    if (p.Cout >= 128) return 3;
    if (p.Cout == 64) return p.K >= 2048 ? 20 : 17;
    if (p.Cout >= 32) return 17;
    return 2;
}

// FmtF16: the 2-part stages leave LDS for a THIRD stage of the 256x128 loader-wave tile:
// +5-17 % on the deep-K layers over the two-stage tile (d0.c1 332 -> 391 TF, l4.c3ds
// 297 -> 345, l4.c3 208 -> 230; profiles/round3_tune_f16.txt)
int num_cus() {
    static int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        return n;
    }();
    return cus;
}

// A/B hook: TCAM_CONV_TILE_MAP="<Cout>x<K>=<id>[s<grid>],..." overrides the choice for those
// shapes (s<grid>: stream-K over that grid)
// (K = Ctot * KH * KW), so a tile can be compared inside the pipelined bench, where other
// streams share the CUs, and not only in isolation
int mapped_tile(ConvX& p) {
    struct Ent { int cout, k, id, sk; };
    static const std::vector<Ent> map = [] {
        std::vector<Ent> m;
        const char* e = getenv("TCAM_CONV_TILE_MAP");
        while (e && *e) {
            Ent x{};
            int used = 0;
            if (sscanf(e, "%dx%d=%d%n", &x.cout, &x.k, &x.id, &used) != 3) break;
            e += used;
            x.sk = 0;
            if (*e == 's' && sscanf(e + 1, "%d%n", &x.sk, &used) == 1) e += 1 + used;
            m.push_back(x);
            if (*e == ',') ++e;
        }
        return m;
    }();
    for (const Ent& x : map)
        if (x.cout == p.Cout && x.k == p.K) {
            p.sk_req = x.sk;
            return x.id;
        }
    return -1;
}

// FmtF16 3-stage loader-wave rings with fragment prefetch (tiles 35 / 36, round 5): the
// same MFMAs as tiles 30 / 26 (bit-identical), the next step's fragments read under this
// step's MFMAs.  Measured per launch at the bench's 32 frames (profiles/round5_fp_tune.txt):
// +1-3 % on the deep 3x3 layers (d0.c1 388 -> 397 TF, l4.c2 374 -> 383, l3.c2 338 -> 341,
// d1.c1 273 -> 281 on the 128x128 form), -1.5 to -8 % on the 1x1 ones (l4.c3 250 -> 230): a
// 3x3's chunk-outer K order re-reads overlapping input windows, a 1x1 streams every step
// from L2 and the deeper DMA ring competes with its epilogue's residual loads.  So: 3x3
// only.  TCAM_CONV_FP=0 keeps the base rings, 2 takes them for every shape (A/B).
int fp_tile(int id, const ConvX& p) {
    static const int on = [] {
        const char* e = getenv("TCAM_CONV_FP");
        return e ? atoi(e) : 1;
    }();
    if (!on || (on == 1 && p.KH * p.KW == 1)) return id;
    return id == 30 ? 35 : (id == 26 ? 36 : id);
}

int choose_tile(ConvX& p, bool aligned, int fmt) {
    const int mid = mapped_tile(p);
    if (mid >= 0) return mid;
    const int id = choose_tile_x6(p, aligned);
    if (fmt == 2 && aligned && (id == 23 || id == 14 || id == 6)) {
        // FmtH1 (AMP, one fp16 product per K-step): the 256x128 tile is bound by its L2 bytes
        // per FLOP; the 256x256 tile moves 2/3 of them.  One 256x256 tile costs ~1.55 of a
        // 256x128 one (both one block per CU), so it wins when it saves whole rounds of
        // tiles: l4.c2 / l4.c1 at 32 frames (392 -> 196 tiles) +22-30 %, every deep layer at
        // the training step's 256 frames +7-17 %; a one-round launch (d0.c1, l3.* at 32
        // frames) stays on 256x128 (profiles/round4_ab_amp_tiles*.txt)
        const long mt = (p.Cout + 255) / 256, cus = num_cus();
        const long r128 = (mt * ((p.N + 127) / 128) + cus - 1) / cus;
        const long r256 = (mt * ((p.N + 255) / 256) + cus - 1) / cus;
        // round 5: with K >= 1024 the fragment-prefetch form (tile 41: the next step's
        // fragments read under this step's MFMAs) runs the training step's deep layers
        // +3-6 % (profiles/round5_ab_amp_fp.txt); l4.c3 (K = 512, 16 steps) stays on 31.
        // TCAM_AMP_FP=0 for A/B.
        static const int amp_fp = getenv("TCAM_AMP_FP") ? atoi(getenv("TCAM_AMP_FP")) : 1;
        if (r256 * 155 < r128 * 100) return amp_fp && p.K >= 1024 ? 41 : 31;
    }
    if (fmt == 1 && aligned && (id == 23 || id == 14) && p.Cout >= 1024 && p.K >= 4096) {
        // FmtF16: a wide, deep launch whose 256x128 tiles take two rounds and whose 256x256
        // tiles fit in one (InceptionV3's SPG heads on an 8-frame 299^2 shard: 344 -> 172
        // tiles) runs on 256x256: +1.5 % family frames/s (profiles/round4_ab_family_heads.txt).
        // Many-round launches stay on 256x128 (256x256 is 10-30 % slower per FLOP there,
        // profiles/round4_ab_f16_tiles256.txt)
        const long mt = (p.Cout + 255) / 256, cus = num_cus();
        const long r128 = (mt * ((p.N + 127) / 128) + cus - 1) / cus;
        const long r192 = (mt * ((p.N + 191) / 192) + cus - 1) / cus;
        const long r256 = (mt * ((p.N + 255) / 256) + cus - 1) / cus;
        // round 5: 256x192 when its rounds x tile width beats both (one full round of 192-pixel
        // tiles: the SPG heads at 8 x 39^2 take 4 x 64 = 256 tiles).  Measured 3-4 % slower on
        // InceptionV3 (its two-stage ring hides less latency than the three-stage 256x128 /
        // 256x256 rings): off by default, TCAM_CONV_T192=1 to A/B (profiles/round5_ab_t192.txt)
        static const int t192 = getenv("TCAM_CONV_T192") ? atoi(getenv("TCAM_CONV_T192")) : 0;
        if (t192 && r192 * 192 < r128 * 128 && r192 * 192 < r256 * 256) return 37;
        if (r256 == 1 && r128 == 2) return 31;
    }
    if (fmt == 1 && id == 6) {
        // FmtF16, an under-filled deep launch (fewer 128x128 tiles than CUs; x6 takes the
        // register-staged stream-K tile there): the 128x128 LDS-DMA tile without stream-K.
        // InceptionV3's decoder block 0 (96 tiles of 256x128 on an 8-frame shard): family
        // 2139-2150 -> 2212-2216 frames/s, against 2119-2122 for a stream-K grid of 256 and
        // 2085-2087 for the register-staged 128x64 (profiles/round4_ab_family_d0.txt)
        return p.KH * p.KW > 1 ? fp_tile(26, p) : 15;
    }
    if (fmt == 1 && id == 3 && aligned && p.Cout == 128 && p.KH * p.KW > 1) {
        // likewise for an under-filled deep 128-channel 3x3 launch (InceptionV3 decoder
        // blocks 1-2): 128x128 LDS-DMA, frac 0.289-0.296 -> 0.297-0.299 in three rounds
        // (profiles/round4_ab_family_c128.txt)
        return fp_tile(26, p);
    }
    if (fmt && (id == 23 || id == 14)) return fp_tile(30, p);
    if (fmt == 1 && id == 26) return fp_tile(26, p);
    return id;
}

}  // namespace

hipEvent_t g_timer_start = nullptr, g_timer_stop = nullptr;

// Arm (or, with nulls, disarm) the launch timer for the next conv call(s): `start` is bound to
// the next conv kernel dispatch, `stop` to every one until disarmed (include/tcam_hip.h).
extern "C" int tcam_timer_arm(void* start, void* stop) {
    g_timer_start = (hipEvent_t)start;
    g_timer_stop = (hipEvent_t)stop;
    return TCAM_OK;
}

extern "C" int tcam_conv_x6_weight_dims(int K, int Cout, int* Kpad, int* Mpad) {
    TCAM_REQUIRE(K > 0 && Cout > 0 && Kpad && Mpad);
    *Kpad = (K + BK - 1) / BK * BK;
    *Mpad = (Cout + 31) / 32 * 32;
    return TCAM_OK;
}

extern "C" int tcam_conv_x6_force_tile(int id) {
    g_force_tile = id;
    return kNumTiles;   // ids 0 .. kNumTiles - 1 (kThinTile = the halo kernel)
}

extern "C" size_t tcam_conv_x6_ws_bytes(void) { return (size_t)SK_WS_BYTES; }

extern "C" int tcam_conv_x6_debug(int flags) {
    g_dbg = flags;
    return TCAM_OK;
}

extern "C" int tcam_conv_x6_force_streamk(int grid) {
    g_force_sk = grid;
    return TCAM_OK;
}

// one output tensor of a (possibly grouped) launch: channels [c_begin, next c_begin) of
// the conv go to channels [coff, ...) of `ptr`, a tensor of cstride channels per pixel
struct Dst {
    void* ptr;
    int c_begin, cstride, coff;
};

// fmt 0: FmtX6 (S3 operands), 1: FmtF16 (S2 operands, wscale + oflow), 2: FmtH1 (S1),
// 3: FmtF16S3 (S2 operands + wscale, S3 output: the f16x3 data gradient)
struct Fmt {
    int fmt;
    const float* wscale;
    int* oflow;
    int eb() const { return fmt == 2 ? 2 : fmt ? 4 : 6; }   // input bytes per element
    int eb_out() const { return fmt == 3 ? 6 : eb(); }      // output bytes per element
};

static int conv2d_x6_launch(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                            const float* bias, const void* residual, const Dst* dst, int nd,
                            int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                            int relu, void* ws, size_t ws_bytes, void* stream, Fmt f);
static int build_convx(ConvX& p, bool& aligned, const tcam_conv_src* srcs, int nsrc, int B,
                       const void* wt, const float* bias, const void* residual, const Dst* dst,
                       int nd, int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                       int relu, void* ws, size_t ws_bytes, Fmt f);

// Buffer offsets inside the kernel are 32-bit: batches whose tensors exceed 2 GiB run as
// consecutive launches over frame chunks (per-frame convolution: exact).
static int conv2d_x6_chunked(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                             const float* bias, const void* residual, const Dst* dst, int nd,
                             int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                             int relu, void* ws, size_t ws_bytes, void* stream, Fmt f) {
    TCAM_REQUIRE(srcs && (nsrc == 1 || nsrc == 2) && B > 0 && Cout > 0 && nd >= 1 && nd <= 3);
    const int eb = f.eb(), ebo = f.eb_out();
    long per = (long)Hout * Wout * Cout * ebo;   // bytes per frame, largest tensor
    for (int i = 0; i < nd; ++i) {
        TCAM_REQUIRE(dst[i].cstride > 0);
        per = std::max(per, (long)Hout * Wout * dst[i].cstride * ebo);
    }
    for (int i = 0; i < nsrc; ++i)
        per = std::max(per, (long)srcs[i].H * srcs[i].W * srcs[i].C * eb);
    const long lim = (long)OOB - (1l << 20);
    if (per * B < lim)
        return conv2d_x6_launch(srcs, nsrc, B, wt, bias, residual, dst, nd, Cout, Hout, Wout,
                                KH, KW, pad_h, pad_w, relu, ws, ws_bytes, stream, f);
    const int fc = (int)std::max(1l, lim / per);
    for (int b0 = 0; b0 < B; b0 += fc) {
        const int nb = std::min(fc, B - b0);
        tcam_conv_src sub[2];
        for (int i = 0; i < nsrc; ++i) {
            sub[i] = srcs[i];
            sub[i].ptr = (const float*)((const char*)srcs[i].ptr +
                                        (long)b0 * srcs[i].H * srcs[i].W * srcs[i].C * eb);
        }
        const long ofr = (long)b0 * Hout * Wout;
        Dst sd[3];
        for (int i = 0; i < nd; ++i) {
            sd[i] = dst[i];
            sd[i].ptr = (void*)((char*)dst[i].ptr + ofr * dst[i].cstride * ebo);
        }
        const int rc = conv2d_x6_launch(
            sub, nsrc, nb, wt, bias,
            residual ? (const void*)((const char*)residual + ofr * Cout * ebo) : nullptr, sd, nd,
            Cout, Hout, Wout, KH, KW, pad_h, pad_w, relu, ws, ws_bytes, stream, f);
        if (rc != TCAM_OK) return rc;
    }
    return TCAM_OK;
}

extern "C" int tcam_conv2d_x6(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                              const float* bias, const void* residual, void* out, int Cout,
                              int Hout, int Wout, int KH, int KW, int pad_h, int pad_w, int relu,
                              int out_cstride, int out_coff, void* ws, size_t ws_bytes,
                              void* stream) {
    const Dst d{out, 0, out_cstride ? out_cstride : Cout, out_coff};
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, residual, &d, 1, Cout, Hout, Wout, KH, KW,
                             pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{0, nullptr, nullptr});
}

extern "C" int tcam_conv2d_f16x3(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                                 const float* wscale, const float* bias, const void* residual,
                                 void* out, int Cout, int Hout, int Wout, int KH, int KW,
                                 int pad_h, int pad_w, int relu, int out_cstride, int out_coff,
                                 int* oflow, void* ws, size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(wscale && ((uintptr_t)wscale & 15) == 0);
    const Dst d{out, 0, out_cstride ? out_cstride : Cout, out_coff};
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, residual, &d, 1, Cout, Hout, Wout, KH, KW,
                             pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{1, wscale, oflow});
}

static unsigned long long* g_bneck_dbg = nullptr;
// (profiling) per-block phase stamps of the fused bottleneck: 4 x blocks uint64 (s_memrealtime
// at the start, after conv1, after conv2, at the end), or null
extern "C" void tcam_bottleneck_set_debug(void* dbg) {
    g_bneck_dbg = reinterpret_cast<unsigned long long*>(dbg);
}

// Fused layer-1 bottleneck (bottleneck_f16x3_kernel): x (B, H, W, cin) S2 -> out (B, H, W, 256)
// S2; w1 (cin -> 64, 1x1), w2 (64 -> 64, 3x3, pad 1), w3 (64 [+ cin when ds] -> 256, 1x1) packed
// by pack_conv_weight_f16 with their scales and biases (BN folded); ds = conv3 carries the
// projection shortcut of x as a K-concat (the first block), else x is the residual (cin 256).
template <class F>
static int bottleneck_launch(const void* x, int B, int H, int W, int cin, const void* w1,
                             const float* s1, const float* b1, const void* w2, const float* s2,
                             const float* b2, const void* w3, const float* s3, const float* b3,
                             int ds, void* out, int* oflow, void* stream) {
    constexpr int eb = F::GB / 8;   // bytes per element (S2: 4, S1: 2)
    TCAM_REQUIRE(x && out && w1 && w2 && w3 && b1 && b2 && b3);
    TCAM_REQUIRE(!F::SCALED || (s1 && s2 && s3));
    TCAM_REQUIRE(B > 0 && H > 0 && W > 0 && (cin == 64 || cin == 256));
    TCAM_REQUIRE(ds ? cin == 64 : cin == 256);
    const void* ptrs[] = {x, out, w1, w2, w3, s1, s2, s3, b1, b2, b3};
    for (const void* q : ptrs) TCAM_REQUIRE(((uintptr_t)q & 15) == 0);
    // buffer offsets inside the kernel are 32-bit: a batch whose output exceeds 2 GiB runs as
    // consecutive launches over frame chunks (each frame's block is independent: exact)
    const long per = (long)H * W * 256 * eb;
    const long lim = (long)OOB - (1l << 20);
    if (per * B >= lim) {
        const int fc = (int)std::max(1l, lim / per);
        TCAM_REQUIRE(per * fc < (long)OOB);
        for (int b0 = 0; b0 < B; b0 += fc) {
            const int nb = std::min(fc, B - b0);
            const int rc = bottleneck_launch<F>(
                (const char*)x + (long)b0 * H * W * cin * eb, nb, H, W, cin, w1, s1, b1, w2, s2,
                b2, w3, s3, b3, ds, (char*)out + (long)b0 * per, oflow, stream);
            if (rc != TCAM_OK) return rc;
        }
        return TCAM_OK;
    }
    BneckArgs a{};
    a.x = x;
    a.out = out;
    a.oflow = oflow;
    a.xbytes = (uint32_t)((long)B * H * W * cin * eb);
    a.B = B;
    a.H = H;
    a.W = W;
    a.Cin = cin;
    a.ds = ds ? 1 : 0;
    // (round 5) TCAM_BNECK_TILE=14: 14x14 tiles, 512 threads, one block per CU (f16x3); default
    // 7: 14x7 tiles, 256 threads, two blocks per CU
    static const int tr = getenv("TCAM_BNECK_TILE") ? atoi(getenv("TCAM_BNECK_TILE")) : 7;
    const int TRr = (tr == 14 && F::NP == 2) ? 14 : 7;
    a.tx = (W + BK_T - 1) / BK_T;
    a.ty = (H + TRr - 1) / TRr;
    a.c1 = BneckConv{w1, s1, b1, (uint32_t)(cin * 64 * eb), 64};
    a.c2 = BneckConv{w2, s2, b2, (uint32_t)(576 * 64 * eb), 64};
    a.c3 = BneckConv{w3, s3, b3, (uint32_t)((64 + (ds ? cin : 0)) * 256 * eb), 256};
    const long blocks = (long)B * a.tx * a.ty;
    TCAM_REQUIRE(blocks < (1L << 31));
    a.dbg = g_bneck_dbg;
    static const int xcd = getenv("TCAM_BNECK_XCD") ? atoi(getenv("TCAM_BNECK_XCD")) : 1;
    a.xcd = xcd;
    if constexpr (F::NP == 2) {
        if (TRr == 14) {
            timed_launch(bottleneck_f16x3_kernel<F, 14, 8, 2>, dim3((unsigned)blocks), dim3(512),
                         as_stream(stream), a);
            TCAM_CHECK_LAUNCH();
            return 0;
        }
    }
    timed_launch(bottleneck_f16x3_kernel<F, 7, 4, 2>, dim3((unsigned)blocks), dim3(256),
                 as_stream(stream), a);
    TCAM_CHECK_LAUNCH();
    return 0;
}

extern "C" int tcam_bottleneck_f16x3(const void* x, int B, int H, int W, int cin,
                                     const void* w1, const float* s1, const float* b1,
                                     const void* w2, const float* s2, const float* b2,
                                     const void* w3, const float* s3, const float* b3, int ds,
                                     void* out, int* oflow, void* stream) {
    return bottleneck_launch<FmtF16>(x, B, H, W, cin, w1, s1, b1, w2, s2, b2, w3, s3, b3, ds,
                                     out, oflow, stream);
}

// The same block on the AMP path (S1 activations, one fp16 product per K-step: the
// FmtH1 weights of pack_conv_weight_h1, no scales), bit-identical to three tcam_conv2d_f16 calls.
extern "C" int tcam_bottleneck_f16(const void* x, int B, int H, int W, int cin, const void* w1,
                                   const float* b1, const void* w2, const float* b2,
                                   const void* w3, const float* b3, int ds, void* out,
                                   void* stream) {
    return bottleneck_launch<FmtH1>(x, B, H, W, cin, w1, nullptr, b1, w2, nullptr, b2, w3,
                                    nullptr, b3, ds, out, nullptr, stream);
}

extern "C" int tcam_conv2d_f16x3_s3out(const tcam_conv_src* srcs, int nsrc, int B,
                                       const void* wt, const float* wscale, const float* bias,
                                       void* out, int Cout, int Hout, int Wout, int KH, int KW,
                                       int pad_h, int pad_w, int relu, int out_cstride,
                                       int out_coff, void* ws, size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(wscale && ((uintptr_t)wscale & 15) == 0);
    const Dst d{out, 0, out_cstride ? out_cstride : Cout, out_coff};
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, nullptr, &d, 1, Cout, Hout, Wout, KH, KW,
                             pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{3, wscale, nullptr});
}

extern "C" int tcam_conv2d_f16(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                               const float* bias, const void* residual, void* out, int Cout,
                               int Hout, int Wout, int KH, int KW, int pad_h, int pad_w, int relu,
                               int out_cstride, int out_coff, void* ws, size_t ws_bytes,
                               void* stream) {
    const Dst d{out, 0, out_cstride ? out_cstride : Cout, out_coff};
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, residual, &d, 1, Cout, Hout, Wout, KH, KW,
                             pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{2, nullptr, nullptr});
}

extern "C" int tcam_conv2d_x6_multi(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                                    const float* bias, int Cout, int Hout, int Wout, int KH,
                                    int KW, int pad_h, int pad_w, int relu,
                                    const tcam_conv_dst* dst, int ndst, void* ws,
                                    size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(dst && ndst >= 1 && ndst <= 3 && dst[0].c_begin == 0);
    Dst d[3];
    for (int i = 0; i < ndst; ++i) {
        const int c1 = i + 1 < ndst ? dst[i + 1].c_begin : Cout;
        TCAM_REQUIRE(dst[i].ptr && dst[i].c_begin % 8 == 0 && c1 > dst[i].c_begin);
        d[i] = Dst{dst[i].ptr, dst[i].c_begin, dst[i].cstride, dst[i].coff};
    }
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, nullptr, d, ndst, Cout, Hout, Wout, KH,
                             KW, pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{0, nullptr, nullptr});
}

extern "C" int tcam_conv2d_f16x3_multi(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                                       const float* wscale, const float* bias, int Cout,
                                       int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                                       int relu, const tcam_conv_dst* dst, int ndst, int* oflow,
                                       void* ws, size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(wscale && ((uintptr_t)wscale & 15) == 0);
    TCAM_REQUIRE(dst && ndst >= 1 && ndst <= 3 && dst[0].c_begin == 0);
    Dst d[3];
    for (int i = 0; i < ndst; ++i) {
        const int c1 = i + 1 < ndst ? dst[i + 1].c_begin : Cout;
        TCAM_REQUIRE(dst[i].ptr && dst[i].c_begin % 8 == 0 && c1 > dst[i].c_begin);
        d[i] = Dst{dst[i].ptr, dst[i].c_begin, dst[i].cstride, dst[i].coff};
    }
    return conv2d_x6_chunked(srcs, nsrc, B, wt, bias, nullptr, d, ndst, Cout, Hout, Wout, KH,
                             KW, pad_h, pad_w, relu, ws, ws_bytes, stream, Fmt{1, wscale, oflow});
}

extern "C" int tcam_conv2d_group(const tcam_conv_prob* probs, int nprob, int B, int fmt,
                                 int tile, int* oflow, void* stream) {
    TCAM_REQUIRE(probs && nprob >= 1 && nprob <= kMaxGroup && (fmt == 0 || fmt == 1));
    TCAM_REQUIRE(tile == -1 || is_group_tile(tile));
    const Fmt f{fmt, nullptr, fmt ? oflow : nullptr};
    ConvX ps[kMaxGroup];
    bool all_aligned = true, taps = false;
    for (int i = 0; i < nprob; ++i) {
        const tcam_conv_prob& q = probs[i];
        Fmt fi = f;
        if (fmt) {
            TCAM_REQUIRE(q.wscale && ((uintptr_t)q.wscale & 15) == 0);
            fi.wscale = q.wscale;
        } else {
            TCAM_REQUIRE(!q.wscale);
        }
        const Dst d{q.out, 0, q.out_cstride ? q.out_cstride : q.Cout, q.out_coff};
        bool aligned;
        const int rc = build_convx(ps[i], aligned, &q.src, 1, B, q.wt, q.bias, nullptr, &d, 1,
                                   q.Cout, q.Hout, q.Wout, q.KH, q.KW, q.pad_h, q.pad_w, q.relu,
                                   nullptr, 0, fi);
        if (rc != TCAM_OK) return rc;
        all_aligned = all_aligned && aligned;
        taps = taps || q.KH * q.KW > 1;
    }
    int id = g_force_tile >= 0 && is_group_tile(g_force_tile) ? g_force_tile : tile;
    if (id < 0) id = all_aligned ? (taps ? 26 : 15) : 18;
    if ((id == 15 || id == 26) && !all_aligned) id = 18;
    return fmt ? launch_group_tile<FmtF16>(id, ps, nprob, as_stream(stream))
               : launch_group_tile<FmtX6>(id, ps, nprob, as_stream(stream));
}

// The kernel parameters of one convolution (every check of the entry points); `aligned`:
// every source C % 32 == 0 (the LDS-DMA tiles need it).
static int build_convx(ConvX& p, bool& aligned, const tcam_conv_src* srcs, int nsrc, int B,
                       const void* wt, const float* bias, const void* residual, const Dst* dst,
                       int nd, int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                       int relu, void* ws, size_t ws_bytes, Fmt f) {
    const int eb = f.eb(), ebo = f.eb_out();
    TCAM_REQUIRE(srcs && (nsrc == 1 || nsrc == 2) && B > 0 && wt && bias && dst);
    TCAM_REQUIRE(KH >= 1 && KH <= 7 && KW >= 1 && KW <= 7 && pad_h >= 0 && pad_w >= 0);
    TCAM_REQUIRE(Cout > 0 && Cout % 8 == 0 && Hout > 0 && Wout > 0);
    TCAM_REQUIRE(((uintptr_t)wt & 15) == 0 && ((uintptr_t)bias & 15) == 0 &&
                 ((uintptr_t)residual & 15) == 0);
    for (int i = 0; i < nd; ++i) {
        const int c1 = i + 1 < nd ? dst[i + 1].c_begin : Cout;
        TCAM_REQUIRE(dst[i].ptr && ((uintptr_t)dst[i].ptr & 15) == 0);
        TCAM_REQUIRE(dst[i].cstride % 8 == 0 && dst[i].coff % 8 == 0 && dst[i].coff >= 0 &&
                     dst[i].coff + (c1 - dst[i].c_begin) <= dst[i].cstride);
        TCAM_REQUIRE((long)B * Hout * Wout * dst[i].cstride * ebo < (long)OOB);
    }
    TCAM_REQUIRE(!residual || (nd == 1 && dst[0].cstride == Cout));
    const int out_cstride = dst[0].cstride, out_coff = dst[0].coff;
    void* out = dst[0].ptr;
    p = ConvX{};
    int ctot = 0;
    for (int i = 0; i < nsrc; ++i) {
        const tcam_conv_src& s = srcs[i];
        TCAM_REQUIRE(s.ptr && s.C > 0 && s.C % 8 == 0 && s.H > 0 && s.W > 0 && s.stride >= 1);
        TCAM_REQUIRE(((uintptr_t)s.ptr & 15) == 0);
        const long bytes = (long)B * s.H * s.W * s.C * eb;
        TCAM_REQUIRE(bytes < (long)OOB);
        p.sp[i] = s.ptr;
        p.sbytes[i] = (uint32_t)bytes;
        p.s[i] = SrcX{s.C, s.H, s.W, s.stride, s.up2 ? 1 : 0, s.C / 8};
        ctot += s.C;
    }
    if (nsrc == 1) {
        p.sp[1] = p.sp[0];
        p.sbytes[1] = p.sbytes[0];
        p.s[1] = p.s[0];
    }
    p.c0 = nsrc == 2 ? srcs[0].C : ctot;
    p.Ctot = ctot;
    p.K = ctot * KH * KW;
    const int Kpad = (p.K + BK - 1) / BK * BK;
    p.Mpad = (Cout + 31) / 32 * 32;
    const long wbytes = (long)Kpad * p.Mpad * eb;
    TCAM_REQUIRE(wbytes < (long)OOB);
    p.wt = wt;
    p.wbytes = (uint32_t)wbytes;
    p.bias = bias;
    p.wscale = f.wscale;
    p.oflow = f.oflow;
    p.res = residual;
    p.out = out;
    p.Cout = Cout;
    p.Gout = Cout / 8;
    p.Hout = Hout;
    p.Wout = Wout;
    p.pad_h = pad_h;
    p.pad_w = pad_w;
    p.relu = relu;
    p.KH = KH;
    p.KW = KW;
    p.out_gs = out_cstride / 8;
    p.out_go = out_coff / 8;
    p.out1 = p.out2 = out;
    p.out1_gs = p.out2_gs = p.out_gs;
    p.out1_go = p.out2_go = p.out_go;
    p.dg1 = p.dg2 = p.Gout;
    if (nd >= 2) {
        p.out1 = dst[1].ptr;
        p.out1_gs = dst[1].cstride / 8;
        p.out1_go = dst[1].coff / 8;
        p.dg1 = dst[1].c_begin / 8;
    }
    if (nd == 3) {
        p.out2 = dst[2].ptr;
        p.out2_gs = dst[2].cstride / 8;
        p.out2_go = dst[2].coff / 8;
        p.dg2 = dst[2].c_begin / 8;
    }
    p.HWo = Hout * Wout;
    const long N = (long)B * Hout * Wout;
    TCAM_REQUIRE(N * out_cstride * ebo < (long)OOB);
    (void)N;
    p.N = (int)N;
    p.nk = Kpad / BK;
    p.dbg = g_dbg;
    p.gm = 0;
    p.corder = (KH * KW > 1 && !(g_dbg & 4)) ? 1 : 0;  // debug bit 4: tap-major (A/B only)
    aligned = true;
    for (int i = 0; i < nsrc; ++i) aligned = aligned && (srcs[i].C % 32 == 0);
    if (ws && ws_bytes >= (size_t)SK_CNT_BYTES + (1u << 20) && ((uintptr_t)ws & 255) == 0) {
        p.sk_cnt = reinterpret_cast<int*>(ws);
        p.sk_part = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) + SK_CNT_BYTES);
        p.sk_part_bytes = (long)ws_bytes - SK_CNT_BYTES;
    }
    return TCAM_OK;
}

static int conv2d_x6_launch(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                            const float* bias, const void* residual, const Dst* dst, int nd,
                            int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                            int relu, void* ws, size_t ws_bytes, void* stream, Fmt f) {
    ConvX p;
    bool aligned;
    const int rc = build_convx(p, aligned, srcs, nsrc, B, wt, bias, residual, dst, nd, Cout, Hout,
                               Wout, KH, KW, pad_h, pad_w, relu, ws, ws_bytes, f);
    if (rc != TCAM_OK) return rc;
    // thin 3x3 layers: the halo-tiled kernel (tile id kThinTile when forced)
    if ((g_force_tile < 0 || g_force_tile == kThinTile) && nd == 1 &&
        thin_ok(p, srcs, nsrc, residual)) {
        const long blocks = (long)B * ((Hout + TH_T - 1) / TH_T) * ((Wout + TH_T - 1) / TH_T);
        if (f.fmt == 2) launch_thin<FmtH1>(p, blocks, Cout, as_stream(stream));
        else if (f.fmt == 3) launch_thin<FmtF16S3>(p, blocks, Cout, as_stream(stream));
        else if (f.fmt) launch_thin<FmtF16>(p, blocks, Cout, as_stream(stream));
        else launch_thin<FmtX6>(p, blocks, Cout, as_stream(stream));
        TCAM_CHECK_LAUNCH();
        return TCAM_OK;
    }
    int id = (g_force_tile >= 0 && g_force_tile < kNumTiles && g_force_tile != kThinTile)
                 ? g_force_tile : choose_tile(p, aligned, f.fmt);
    if (is_g_tile(id) && !aligned) id = choose_tile(p, false, f.fmt);
    if (is_f16_only_tile(id) && !f.fmt) id = choose_tile(p, aligned, 0);
    // a grouped launch needs the 16x16x32 tiles' epilogue (per-group destinations)
    if (nd > 1 && !is_m16_tile(id)) id = aligned ? 15 : 18;
    // l4.c3 (205 MB of residual): 0.235 -> 0.219 ms with non-temporal residual reads on its
    // 256x128 LDS-DMA tile; the register-staged tiles (l3.c3) measured slower with them
    // (profiles/round4_ab_nt_residual.txt)
    p.ntres = is_g_tile(id) ? 1 : 0;
    if (f.fmt == 2) return launch_tile<FmtH1>(id, p, as_stream(stream));
    if (f.fmt == 3) return launch_tile<FmtF16S3>(id, p, as_stream(stream));
    return f.fmt ? launch_tile<FmtF16>(id, p, as_stream(stream))
                 : launch_tile<FmtX6>(id, p, as_stream(stream));
}
