// Training-step kernels of the ResNet50 WSOL encoder (stage 1, task STD_CL: the classifier
// trained end to end, learning/train_wsol.py:710-714 with --freeze_encoder False; the
// README.md:239-266 run).  The convolutions themselves are the inference kernels
// (conv_x6.hip: forward, and the data gradient as the forward conv of dy with the packed
// transposed weight); the BatchNorm statistics / BN-ReLU / its backward are train.hip's.
// This file adds what the encoder has and the decoder does not:
//
//   bn_add_relu     the Bottleneck tail (encoders/resnet.py:221-232):
//                   out = relu(bn3(y3) + (bn_ds(yd) | x))
//   grad_add_mask   dx = a + [out > 0] dout: the identity shortcut's gradient joined to the
//                   conv1 data gradient
//   maxpool_bwd     MaxPool2d(3, 2, 1) backward (resnet.py:97): the gradient goes to the
//                   window's first maximum in (kh, kw) scan order (torch's CPU / CUDA rule)
//   zero_up2        zero insertion: the data gradient of a stride-2 conv is the stride-1
//                   conv (rotated taps) of dy spread onto the even pixels of the input grid
//   wgrad11         the 1x1 weight gradient dW[co][ci] = sum_p dy[p][co] x[s p][ci] (every
//                   conv1 / conv3 / projection of a Bottleneck): a GEMM over pixels on the
//                   fp16 MFMA — f16x3 (scaled S2 dy, S2 x, three products) or AMP (S1, one
//                   product) — with the operands transposed in LDS by ds_read_b64_tr_b16
//   cls head        WGAP's avgpool + fc (poolings/core.py:96-115), nn.CrossEntropyLoss
//                   (losses/std.py:19-53) and their backward
#include "common.h"
#include "s3_util.h"

using s3::G8;

namespace {

constexpr int kB = 256;

// ---------------------------------------------------------- bn_add_relu
// R16 (AMP): autocast's fp16 tensors — each BatchNorm output and the sum are fp16
template <class L, bool R16>
__global__ __launch_bounds__(kB) void bn_add_relu_kernel(
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const uint8_t* __restrict__ yd,
    const float* __restrict__ meand, const float* __restrict__ invstdd,
    const float* __restrict__ gammad, const float* __restrict__ betad,
    const uint8_t* __restrict__ res, uint8_t* __restrict__ out, long total, int G) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    const G8 v = L::load(y + i * L::GB);
    const G8 r = L::load((yd ? yd : res) + i * L::GB);
    G8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        float a = gamma[c] * ((v.v[e] - mean[c]) * invstd[c]) + beta[c];
        float b = r.v[e];
        if (yd) b = gammad[c] * ((b - meand[c]) * invstdd[c]) + betad[c];
        if (R16) {
            a = (float)(_Float16)a;
            b = (float)(_Float16)b;
        }
        o.v[e] = relu_nan(a + b);
    }
    L::store(out + i * L::GB, o);
}

// The same over a fixed grid whose stride is a multiple of G (kB % G == 0): a thread keeps
// one channel group, its per-channel parameters are read once into registers (the kernel
// above issues them per element, one waited-on load each: ~17 k groups per us against ~100 k
// for bn_relu), and two elements are loaded before either is computed.
template <class L, bool R16, bool DS>
__global__ __launch_bounds__(kB) void bn_add_relu_g_kernel(
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const uint8_t* __restrict__ yd,
    const float* __restrict__ meand, const float* __restrict__ invstdd,
    const float* __restrict__ gammad, const float* __restrict__ betad,
    const uint8_t* __restrict__ res, uint8_t* __restrict__ out, long total, int G) {
    const int g = (int)(threadIdx.x % (unsigned)G);
    float mu[8], is[8], gm[8], bt[8], mud[8], isd[8], gmd[8], btd[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        mu[e] = mean[c];
        is[e] = invstd[c];
        gm[e] = gamma[c];
        bt[e] = beta[c];
        if (DS) {
            mud[e] = meand[c];
            isd[e] = invstdd[c];
            gmd[e] = gammad[c];
            btd[e] = betad[c];
        }
    }
    const uint8_t* src = DS ? yd : res;
    auto tail = [&](const G8& v, const G8& r) {
        G8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float a = gm[e] * ((v.v[e] - mu[e]) * is[e]) + bt[e];
            float b = r.v[e];
            if (DS) b = gmd[e] * ((b - mud[e]) * isd[e]) + btd[e];
            if (R16) {
                a = (float)(_Float16)a;
                b = (float)(_Float16)b;
            }
            o.v[e] = relu_nan(a + b);
        }
        return o;
    };
    const long stride = (long)gridDim.x * kB;
    long i = (long)blockIdx.x * kB + threadIdx.x;
    for (; i + stride < total; i += 2 * stride) {
        const G8 v0 = L::load(y + i * L::GB), r0 = L::load(src + i * L::GB);
        const G8 v1 = L::load(y + (i + stride) * L::GB), r1 = L::load(src + (i + stride) * L::GB);
        L::store(out + i * L::GB, tail(v0, r0));
        L::store(out + (i + stride) * L::GB, tail(v1, r1));
    }
    if (i < total) L::store(out + i * L::GB, tail(L::load(y + i * L::GB), L::load(src + i * L::GB)));
}

// -------------------------------------------------------- grad_add_mask
// r = a + [o > 0] d   (LG: the gradients' layout, LA: the activation's)
template <class LG, class LA>
__global__ __launch_bounds__(kB) void grad_add_mask_kernel(const uint8_t* __restrict__ a,
                                                           const uint8_t* __restrict__ d,
                                                           const uint8_t* __restrict__ o,
                                                           uint8_t* __restrict__ r, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const G8 x = LG::load(a + i * LG::GB), y = LG::load(d + i * LG::GB),
             m = LA::load(o + i * LA::GB);
    G8 s;
#pragma unroll
    for (int e = 0; e < 8; ++e) s.v[e] = x.v[e] + (m.v[e] > 0.f ? y.v[e] : 0.f);
    LG::store(r + i * LG::GB, s);
}

// ---------------------------------------------------------- maxpool bwd
// pass 1: per output pixel and channel, the (kh * 3 + kw) of its window's argmax
template <class LA>
__global__ __launch_bounds__(kB) void maxpool_argmax_kernel(const uint8_t* __restrict__ x,
                                                            uint8_t* __restrict__ idx, int G,
                                                            int H, int W, int Ho, int Wo,
                                                            long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * Ho * Wo * G
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int ox = (int)(t % Wo);
    t /= Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    // torch's max_pool2d: maxindex = the first in-bounds tap, maxval = -inf, then every
    // in-bounds tap in (kh, kw) order replaces when (val > maxval || isnan(val))
    const int kh0 = oy == 0 ? 1 : 0, kw0 = ox == 0 ? 1 : 0;
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        best[e] = -INFINITY;
        arg[e] = (uint32_t)(kh0 * 3 + kw0);
    }
    for (int kh = kh0; kh < 3; ++kh) {
        const int iy = 2 * oy - 1 + kh;
        if (iy >= H) break;
        for (int kw = kw0; kw < 3; ++kw) {
            const int ix = 2 * ox - 1 + kw;
            if (ix >= W) break;
            const G8 v = LA::load(x + (((b * H + iy) * W + ix) * G + g) * LA::GB);
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (v.v[e] > best[e] || isnan(v.v[e])) {
                    best[e] = v.v[e];
                    arg[e] = (uint32_t)(kh * 3 + kw);
                }
        }
    }
    uint2 pk;
    pk.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    pk.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + i * 8) = pk;
}

// pass 2: per input pixel, the sum of the gradients of the (<= 4) outputs whose argmax it is,
// in (oy, ox) order (deterministic)
template <class LG>
__global__ __launch_bounds__(kB) void maxpool_bwd_kernel(const uint8_t* __restrict__ gout,
                                                         const uint8_t* __restrict__ idx,
                                                         uint8_t* __restrict__ gin, int G, int H,
                                                         int W, int Ho, int Wo, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * H * W * G
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int ix = (int)(t % W);
    t /= W;
    const int iy = (int)(t % H);
    const long b = t / H;
    G8 acc;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc.v[e] = 0.f;
    // outputs oy with 2 oy - 1 <= iy <= 2 oy + 1
    const int oy0 = iy / 2, oy1 = min(Ho - 1, (iy + 1) / 2);
    const int ox0 = ix / 2, ox1 = min(Wo - 1, (ix + 1) / 2);
    for (int oy = oy0; oy <= oy1; ++oy) {
        const int kh = iy - (2 * oy - 1);
        if (kh < 0 || kh > 2) continue;
        for (int ox = ox0; ox <= ox1; ++ox) {
            const int kw = ix - (2 * ox - 1);
            if (kw < 0 || kw > 2) continue;
            const long o = ((b * Ho + oy) * Wo + ox) * G + g;
            const uint2 pk = *reinterpret_cast<const uint2*>(idx + o * 8);
            const uint32_t tap = (uint32_t)(kh * 3 + kw);
            bool any = false;
            uint32_t hit[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                hit[e] = (((e < 4 ? pk.x : pk.y) >> (8 * (e & 3))) & 0xffu) == tap;
                any |= hit[e] != 0;
            }
            if (!any) continue;
            const G8 v = LG::load(gout + o * LG::GB);
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (hit[e]) acc.v[e] += v.v[e];
        }
    }
    LG::store(gin + i * LG::GB, acc);
}

// -------------------------------------------------------------- zero_up2
// out (B, H, W, G groups of GB bytes): out[2y][2x] = in[y][x] (y < Hi, x < Wi), 0 elsewhere
template <int GB>
__global__ __launch_bounds__(kB) void zero_up2_kernel(const uint8_t* __restrict__ in,
                                                      uint8_t* __restrict__ out, int G, int H,
                                                      int W, int Hi, int Wi, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * H * W * G
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const long b = t / H;
    uint4* dst = reinterpret_cast<uint4*>(out + i * GB);
    if (!(x & 1) && !(y & 1) && (y >> 1) < Hi && (x >> 1) < Wi) {
        const uint4* src = reinterpret_cast<const uint4*>(
            in + (((b * Hi + (y >> 1)) * Wi + (x >> 1)) * G + g) * GB);
#pragma unroll
        for (int k = 0; k < GB / 16; ++k) dst[k] = src[k];
    } else {
#pragma unroll
        for (int k = 0; k < GB / 16; ++k) dst[k] = make_uint4(0, 0, 0, 0);
    }
}

// ----------------------------------------------------------------- im2col
// out (B, Ho, Wo, KH KW G groups of GB bytes): out[p][(kh KW + kw) G + g] = x[b][s oy - pad +
// kh][s ox - pad + kw][g], 0 outside the frame — every output pixel's KxK / stride-s patch as
// 8-channel groups, so a KxK weight gradient is wgrad11's GEMM over pixels with KH KW C
// "input channels" (the 7x7/2 stem: 49 taps x one group)
template <int GB>
__global__ __launch_bounds__(kB) void im2col_kernel(const uint8_t* __restrict__ x,
                                                    uint8_t* __restrict__ out, int G, int H,
                                                    int W, int KH, int KW, int stride, int pad,
                                                    int Ho, int Wo, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B Ho Wo KH KW G
    if (i >= total) return;
    const int KG = KH * KW * G;
    const long p = i / KG;
    const int r = (int)(i - p * KG);
    const int tap = r / G, g = r - tap * G;
    const int kh = tap / KW, kw = tap - kh * KW;
    const int ox = (int)(p % Wo);
    const long t = p / Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    const int iy = oy * stride - pad + kh, ix = ox * stride - pad + kw;
    uint4* dst = reinterpret_cast<uint4*>(out + i * GB);
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
        const uint4* src = reinterpret_cast<const uint4*>(x + (((b * H + iy) * W + ix) * G + g) * GB);
        uint4 v[GB / 16];
#pragma unroll
        for (int k = 0; k < GB / 16; ++k) v[k] = src[k];
#pragma unroll
        for (int k = 0; k < GB / 16; ++k) dst[k] = v[k];
    } else {
#pragma unroll
        for (int k = 0; k < GB / 16; ++k) dst[k] = make_uint4(0, 0, 0, 0);
    }
}

// ---------------------------------------------------------------- wgrad11
// dW[m][n] = sum_p dy[p][m] x[pix(p)][n]: M = the conv's output channels (dy), N = its input
// channels (x, read at the stride-s position of output pixel p), K = the B*Ho*Wo pixels.
// Block tile MT x NT = (64 WM) x (64 WN), one wave per 64x64 (2 x 2 MFMA 32x32 tiles);
// K in chunks of KP = 32 pixels (two 32x32x16 K-steps), double-buffered in LDS as pixel-major
// images per part ([pixel][channel], as loaded: 16-B groups), read as MFMA fragments with
// ds_read_b64_tr_b16 (a 16-lane group reads 4 pixels x 16 channels; lane i gets channel i of
// the 4 pixels = 4 consecutive K of one row / column), as train.hip's 3x3 weight gradient.
// The pixel range is split over blockIdx.y (partial slabs, reduced in a fixed order).
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// operand formats: F2 = f16x3 on S2 (dy a per-channel power-of-two scaled copy, three
// products dl*xh + dh*xl + dh*xh, the dropped dl*xl < 2^-22 |dy x|); H1 = the AMP path's S1
// (one fp16 product)
struct W11F2 {
    static constexpr int NP = 2, NTERM = 3, GB = 32;
    static constexpr int ta(int t) { return t == 0 ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 1 : 0; }
};
struct W11H1 {
    static constexpr int NP = 1, NTERM = 1, GB = 16;
    static constexpr int ta(int) { return 0; }
    static constexpr int tb(int) { return 0; }
};

struct W11Args {
    const uint8_t* x;
    int Cin, Gin, Hin, Win, stride;
    const uint8_t* dy;
    int Cout, Gout, Ho, Wo;
    long P;        // B * Ho * Wo
    long nchunk;   // ceil(P / KP)
    long cps;      // chunks per split
    int ntm, ntn, ntiles;
    float* part;   // [split][tile][MT][NT]
};

constexpr int kKP = 32;

template <int MT>
struct W11Row {
    // bytes per pixel row of a part image: MT channels, padded so that 4 consecutive rows
    // fall in distinct quarters of the 64 banks (stride = 64 mod 128 bytes)
    static constexpr int R = MT * 2 + ((MT * 2) % 128 == 0 ? 64 : 0);
};

__device__ __forceinline__ v4i16 tr_read(const uint8_t* lds, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(lds + off));
}

__device__ __forceinline__ halfx8 frag(v4i16 a, v4i16 b) {
    const v8i16 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(halfx8, v);
}

template <class F, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void wgrad11_kernel(W11Args a) {
    constexpr int NT_THR = 64 * WM * WN;
    constexpr int MT = 64 * WM, NT = 64 * WN;
    constexpr int NP = F::NP;
    constexpr int RA = W11Row<MT>::R, RB = W11Row<NT>::R;
    constexpr int APART = kKP * RA, BPART = kKP * RB;
    constexpr int BUF = NP * (APART + BPART);
    constexpr int AIT = (kKP * (MT / 8) + NT_THR - 1) / NT_THR;
    constexpr int BIT = (kKP * (NT / 8) + NT_THR - 1) / NT_THR;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * BUF];

    const int tile = blockIdx.x;
    const int mt = tile % a.ntm, nt = tile / a.ntm;
    const long c0 = (long)blockIdx.y * a.cps;
    const long c1 = min(a.nchunk, c0 + a.cps);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int g16 = lane >> 4, i16 = lane & 15;
    const int rq = i16 >> 2, cp = i16 & 3;
    const int hh = g16 >> 1;
    const int colb = 16 * (g16 & 1) + 4 * cp;
    const int HWo = a.Ho * a.Wo;

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    uint4 av[AIT][NP], bv[BIT][NP];
    auto load_chunk = [&](long c) {
        const long p0 = c * kKP;
#pragma unroll
        for (int j = 0; j < AIT; ++j) {
            const int it = tid + j * NT_THR;
            const int g = it % (MT / 8), pix = it / (MT / 8);
            const long p = p0 + pix;
            const int m = mt * MT + g * 8;
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) av[j][pp] = make_uint4(0, 0, 0, 0);
            if (it < kKP * (MT / 8) && p < a.P && m < a.Cout) {
                const uint8_t* src = a.dy + (p * a.Gout + m / 8) * F::GB;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    av[j][pp] = *reinterpret_cast<const uint4*>(src + 16 * pp);
            }
        }
#pragma unroll
        for (int j = 0; j < BIT; ++j) {
            const int it = tid + j * NT_THR;
            const int g = it % (NT / 8), pix = it / (NT / 8);
            const long p = p0 + pix;
            const int n = nt * NT + g * 8;
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) bv[j][pp] = make_uint4(0, 0, 0, 0);
            if (it < kKP * (NT / 8) && p < a.P && n < a.Cin) {
                const long b = p / HWo;
                const int r = (int)(p - b * HWo);
                const int oy = r / a.Wo, ox = r - oy * a.Wo;
                const uint8_t* src =
                    a.x + (((b * a.Hin + oy * a.stride) * a.Win + ox * a.stride) * a.Gin + n / 8) *
                              F::GB;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    bv[j][pp] = *reinterpret_cast<const uint4*>(src + 16 * pp);
            }
        }
    };
    auto store_chunk = [&](uint8_t* buf) {
#pragma unroll
        for (int j = 0; j < AIT; ++j) {
            const int it = tid + j * NT_THR;
            if (it < kKP * (MT / 8)) {
                const int g = it % (MT / 8), pix = it / (MT / 8);
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    *reinterpret_cast<uint4*>(buf + pp * APART + pix * RA + g * 16) = av[j][pp];
            }
        }
#pragma unroll
        for (int j = 0; j < BIT; ++j) {
            const int it = tid + j * NT_THR;
            if (it < kKP * (NT / 8)) {
                const int g = it % (NT / 8), pix = it / (NT / 8);
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    *reinterpret_cast<uint4*>(buf + NP * APART + pp * BPART + pix * RB + g * 16) =
                        bv[j][pp];
            }
        }
    };

    if (c0 < c1) {
        load_chunk(c0);
        store_chunk(lds);
    }
    __syncthreads();
    int cur = 0;
    for (long c = c0; c < c1; ++c) {
        const bool more = c + 1 < c1;
        if (more) load_chunk(c + 1);
        const uint8_t* abuf = lds + cur * BUF;
        const uint8_t* bbuf = abuf + NP * APART;
#pragma unroll
        for (int ks = 0; ks < kKP / 16; ++ks) {
            halfx8 fa[2][NP], fb[2][NP];
            const int k0 = 16 * ks + 8 * hh + rq;
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int off = pp * APART + k0 * RA + (wm * 64 + 32 * i + colb) * 2;
                    fa[i][pp] = frag(tr_read(abuf, off), tr_read(abuf, off + 4 * RA));
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int off = pp * BPART + k0 * RB + (wn * 64 + 32 * j + colb) * 2;
                    fb[j][pp] = frag(tr_read(bbuf, off), tr_read(bbuf, off + 4 * RB));
                }
            }
#pragma unroll
            for (int t = 0; t < F::NTERM; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                            fa[i][F::ta(t)], fb[j][F::tb(t)], acc[i][j], 0, 0, 0);
        }
        if (more) store_chunk(lds + (cur ^ 1) * BUF);
        __syncthreads();
        cur ^= 1;
    }
    // partial slab [split][tile][MT][NT]
    float* out = a.part + ((long)blockIdx.y * a.ntiles + tile) * (MT * NT);
    const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * 64 + 32 * i + 8 * (r >> 2) + 4 * h + (r & 3);
                const int col = wn * 64 + 32 * j + r32;
                out[row * NT + col] = acc[i][j][r];
            }
}

// dW[m][n] (PyTorch (Cout, Cin, 1, 1)) = sum over the splits in order / dscale[m]
__global__ __launch_bounds__(kB) void wgrad11_reduce_kernel(const float* __restrict__ part,
                                                            int splits, int ntiles, int ntm,
                                                            int MT, int NT, int Cout, int Cin,
                                                            const float* __restrict__ dscale,
                                                            float* __restrict__ dw, int r16) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over Cout * Cin
    if (i >= (long)Cout * Cin) return;
    const int m = (int)(i / Cin), n = (int)(i - (long)m * Cin);
    const int tile = (n / NT) * ntm + m / MT;
    const long off = (long)tile * MT * NT + (m % MT) * NT + (n % NT);
    const long slab = (long)ntiles * MT * NT;
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part[(long)k * slab + off];
    if (dscale) s /= dscale[m];   // a power of two: exact
    dw[i] = r16 ? (float)(_Float16)s : s;
}

// ---------------------------------------------------------------- cls head
// WGAP forward for training: pooled[b][c] = mean over the H*W pixels (fixed-order fp32
// sums: a thread per (b, 8-channel group, pixel slice), then the slices in order), and
// logits = pooled fc^T + bias.  R16 (AMP): the pooled tensor and the logits are fp16.
constexpr int kPoolSlices = 32;

template <class L>
__global__ __launch_bounds__(kB) void pool_partial_kernel(const uint8_t* __restrict__ x, int G,
                                                          long HW, float* __restrict__ part,
                                                          long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * kPoolSlices * G
    if (i >= total) return;
    const int g = (int)(i % G);
    const long t = i / G;
    const int sl = (int)(t % kPoolSlices);
    const long b = t / kPoolSlices;
    const long per = (HW + kPoolSlices - 1) / kPoolSlices;
    const long p0 = sl * per, p1 = min(HW, p0 + per);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (long p = p0; p < p1; ++p) {
        const G8 v = L::load(x + ((b * HW + p) * G + g) * L::GB);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += v.v[e];
    }
    float* o = part + ((b * kPoolSlices + sl) * G + g) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = s[e];
}

__global__ __launch_bounds__(kB) void pool_final_kernel(const float* __restrict__ part, int C,
                                                        long HW, int r16,
                                                        float* __restrict__ pooled, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * C
    if (i >= total) return;
    const int c = (int)(i % C);
    const long b = i / C;
    float s = 0.f;
    for (int sl = 0; sl < kPoolSlices; ++sl) s += part[(b * kPoolSlices + sl) * C + c];
    const float v = s / (float)HW;
    pooled[i] = r16 ? (float)(_Float16)v : v;
}

// logits[b][k] = sum_c pooled[b][c] w[k][c] + bias[k]: one wave per (b, k)
__global__ __launch_bounds__(kB) void fc_fwd_kernel(const float* __restrict__ pooled,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ bias, int B,
                                                    int K, int C, int r16,
                                                    float* __restrict__ logits) {
    const int wv = blockIdx.x * (kB / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wv >= B * K) return;
    const int b = wv / K, k = wv - b * K;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) {
        float wc = w[(long)k * C + c];
        if (r16) wc = (float)(_Float16)wc;
        s += pooled[(long)b * C + c] * wc;
    }
    s = wave_sum(s);
    if (lane == 0) {
        float bb = bias[k];
        if (r16) bb = (float)(_Float16)bb;
        const float v = s + bb;
        logits[wv] = r16 ? (float)(_Float16)v : v;
    }
}

// nn.CrossEntropyLoss(reduction="mean") (losses/std.py:23, 53): loss = mean_b (logsumexp_k
// z[b] - z[b][y_b]) * lam; dz = lam (softmax(z[b]) - onehot(y_b)) / B * gscale (the AMP
// loss scale, *gscale_ptr when given).  One block; fp64 accumulation of the loss.
__global__ __launch_bounds__(kB) void ce_loss_kernel(const float* __restrict__ z,
                                                     const int32_t* __restrict__ y, int B, int K,
                                                     float lam, const float* __restrict__ gsc,
                                                     float* __restrict__ loss,
                                                     float* __restrict__ dz) {
    __shared__ double red[kB];
    double acc = 0.0;
    const float gs = gsc ? *gsc : 1.f;
    for (int b = threadIdx.x; b < B; b += kB) {
        const float* zb = z + (long)b * K;
        float mx = -INFINITY;
        for (int k = 0; k < K; ++k) mx = fmaxf(mx, zb[k]);
        double se = 0.0;
        for (int k = 0; k < K; ++k) se += exp((double)zb[k] - (double)mx);
        const double lse = (double)mx + log(se);
        const int t = y[b];
        const bool ok = t >= 0 && t < K;
        acc += ok ? lse - (double)zb[t] : NAN;
        if (dz) {
            for (int k = 0; k < K; ++k) {
                const double p = exp((double)zb[k] - lse);
                dz[(long)b * K + k] =
                    (float)(((p - (k == t ? 1.0 : 0.0)) / (double)B) * (double)lam * (double)gs);
            }
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < kB; ++i) s += red[i];
        loss[0] = (float)(s / (double)B * (double)lam);
    }
}

// fc backward: dW[k][c] = sum_b dz[b][k] pooled[b][c]; db[k] = sum_b dz[b][k];
// dpooled[b][c] = sum_k dz[b][k] w[k][c] (R16: autocast's fp16 tensors — dz is the gradient
// of the fp16 logits, rounded to fp16 as it enters; fp16 results).  Thread per c.
__global__ __launch_bounds__(kB) void fc_bwd_kernel(const float* __restrict__ dz,
                                                    const float* __restrict__ pooled,
                                                    const float* __restrict__ w, int B, int K,
                                                    int C, int r16, float* __restrict__ dw,
                                                    float* __restrict__ db,
                                                    float* __restrict__ dpooled) {
    const int c = blockIdx.x * kB + threadIdx.x;
    auto g = [&](long i) { return r16 ? (float)(_Float16)dz[i] : dz[i]; };
    if (c < C) {
        for (int k = 0; k < K; ++k) {
            float s = 0.f;
            for (int b = 0; b < B; ++b) s += g((long)b * K + k) * pooled[(long)b * C + c];
            dw[(long)k * C + c] = r16 ? (float)(_Float16)s : s;
        }
        for (int b = 0; b < B; ++b) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) {
                float wk = w[(long)k * C + c];
                if (r16) wk = (float)(_Float16)wk;
                s += g((long)b * K + k) * wk;
            }
            dpooled[(long)b * C + c] = r16 ? (float)(_Float16)s : s;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < K) {
        const int k = threadIdx.x;
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += g((long)b * K + k);
        db[k] = r16 ? (float)(_Float16)s : s;
    }
}

// AdaptiveAvgPool2d(1) backward: dout[b][p][c] = dpooled[b][c] / HW, in layout L
template <class L>
__global__ __launch_bounds__(kB) void pool_bwd_kernel(const float* __restrict__ dpooled, int G,
                                                      long HW, uint8_t* __restrict__ dout,
                                                      long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over B * HW * G
    if (i >= total) return;
    const int g = (int)(i % G);
    const long b = i / G / HW;
    const float inv = 1.f / (float)HW;
    G8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v.v[e] = dpooled[b * (G * 8) + g * 8 + e] * inv;
    L::store(dout + i * L::GB, v);
}

}  // namespace

// ================================================================== C ABI
template <class L, bool R16>
static int bn_add_relu(const void* y, const float* mean, const float* invstd,
                       const float* gamma, const float* beta, const void* yd,
                       const float* meand, const float* invstdd, const float* gammad,
                       const float* betad, const void* res, void* out, long P, int C,
                       void* stream) {
    TCAM_REQUIRE(y && mean && invstd && gamma && beta && out && P > 0 && C > 0 && C % 8 == 0);
    TCAM_REQUIRE((yd != nullptr) != (res != nullptr));
    TCAM_REQUIRE(!yd || (meand && invstdd && gammad && betad));
    const long total = P * (C / 8);
    hipStream_t st = as_stream(stream);
    if (kB % (C / 8) == 0) {
        // a few elements per thread (the stride is a multiple of G: one group per thread)
        const int nb = (int)std::min<long>(cdiv(total, 4L * kB), 8192);
        if (yd)
            bn_add_relu_g_kernel<L, R16, true><<<nb, kB, 0, st>>>(
                (const uint8_t*)y, mean, invstd, gamma, beta, (const uint8_t*)yd, meand, invstdd,
                gammad, betad, nullptr, (uint8_t*)out, total, C / 8);
        else
            bn_add_relu_g_kernel<L, R16, false><<<nb, kB, 0, st>>>(
                (const uint8_t*)y, mean, invstd, gamma, beta, nullptr, nullptr, nullptr, nullptr,
                nullptr, (const uint8_t*)res, (uint8_t*)out, total, C / 8);
    } else {
        bn_add_relu_kernel<L, R16><<<cdiv(total, kB), kB, 0, st>>>(
            (const uint8_t*)y, mean, invstd, gamma, beta, (const uint8_t*)yd, meand, invstdd,
            gammad, betad, (const uint8_t*)res, (uint8_t*)out, total, C / 8);
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_bn_add_relu_s2(const void* y, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, const void* yd,
                                   const float* meand, const float* invstdd, const float* gammad,
                                   const float* betad, const void* res, void* out, long P, int C,
                                   void* stream) {
    return bn_add_relu<LayS2, false>(y, mean, invstd, gamma, beta, yd, meand, invstdd, gammad,
                                     betad, res, out, P, C, stream);
}
extern "C" int tcam_bn_add_relu_s1(const void* y, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, const void* yd,
                                   const float* meand, const float* invstdd, const float* gammad,
                                   const float* betad, const void* res, void* out, long P, int C,
                                   void* stream) {
    return bn_add_relu<LayS1, true>(y, mean, invstd, gamma, beta, yd, meand, invstdd, gammad,
                                    betad, res, out, P, C, stream);
}

template <class LG, class LA>
static int grad_add_mask(const void* a, const void* d, const void* o, void* r, long P, int C,
                         void* stream) {
    TCAM_REQUIRE(a && d && o && r && P > 0 && C > 0 && C % 8 == 0);
    const long total = P * (C / 8);
    grad_add_mask_kernel<LG, LA><<<cdiv(total, kB), kB, 0, as_stream(stream)>>>(
        (const uint8_t*)a, (const uint8_t*)d, (const uint8_t*)o, (uint8_t*)r, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
extern "C" int tcam_grad_add_mask_s3s2(const void* a, const void* d, const void* o, void* r,
                                       long P, int C, void* stream) {
    return grad_add_mask<LayS3, LayS2>(a, d, o, r, P, C, stream);
}
extern "C" int tcam_grad_add_mask_s1(const void* a, const void* d, const void* o, void* r,
                                     long P, int C, void* stream) {
    return grad_add_mask<LayS1, LayS1>(a, d, o, r, P, C, stream);
}

template <class LG, class LA>
static int maxpool_bwd(const void* gout, const void* x, void* gin, void* ws, int B, int C, int H,
                       int W, int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(gout && x && gin && ws && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    TCAM_REQUIRE(Ho == (H + 2 - 3) / 2 + 1 && Wo == (W + 2 - 3) / 2 + 1);
    hipStream_t st = as_stream(stream);
    const int G = C / 8;
    const long to = (long)B * Ho * Wo * G;
    maxpool_argmax_kernel<LA><<<cdiv(to, kB), kB, 0, st>>>((const uint8_t*)x, (uint8_t*)ws, G, H,
                                                          W, Ho, Wo, to);
    TCAM_CHECK_LAUNCH();
    const long ti = (long)B * H * W * G;
    maxpool_bwd_kernel<LG><<<cdiv(ti, kB), kB, 0, st>>>((const uint8_t*)gout, (const uint8_t*)ws,
                                                       (uint8_t*)gin, G, H, W, Ho, Wo, ti);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
extern "C" size_t tcam_maxpool_bwd_ws_bytes(int B, int C, int Ho, int Wo) {
    return (size_t)B * Ho * Wo * C + 256;
}
extern "C" int tcam_maxpool3x3s2_bwd_s3s2(const void* gout, const void* x, void* gin, void* ws,
                                          int B, int C, int H, int W, int Ho, int Wo,
                                          void* stream) {
    return maxpool_bwd<LayS3, LayS2>(gout, x, gin, ws, B, C, H, W, Ho, Wo, stream);
}
extern "C" int tcam_maxpool3x3s2_bwd_s1(const void* gout, const void* x, void* gin, void* ws,
                                        int B, int C, int H, int W, int Ho, int Wo,
                                        void* stream) {
    return maxpool_bwd<LayS1, LayS1>(gout, x, gin, ws, B, C, H, W, Ho, Wo, stream);
}

extern "C" int tcam_zero_up2(const void* in, void* out, int gbytes, int B, int C, int H, int W,
                             int Hi, int Wi, void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    TCAM_REQUIRE(Hi > 0 && Wi > 0 && 2 * (Hi - 1) < H && 2 * (Wi - 1) < W);
    const long total = (long)B * H * W * (C / 8);
    hipStream_t st = as_stream(stream);
    switch (gbytes) {
    case 16:
        zero_up2_kernel<16><<<cdiv(total, kB), kB, 0, st>>>((const uint8_t*)in, (uint8_t*)out,
                                                           C / 8, H, W, Hi, Wi, total);
        break;
    case 32:
        zero_up2_kernel<32><<<cdiv(total, kB), kB, 0, st>>>((const uint8_t*)in, (uint8_t*)out,
                                                           C / 8, H, W, Hi, Wi, total);
        break;
    case 48:
        zero_up2_kernel<48><<<cdiv(total, kB), kB, 0, st>>>((const uint8_t*)in, (uint8_t*)out,
                                                           C / 8, H, W, Hi, Wi, total);
        break;
    default:
        return TCAM_E_ARG;
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_im2col(const void* x, void* out, int gbytes, int B, int C, int H, int W,
                           int KH, int KW, int stride, int pad, int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(x && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    TCAM_REQUIRE(KH > 0 && KW > 0 && stride > 0 && pad >= 0 && Ho > 0 && Wo > 0);
    const long total = (long)B * Ho * Wo * KH * KW * (C / 8);
    hipStream_t st = as_stream(stream);
    switch (gbytes) {
    case 16:
        im2col_kernel<16><<<cdiv(total, kB), kB, 0, st>>>((const uint8_t*)x, (uint8_t*)out, C / 8,
                                                         H, W, KH, KW, stride, pad, Ho, Wo, total);
        break;
    case 32:
        im2col_kernel<32><<<cdiv(total, kB), kB, 0, st>>>((const uint8_t*)x, (uint8_t*)out, C / 8,
                                                         H, W, KH, KW, stride, pad, Ho, Wo, total);
        break;
    default:
        return TCAM_E_ARG;
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

// ---- wgrad11 launch geometry
namespace {
struct W11Plan {
    W11Args a;
    int wm, wn, splits;
};

bool make_w11(const void* x, int B, int Cin, int Hin, int Win, int stride, const void* dy,
              int Cout, int Ho, int Wo, W11Plan* pl) {
    if (B <= 0 || Cin <= 0 || Cin % 8 || Cout <= 0 || Cout % 8 || stride < 1) return false;
    if (Ho <= 0 || Wo <= 0 || (Ho - 1) * stride >= Hin || (Wo - 1) * stride >= Win) return false;
    W11Args& a = pl->a;
    a.x = (const uint8_t*)x;
    a.Cin = Cin;
    a.Gin = Cin / 8;
    a.Hin = Hin;
    a.Win = Win;
    a.stride = stride;
    a.dy = (const uint8_t*)dy;
    a.Cout = Cout;
    a.Gout = Cout / 8;
    a.Ho = Ho;
    a.Wo = Wo;
    a.P = (long)B * Ho * Wo;
    a.nchunk = (a.P + kKP - 1) / kKP;
    pl->wm = Cout > 64 ? 2 : 1;
    pl->wn = Cin > 64 ? 2 : 1;
    const int MT = 64 * pl->wm, NT = 64 * pl->wn;
    a.ntm = (Cout + MT - 1) / MT;
    a.ntn = (Cin + NT - 1) / NT;
    a.ntiles = a.ntm * a.ntn;
    // ~1024 blocks in flight, >= 8 chunks (256 pixels) per split, <= 64 splits
    long s = (1024 + a.ntiles - 1) / a.ntiles;
    s = std::max(1l, std::min(s, std::min(64l, a.nchunk / 8)));
    a.cps = (a.nchunk + s - 1) / s;
    pl->splits = (int)((a.nchunk + a.cps - 1) / a.cps);
    return true;
}

size_t w11_ws(const W11Plan& pl) {
    return (size_t)pl.splits * pl.a.ntiles * (64 * pl.wm) * (64 * pl.wn) * sizeof(float) + 256;
}

template <class F>
int wgrad11(const void* x, int B, int Cin, int Hin, int Win, int stride, const void* dy,
            const float* dscale, int Cout, int Ho, int Wo, float* dw, void* ws, size_t ws_bytes,
            int r16, void* stream) {
    W11Plan pl{};
    TCAM_REQUIRE(x && dy && dw && ws);
    TCAM_REQUIRE(make_w11(x, B, Cin, Hin, Win, stride, dy, Cout, Ho, Wo, &pl));
    TCAM_REQUIRE(ws_bytes >= w11_ws(pl));
    pl.a.part = (float*)ws;
    hipStream_t st = as_stream(stream);
    const dim3 grid(pl.a.ntiles, pl.splits);
    if (pl.wm == 2 && pl.wn == 2)
        wgrad11_kernel<F, 2, 2><<<grid, 256, 0, st>>>(pl.a);
    else if (pl.wm == 2)
        wgrad11_kernel<F, 2, 1><<<grid, 128, 0, st>>>(pl.a);
    else if (pl.wn == 2)
        wgrad11_kernel<F, 1, 2><<<grid, 128, 0, st>>>(pl.a);
    else
        wgrad11_kernel<F, 1, 1><<<grid, 64, 0, st>>>(pl.a);
    TCAM_CHECK_LAUNCH();
    const long total = (long)Cout * Cin;
    wgrad11_reduce_kernel<<<cdiv(total, kB), kB, 0, st>>>(
        pl.a.part, pl.splits, pl.a.ntiles, pl.a.ntm, 64 * pl.wm, 64 * pl.wn, Cout, Cin, dscale,
        dw, r16);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
}  // namespace

extern "C" size_t tcam_wgrad11_ws_bytes(int B, int Cin, int Hin, int Win, int stride, int Cout,
                                        int Ho, int Wo) {
    W11Plan pl{};
    int dummy = 0;
    if (!make_w11(&dummy, B, Cin, Hin, Win, stride, &dummy, Cout, Ho, Wo, &pl)) return 0;
    return w11_ws(pl);
}

extern "C" int tcam_wgrad11_s2_f16x3(const void* x, int B, int Cin, int Hin, int Win, int stride,
                                     const void* dy2, const float* dscale, int Cout, int Ho,
                                     int Wo, float* dw, void* ws, size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(dscale);
    return wgrad11<W11F2>(x, B, Cin, Hin, Win, stride, dy2, dscale, Cout, Ho, Wo, dw, ws, ws_bytes,
                          0, stream);
}

extern "C" int tcam_wgrad11_s1(const void* x, int B, int Cin, int Hin, int Win, int stride,
                               const void* dy, int Cout, int Ho, int Wo, float* dw, void* ws,
                               size_t ws_bytes, void* stream) {
    return wgrad11<W11H1>(x, B, Cin, Hin, Win, stride, dy, nullptr, Cout, Ho, Wo, dw, ws, ws_bytes,
                          1, stream);
}

// ---- classifier head
extern "C" size_t tcam_cls_pool_ws_bytes(int B, int C) {
    return (size_t)B * kPoolSlices * C * sizeof(float) + 256;
}

template <class L>
static int cls_fwd(const void* x, int B, long HW, int C, const float* w, const float* bias,
                   int K, float* pooled, float* logits, void* ws, int r16, void* stream) {
    TCAM_REQUIRE(x && w && bias && pooled && logits && ws && B > 0 && HW > 0 && C > 0 &&
                 C % 8 == 0 && K > 0);
    hipStream_t st = as_stream(stream);
    const int G = C / 8;
    const long tp = (long)B * kPoolSlices * G;
    pool_partial_kernel<L><<<cdiv(tp, kB), kB, 0, st>>>((const uint8_t*)x, G, HW, (float*)ws, tp);
    TCAM_CHECK_LAUNCH();
    const long tf = (long)B * C;
    pool_final_kernel<<<cdiv(tf, kB), kB, 0, st>>>((const float*)ws, C, HW, r16, pooled, tf);
    TCAM_CHECK_LAUNCH();
    fc_fwd_kernel<<<cdiv((long)B * K, kB / 64), kB, 0, st>>>(pooled, w, bias, B, K, C, r16,
                                                             logits);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
extern "C" int tcam_cls_fwd_s2(const void* x, int B, long HW, int C, const float* w,
                               const float* bias, int K, float* pooled, float* logits, void* ws,
                               void* stream) {
    return cls_fwd<LayS2>(x, B, HW, C, w, bias, K, pooled, logits, ws, 0, stream);
}
extern "C" int tcam_cls_fwd_s1(const void* x, int B, long HW, int C, const float* w,
                               const float* bias, int K, float* pooled, float* logits, void* ws,
                               void* stream) {
    return cls_fwd<LayS1>(x, B, HW, C, w, bias, K, pooled, logits, ws, 1, stream);
}

extern "C" int tcam_ce_loss(const float* logits, const int32_t* labels, int B, int K, float lam,
                            const float* gscale, float* loss, float* dlogits, void* stream) {
    TCAM_REQUIRE(logits && labels && loss && B > 0 && K > 0);
    ce_loss_kernel<<<1, kB, 0, as_stream(stream)>>>(logits, labels, B, K, lam, gscale, loss,
                                                    dlogits);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_cls_bwd(const float* dlogits, const float* pooled, const float* w, int B,
                            int K, int C, int r16, float* dw, float* db, float* dpooled,
                            void* stream) {
    TCAM_REQUIRE(dlogits && pooled && w && dw && db && dpooled && B > 0 && K > 0 && K <= kB &&
                 C > 0);
    fc_bwd_kernel<<<cdiv(C, kB), kB, 0, as_stream(stream)>>>(dlogits, pooled, w, B, K, C, r16, dw,
                                                             db, dpooled);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int pool_bwd(const float* dpooled, int B, long HW, int C, void* dout, void* stream) {
    TCAM_REQUIRE(dpooled && dout && B > 0 && HW > 0 && C > 0 && C % 8 == 0);
    const long total = (long)B * HW * (C / 8);
    pool_bwd_kernel<L><<<cdiv(total, kB), kB, 0, as_stream(stream)>>>(dpooled, C / 8, HW,
                                                                     (uint8_t*)dout, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
extern "C" int tcam_pool_bwd_s3(const float* dpooled, int B, long HW, int C, void* dout,
                                void* stream) {
    return pool_bwd<LayS3>(dpooled, B, HW, C, dout, stream);
}
extern "C" int tcam_pool_bwd_s1(const float* dpooled, int B, long HW, int C, void* dout,
                                void* stream) {
    return pool_bwd<LayS1>(dpooled, B, HW, C, dout, stream);
}
