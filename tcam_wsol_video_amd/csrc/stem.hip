// The encoder stem (first convolution over the 3-channel image) on the f16x3 path, read
// straight from the fp32 NCHW image: ResNet50's conv1 7x7 / stride 2 / pad 3 + folded bn1 +
// ReLU (encoders/resnet.py:60-62, 175-232), 3 -> 64 channels.
//
// The generic implicit GEMM needs its input in the S2 layout with channels padded to a whole
// 8-channel group, so the stem read 8 channels per tap (K = 49 x 8 = 392 for 147 real MACs
// per output) after a separate NCHW -> S2 pass.  Here K is the 147 real (tap, channel) pairs
// padded to 160: each lane gathers its 8 K values of a K-step for one output pixel from the
// block's LDS window of the image (staged once per block, split into fp16 h | l << 16 words, so
// a gather is one ds_read_b32 and two v_perm per pair) — and the product is f16x3's (al*bh + ah*bl + ah*bh on v_mfma_f32_16x16x32_f16,
// fp32 accumulation; per-channel power-of-two weight scales undone in the epilogue).  The K
// order is the host's: ktab[k] = the window offset c * IR * IC + kh * IC + kw of packed row k
// (-1 = zero padding; tcam_stem_window gives IR x IC), the weight rows packed in the same
// order (ops.StemF16).
//
// Block: a 16-row x 16-column output tile (8 waves); its input window (all channels) and the whole
// packed weight (<= 40 KiB) are staged in LDS once, and the gathers read LDS.  Wave w owns
// output rows 2w, 2w + 1 (two 16-pixel MFMA column subtiles) x MT 16-row Cout subtiles (rows
// in the channel-grouped order of conv_x6.hip's mma16: lane (q, c16) then holds the 8
// channels of group 4t + q, one 16-B store per part).
#include "common.h"
#include "s3_util.h"

#include <algorithm>

namespace {

typedef _Float16 halfx8s __attribute__((ext_vector_type(8)));

struct StemArgs {
    const float* img;          // (B, C, H, W) fp32
    const uint4* wt;           // (nk, 4, 2, Mpad, 8) fp16: [ks][q][part][m][e]
    const float* wscale;       // (Mpad,) powers of two
    const float* bias;         // (Mpad,)
    const int32_t* ktab;       // (nk * 32,) c * IR * IC + kh * IC + kw, -1 = padding
    uint8_t* out;              // S2 (B, Ho, Wo, Cout / 8, 2, 8)
    int* oflow;
    int C, H, W, Ho, Wo, stride, pad, nk, Mpad, Gout, IR, IC, tiles_x, tiles_y;
};

// Output tile of a block: kTR rows x 16 columns; wave w owns rows 2w, 2w + 1 (one 16-pixel
// MFMA column subtile each).
constexpr int kStemWaves = 8;
constexpr int kTR = 2 * kStemWaves;
constexpr int kImgWords = 4608;     // LDS image window (C x IR x IC words): 18 KiB
constexpr int kMaxNk = 8;           // K-steps (K <= 256)
constexpr int kWtUint4 = 2560 + 128;   // LDS weights (nk x 4 x 2 x Mpad uint4 + 4 per plane pair)

template <int MT>
__global__ __launch_bounds__(64 * kStemWaves) void stem_f16x3_kernel(StemArgs p) {
    __shared__ uint32_t ximg[kImgWords];
    __shared__ uint4 wl[kWtUint4];
    __shared__ int4 tl[kMaxNk * 8];    // ktab: (K-step, K group) -> 8 window offsets
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int q = lane >> 4, c16 = lane & 15;
    const int per = p.tiles_x * p.tiles_y;
    const int b = blockIdx.x / per;
    const int tr = blockIdx.x - b * per;
    const int oy0 = (tr / p.tiles_x) * kTR, ox0 = (tr % p.tiles_x) * 16;
    // stage the block's input window (all channels; zero outside the image), split once into
    // fp16 h | l << 16 words, and the whole packed weight (each (K-step, K group) plane pair
    // shifted 4 uint4 past the previous one: the permuted ds_read_b128 rows of the 4 groups
    // of a K-step fall in different banks)
    {
        // (every load of the stage is issued before the first is used: one latency, not nine)
        constexpr int NTHR = 64 * kStemWaves;
        constexpr int IMG_PER = (kImgWords + NTHR - 1) / NTHR;
        constexpr int W_PER = (kWtUint4 + NTHR - 1) / NTHR;
        const float* src = p.img + (long)b * p.C * p.H * p.W;
        const int iy0 = oy0 * p.stride - p.pad, ix0 = ox0 * p.stride - p.pad;
        const int rc = p.IR * p.IC, tot = p.C * rc;
        const int nw = p.nk * 8 * p.Mpad;
        float v[IMG_PER];
#pragma unroll
        for (int u = 0; u < IMG_PER; ++u) {
            const int i = tid + u * NTHR;
            const int c = i / rc, r = (i - c * rc) / p.IC, cc = i - c * rc - r * p.IC;
            const int iy = iy0 + r, ix = ix0 + cc;
            v[u] = 0.f;
            if (i < tot && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)
                v[u] = src[((long)c * p.H + iy) * p.W + ix];
        }
#pragma unroll
        for (int u = 0; u < IMG_PER; ++u) {
            const int i = tid + u * NTHR;
            if (i < tot) {
                uint32_t h, l;
                s2::split2(v[u], h, l);
                ximg[i] = h | (l << 16);
            }
        }
        uint4 wv[W_PER];
#pragma unroll
        for (int u = 0; u < W_PER; ++u) {
            const int i = tid + u * NTHR;
            wv[u] = p.wt[i < nw ? i : nw - 1];   // (unconditional: keeps wv in registers)
        }
        int4 tv = make_int4(0, 0, 0, 0);
        if (tid < p.nk * 8) tv = reinterpret_cast<const int4*>(p.ktab)[tid];
#pragma unroll
        for (int u = 0; u < W_PER; ++u) {
            const int i = tid + u * NTHR;
            if (i < nw) wl[i + 4 * (i / (2 * p.Mpad))] = wv[u];
        }
        if (tid < p.nk * 8) tl[tid] = tv;
    }
    __syncthreads();
    // this lane's two output pixels: rows oy0 + 2w + j, column ox0 + c16 -> window base
    int pbase[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) pbase[j] = (2 * w + j) * p.stride * p.IC + c16 * p.stride;
    const int arow = 8 * (c16 >> 2) + (c16 & 3);
    floatx4 acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < p.nk; ++ks) {
        // A: the weight rows of this lane's K group q (part 0 = h, 1 = l)
        halfx8s fa[MT][2];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int m = 32 * (i >> 1) + 4 * (i & 1) + arow;
#pragma unroll
            for (int pp = 0; pp < 2; ++pp)
                fa[i][pp] = __builtin_bit_cast(halfx8s,
                                               wl[((ks * 4 + q) * 2 + pp) * p.Mpad +
                                                  4 * (ks * 4 + q) + m]);
        }
        // B: 8 K values of each pixel, one LDS word (h | l << 16) each
        const int4 t0 = tl[(ks * 4 + q) * 2], t1 = tl[(ks * 4 + q) * 2 + 1];
        const int tk[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
        halfx8s fb[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint32_t u[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) u[e] = tk[e] >= 0 ? ximg[tk[e] + pbase[j]] : 0u;
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
                hw[e2] = __builtin_amdgcn_perm(u[2 * e2 + 1], u[2 * e2], 0x05040100u);
                lw[e2] = __builtin_amdgcn_perm(u[2 * e2 + 1], u[2 * e2], 0x07060302u);
            }
            fb[j][0] = __builtin_bit_cast(halfx8s, make_uint4(hw[0], hw[1], hw[2], hw[3]));
            fb[j][1] = __builtin_bit_cast(halfx8s, make_uint4(lw[0], lw[1], lw[2], lw[3]));
        }
        // al*bh + ah*bl + ah*bh (small terms first), as FmtF16
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        fa[i][t == 0 ? 1 : 0], fb[j][t == 1 ? 1 : 0], acc[i][j], 0, 0, 0);
    }
    // epilogue: acc * scale + bias, ReLU, S2 split; lane (q, c16) holds group 4 t + q.  Per
    // output row j the wave's 16 pixels x Gout groups are staged in LDS (the weight region,
    // free after the barrier) and written as whole 256-B pixel rows: 16-B pieces at a 32-B
    // stride straight from the MFMA layout leave every line half-written per instruction.
    __syncthreads();
    uint4* stg = wl + w * 256;        // 16 pixels x 16 uint4 (8 groups x 2 parts)
    bool bad = false;
    const int ox = ox0 + c16;
    const int GP = 2 * p.Gout;         // uint4 per pixel
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int oy = oy0 + 2 * w + j;
#pragma unroll
        for (int t = 0; t < MT / 2; ++t) {
            const int g = 4 * t + q;
            if (g >= p.Gout) continue;
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
                uint32_t hh[2], ll[2];
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const int e = 2 * e2 + h2, ch = 8 * g + e;
                    const float a = e < 4 ? acc[2 * t][j][e] : acc[2 * t + 1][j][e - 4];
                    const float y = relu_nan(a * p.wscale[ch] + p.bias[ch]);
                    bad |= fabsf(y) > 65504.f && oy < p.Ho && ox < p.Wo;
                    s2::split2(y, hh[h2], ll[h2]);
                }
                hw[e2] = hh[0] | (hh[1] << 16);
                lw[e2] = ll[0] | (ll[1] << 16);
            }
            stg[c16 * GP + 2 * g] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            stg[c16 * GP + 2 * g + 1] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
        // (LDS accesses of one wave execute in order: the sweep reads what the other lanes
        // of this wave wrote above)
        if (oy < p.Ho) {
            uint4* orow = reinterpret_cast<uint4*>(p.out) + ((long)b * p.Ho + oy) * p.Wo * GP +
                          (long)ox0 * GP;
            for (int i = lane; i < 16 * GP; i += 64) {
                if (ox0 + i / GP < p.Wo) orow[i] = stg[i];
            }
        }
    }
    if (bad && p.oflow) *p.oflow = 1;
}

// Geometry shared by the host entry points: output tiles, window, planar image size.
struct StemGeo {
    int Ho, Wo, tx, ty, IR, IC;
};
StemGeo stem_geo(int H, int W, int KH, int KW, int stride, int pad) {
    StemGeo g;
    g.Ho = (H + 2 * pad - KH) / stride + 1;
    g.Wo = (W + 2 * pad - KW) / stride + 1;
    g.tx = (g.Wo + 15) / 16;
    g.ty = (g.Ho + kTR - 1) / kTR;
    g.IR = (kTR - 1) * stride + KH;
    g.IC = 15 * stride + KW;
    return g;
}

}  // namespace

extern "C" int tcam_stem_window(int KH, int KW, int stride, int* IR, int* IC) {
    TCAM_REQUIRE(KH > 0 && KW > 0 && stride > 0 && IR && IC);
    *IR = (kTR - 1) * stride + KH;
    *IC = 15 * stride + KW;
    return TCAM_OK;
}

extern "C" int tcam_stem_f16x3(const float* img, const void* wt, const float* wscale,
                               const float* bias, const int32_t* ktab, int nk, void* out, int B,
                               int C, int H, int W, int Cout, int KH, int KW, int stride, int pad,
                               int* oflow, void* stream) {
    TCAM_REQUIRE(img && wt && wscale && bias && ktab && out && B > 0 && C > 0);
    TCAM_REQUIRE(H > 0 && W > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0);
    TCAM_REQUIRE(nk > 0 && nk <= kMaxNk && nk * 32 >= C * KH * KW);
    TCAM_REQUIRE(Cout > 0 && Cout % 8 == 0 && Cout <= 64);
    TCAM_REQUIRE(((uintptr_t)wt & 15) == 0 && ((uintptr_t)ktab & 15) == 0 &&
                 ((uintptr_t)out & 15) == 0);
    const StemGeo g = stem_geo(H, W, KH, KW, stride, pad);
    TCAM_REQUIRE(g.Ho > 0 && g.Wo > 0);
    StemArgs p;
    p.img = img;
    p.wt = (const uint4*)wt;
    p.wscale = wscale;
    p.bias = bias;
    p.ktab = ktab;
    p.out = (uint8_t*)out;
    p.oflow = oflow;
    p.C = C;
    p.H = H;
    p.W = W;
    p.pad = pad;
    p.Ho = g.Ho;
    p.Wo = g.Wo;
    p.stride = stride;
    p.nk = nk;
    p.Mpad = Cout <= 32 ? 32 : 64;
    p.Gout = Cout / 8;
    p.IR = g.IR;
    p.IC = g.IC;
    p.tiles_x = g.tx;
    p.tiles_y = g.ty;
    TCAM_REQUIRE((long)C * g.IR * g.IC <= kImgWords &&
                 (long)nk * 8 * p.Mpad + 16 * nk <= kWtUint4);
    TCAM_REQUIRE((long)B * g.tx * g.ty < (1l << 31));
    hipStream_t st = as_stream(stream);
    const unsigned blocks = (unsigned)((long)B * g.tx * g.ty);
    if (p.Mpad == 32)
        timed_launch(stem_f16x3_kernel<2>, dim3(blocks), dim3(64 * kStemWaves), st, p);
    else
        timed_launch(stem_f16x3_kernel<4>, dim3(blocks), dim3(64 * kStemWaves), st, p);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
