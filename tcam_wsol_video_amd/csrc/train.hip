// Training-step kernels of the TCAM decoder:
// the frozen encoder runs the inference path; the U-Net decoder + segmentation head
// train with batch-statistics BatchNorm and the TCAM losses, exactly the reference's
// Trainer._wsol_training (learning/train_wsol.py:685-884) with freeze_cl=True.
//
//   bn_stats        per-channel batch mean / biased var over (B, H, W) in fp64 partials
//                   (fixed-order two-level sum), running-stat update (momentum 0.1,
//                   unbiased var) — nn.BatchNorm2d.train() semantics
//   bn_relu         out = relu(gamma (y - mean) invstd + beta)
//   bn_relu_bwd     g = dout [out > 0]; dgamma = sum g xhat; dbeta = sum g;
//                   dy = gamma invstd (g - dbeta/n - xhat dgamma/n)
//   up2_bwd         gradient of nearest x2 (decoder.py:43): sum of each 2x2 block
//   wgrad           dW[co][c][kh][kw] = sum_p dy[p][co] x[p + tap][c], fp32 MFMA
//                   (v_mfma_f32_32x32x2_f32) over LDS tiles, split over pixels into
//                   fp32 slabs reduced in fixed order (deterministic); sources as the
//                   forward conv (concat of two, nearest-x2 on the first)
//   pack_weight     PyTorch (Cout, Ctot, KH, KW) fp32 -> the split x6 operand; mode 1
//                   packs the transposed, 180-degree-rotated slice used for dgrad (the
//                   data gradient is then the forward x6 convolution of dy)
//   chansum         deterministic per-channel sum of an NCHW fp32 tensor (bias grads)
//   tcam_losses     SelfLearningTcams CE(ignore -255) + ConRanFieldTcams + the ELB size
//                   term of MaxSizePositiveTcams (losses/tcam.py:48-278, elb.py:119-137),
//                   forward values and d loss / d fcams through the 2-way softmax
//   sgd_nesterov    torch.optim.SGD(momentum, dampening, weight_decay, nesterov) step
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "s3_util.h"

using s3::G8;
using s3::load_g8;
using s3::store_g8;

namespace {

constexpr int kB = 256;

// ---------------------------------------------------------------- BN
// Partial sums in fp64 ([chunk][C][2]: x and x^2 for the statistics, g and g*xhat for the
// backward), then one finalize block per channel.  bn_bwd_partial_kernel (the unfused
// backward for C / 8 not dividing 256): grid (chunks, G), a thread strides its chunk's pixels.
constexpr int kChunkPix = 4096;

// Sum of the chunk partials of channel c = blockIdx.x in a fixed order (strided per thread,
// then a fixed tree): one block per channel, deterministic.
__device__ __forceinline__ void chunk_sum2(const double* __restrict__ part, int nchunks, int C,
                                           int c, double& s, double& q) {
    __shared__ double red[kB / 64][2];
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < nchunks; k += kB) {
        a += part[((long)k * C + c) * 2];
        b += part[((long)k * C + c) * 2 + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = a;
        red[threadIdx.x >> 6][1] = b;
    }
    __syncthreads();
    s = q = 0.0;
    for (int w = 0; w < kB / 64; ++w) {
        s += red[w][0];
        q += red[w][1];
    }
}

__global__ __launch_bounds__(kB) void bn_finalize_kernel(const double* __restrict__ part,
                                                         int nchunks, int C, long P, float eps,
                                                         float momentum, float* __restrict__ mean,
                                                         float* __restrict__ invstd,
                                                         float* __restrict__ run_mean,
                                                         float* __restrict__ run_var) {
    const int c = blockIdx.x;
    double s, q;
    chunk_sum2(part, nchunks, C, c, s, q);
    if (threadIdx.x != 0) return;
    const double m = s / (double)P;
    const double var = fmax(q / (double)P - m * m, 0.0);   // biased (normalisation)
    mean[c] = (float)m;
    invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
        const double unb = P > 1 ? var * (double)P / (double)(P - 1) : var;
        run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * m);
        run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
}

template <class L>
__global__ __launch_bounds__(kB) void bn_relu_kernel(const uint8_t* __restrict__ y,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ invstd,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     uint8_t* __restrict__ out, long total,
                                                     int G) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    G8 v = L::load(y + i * L::GB);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        const float xh = (v.v[e] - mean[c]) * invstd[c];
        // (an explicit fma: the fused backward recomputes this pre-activation bit for bit to
        // take the ReLU's mask from y instead of reading the output)
        v.v[e] = relu_nan(__builtin_fmaf(gamma[c], xh, beta[c]));
    }
    L::store(out + i * L::GB, v);
}

// backward partials: sum g and sum g * xhat (g = dout masked by relu(out) > 0).
// L: the layout of the gradients (dout, dy); LA: of the forward's activations (out, y) —
// the f16x3 training step keeps activations in S2 and gradients in S3.
template <class L, class LA = L>
__global__ __launch_bounds__(kB) void bn_bwd_partial_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, long P, int G, double* __restrict__ part) {
    const int g = blockIdx.y;
    const long p0 = (long)blockIdx.x * kChunkPix;
    const long p1 = min(P, p0 + kChunkPix);
    double s[8], q[8];
    float mu[8], is[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s[e] = q[e] = 0.0;
        mu[e] = mean[8 * g + e];
        is[e] = invstd[8 * g + e];
    }
    for (long p = p0 + threadIdx.x; p < p1; p += kB) {
        const long gi = p * G + g;
        const G8 d = L::load(dout + gi * L::GB), o = LA::load(out + gi * LA::GB),
                 v = LA::load(y + gi * LA::GB);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float gg = o.v[e] > 0.f ? d.v[e] : 0.f;
            const float xh = (v.v[e] - mu[e]) * is[e];
            s[e] += (double)gg;
            q[e] += (double)gg * (double)xh;
        }
    }
    __shared__ double red[kB / 64][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        for (int o = 32; o > 0; o >>= 1) {
            s[e] += __shfl_xor(s[e], o, 64);
            q[e] += __shfl_xor(q[e], o, 64);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            red[w][e] = s[e];
            red[w][8 + e] = q[e];
        }
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        double t = 0.0;
        for (int i = 0; i < kB / 64; ++i) t += red[i][threadIdx.x];
        const int e = threadIdx.x & 7, which = threadIdx.x >> 3;
        part[((long)blockIdx.x * G * 8 + g * 8 + e) * 2 + which] = t;
    }
}

// The same partials with coalesced reads: a block owns kBwdChunkPix pixels x all G groups,
// consecutive threads take consecutive 48-byte groups (kB % G == 0, so each thread keeps one
// group), and the threads of one group are summed in fixed order (deterministic).
constexpr int kBwdChunkPix = 512;

template <class L, class LA = L>
__global__ __launch_bounds__(kB) void bn_bwd_partial_co_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, long P, int G, double* __restrict__ part) {
    const long i0 = (long)blockIdx.x * kBwdChunkPix * G;
    const long i1 = min(P * G, i0 + (long)kBwdChunkPix * G);
    const int g = threadIdx.x % G;
    double s[8], q[8];
    float mu[8], is[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s[e] = q[e] = 0.0;
        mu[e] = mean[8 * g + e];
        is[e] = invstd[8 * g + e];
    }
    for (long i = i0 + threadIdx.x; i < i1; i += kB) {
        const G8 d = L::load(dout + i * L::GB), o = LA::load(out + i * LA::GB),
                 v = LA::load(y + i * LA::GB);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float gg = o.v[e] > 0.f ? d.v[e] : 0.f;
            const float xh = (v.v[e] - mu[e]) * is[e];
            s[e] += (double)gg;
            q[e] += (double)gg * (double)xh;
        }
    }
    __shared__ double red[kB][17];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        red[threadIdx.x][e] = s[e];
        red[threadIdx.x][8 + e] = q[e];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < G * 16; r += kB) {
        const int gg = r >> 4, k = r & 15;
        double t = 0.0;
        for (int j = gg; j < kB; j += G) t += red[j][k];
        const int e = k & 7, which = k >> 3;
        part[((long)blockIdx.x * G * 8 + gg * 8 + e) * 2 + which] = t;
    }
}

__global__ __launch_bounds__(kB) void bn_bwd_finalize_kernel(const double* __restrict__ part,
                                                             int nchunks, int C,
                                                             float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta,
                                                             float* __restrict__ coef) {
    const int c = blockIdx.x;
    double s, q;
    chunk_sum2(part, nchunks, C, c, s, q);
    if (threadIdx.x != 0) return;
    dbeta[c] = (float)s;
    dgamma[c] = (float)q;
    coef[2 * c] = (float)s;
    coef[2 * c + 1] = (float)q;
}

template <class L, class LA = L>
__global__ __launch_bounds__(kB) void bn_bwd_apply_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ coef, float inv_n, uint8_t* __restrict__ dy, long total, int G) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    const G8 d = L::load(dout + i * L::GB), o = LA::load(out + i * LA::GB),
             v = LA::load(y + i * LA::GB);
    G8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        const float gg = o.v[e] > 0.f ? d.v[e] : 0.f;
        const float xh = (v.v[e] - mean[c]) * invstd[c];
        r.v[e] = gamma[c] * invstd[c] *
                 (gg - coef[2 * c] * inv_n - xh * (coef[2 * c + 1] * inv_n));
    }
    L::store(dy + i * L::GB, r);
}

// The same with the per-channel max |dy| folded in (the f16x3 step's dy scales): a fixed
// grid strides over the groups (the stride is a multiple of G, so a thread keeps one
// channel group), per-block maxima in LDS, one global atomicMax per block and channel
// (non-negative floats order as their bit patterns).
template <class L, class LA>
__global__ __launch_bounds__(kB) void bn_bwd_apply_amax_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ coef, float inv_n, uint8_t* __restrict__ dy, long total, int G,
    uint32_t* __restrict__ amax) {
    __shared__ uint32_t red[2048];
    for (int k = threadIdx.x; k < G * 8; k += kB) red[k] = 0u;
    __syncthreads();
    const long i0 = (long)blockIdx.x * kB + threadIdx.x;
    const int g = (int)(i0 % G);
    float cm[8], ci[8], cg[8], c0[8], c1[8], m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        cm[e] = mean[c];
        ci[e] = invstd[c];
        cg[e] = gamma[c] * invstd[c];
        c0[e] = coef[2 * c] * inv_n;
        c1[e] = coef[2 * c + 1] * inv_n;
        m[e] = 0.f;
    }
    const long stride = (long)gridDim.x * kB;
    for (long i = i0; i < total; i += stride) {
        const G8 d = L::load(dout + i * L::GB), o = LA::load(out + i * LA::GB),
                 v = LA::load(y + i * LA::GB);
        G8 r;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float gg = o.v[e] > 0.f ? d.v[e] : 0.f;
            const float xh = (v.v[e] - cm[e]) * ci[e];
            r.v[e] = cg[e] * (gg - c0[e] - xh * c1[e]);
            m[e] = fmaxf(m[e], fabsf(r.v[e]));
        }
        L::store(dy + i * L::GB, r);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicMax(&red[g * 8 + e], __float_as_uint(m[e]));
    __syncthreads();
    for (int k = threadIdx.x; k < G * 8; k += kB)
        if (red[k]) atomicMax(&amax[k], red[k]);
}

// ---- the fused BN-ReLU backward of the f16x3 steps (round 6): dy goes straight to the
// per-channel scaled S2 copy the MFMA gradients read (no S3 dy, no max pass, no re-split),
// with the scale from a bound: |dy_c| <= |gamma invstd| (max|g| + |mean g| + max|xh|
// |mean g xh|), so max|dy_c| s_c < 2^15 holds without knowing the exact max (the bound is
// within a small factor of it: values down to ~2^-15 of the channel max keep all 22 bits).
// MASKY: the ReLU mask is recomputed from y (pre-activation gamma xh + beta > 0, the
// forward's fma bit for bit) instead of read from the output (a BN-ReLU; the Bottleneck
// tail's mask includes the shortcut and reads `out`).
// the stored activation of pre-activation z in layout LA is > 0: z as that layout rounds it
// (S1: fp16(z); S2: fp16(z) + fp16(z - fp16(z)) — a z below fp16's subnormal range stores 0)
template <class LA>
__device__ __forceinline__ bool stored_pos(float z) {
    if constexpr (LA::GB == 16) return (float)(_Float16)z > 0.f;
    if constexpr (LA::GB == 32) {
        const float h = (float)(_Float16)z;
        return h + (float)(_Float16)(z - h) > 0.f;
    }
    return z > 0.f;
}

template <class LA, bool MASKY>
__device__ __forceinline__ float bwd_g(float d, float o, float xh, float gm, float bt) {
    if (MASKY) return stored_pos<LA>(__builtin_fmaf(gm, xh, bt)) ? d : 0.f;
    return o > 0.f ? d : 0.f;
}

// the channel's [max |g|, max |xh|] over the chunks' partial maxima (pmax [chunk][C][2])
__device__ __forceinline__ void chunk_max2(const float* __restrict__ pmax, int nchunks, int C,
                                           int c, float& ma, float& mb) {
    __shared__ float red[kB / 64][2];
    float a = 0.f, b = 0.f;
    for (int k = threadIdx.x; k < nchunks; k += kB) {
        a = fmaxf(a, pmax[((long)k * C + c) * 2]);
        b = fmaxf(b, pmax[((long)k * C + c) * 2 + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        a = fmaxf(a, __shfl_xor(a, o, 64));
        b = fmaxf(b, __shfl_xor(b, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = a;
        red[threadIdx.x >> 6][1] = b;
    }
    __syncthreads();
    ma = mb = 0.f;
    for (int w = 0; w < kB / 64; ++w) {
        ma = fmaxf(ma, red[w][0]);
        mb = fmaxf(mb, red[w][1]);
    }
}

__global__ __launch_bounds__(kB) void bn_bwd_finalize_sc_kernel(
    const double* __restrict__ part, int nchunks, int C, long P, const float* __restrict__ gamma,
    const float* __restrict__ invstd, const float* __restrict__ pmax,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ coef,
    float* __restrict__ scale) {
    const int c = blockIdx.x;
    double s, q;
    chunk_sum2(part, nchunks, C, c, s, q);
    float gmx = 0.f, xmx = 0.f;
    if (scale) chunk_max2(pmax, nchunks, C, c, gmx, xmx);
    if (threadIdx.x != 0) return;
    dbeta[c] = (float)s;
    dgamma[c] = (float)q;
    coef[2 * c] = (float)s;
    coef[2 * c + 1] = (float)q;
    if (!scale) return;
    const double n = (double)P;
    const double bound = fabs((double)gamma[c] * (double)invstd[c]) *
                         ((double)gmx + fabs(s) / n + (double)xmx * fabs(q) / n);
    int k = 0;
    if (bound > 0.0 && isfinite(bound)) {
        int ex = 0;
        frexp(bound, &ex);   // bound in [2^(ex-1), 2^ex)
        k = max(-126, min(126, 15 - ex));
    }
    scale[c] = ldexpf(1.f, k);
}

// ---- coalesced partial sums over a 2-D grid (round 6): block (k, j) of (nchunks, G / GS)
// reduces chunk k's pixels for the GS channel groups of slice j; its kB threads are GS
// groups x NL = kB / GS pixel lanes, so consecutive threads read consecutive 8-channel groups
// (GS x GB contiguous bytes per pixel) and a launch has ~kBnBlocks blocks whatever C is.  The
// one-group-per-thread kernels above give a deep layer (P = 25088, C = 2048) 49 blocks
// (bwd) or strided 32-byte reads (bn_partial_kernel): 1.5-1.7 TB/s.  The NL lanes of a group
// are summed in fixed order (deterministic); partials keep the [chunk][C][2] layout.
constexpr int kBnBlocks = 1024;

struct BnPlan {
    int GS, NL, nchunks;
    long cp;   // pixels per chunk (a multiple of NL)
};

static BnPlan bn_plan(long P, int G) {
    BnPlan b;
    b.GS = 1;
    while (b.GS < 32 && G % (2 * b.GS) == 0 && kB % (2 * b.GS) == 0) b.GS *= 2;
    b.NL = kB / b.GS;
    const long slices = G / b.GS;
    long cp = (P * slices + kBnBlocks - 1) / kBnBlocks;
    cp = std::max<long>(cp, 4L * b.NL);
    b.cp = (cp + b.NL - 1) / b.NL * b.NL;
    b.nchunks = (int)((P + b.cp - 1) / b.cp);
    return b;
}

// the block's 16 sums (+ 16 maxima when MX) per thread -> one partial row per channel
template <bool MX>
__device__ __forceinline__ void bn_fold_write(const double (&s)[8], const double (&q)[8],
                                              const float (&ma)[8], const float (&mb)[8], int GS,
                                              int j, int k, int C, double* __restrict__ part,
                                              float* __restrict__ pmax) {
    __shared__ double red[kB][17];
    __shared__ float rmx[MX ? kB : 1][17];
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        red[t][e] = s[e];
        red[t][8 + e] = q[e];
        if (MX) {
            rmx[t][e] = ma[e];
            rmx[t][8 + e] = mb[e];
        }
    }
    __syncthreads();
    const int NL = kB / GS;
    for (int r = t; r < GS * 16; r += kB) {
        const int gl = r >> 4, kk = r & 15;
        double acc = 0.0;
        float m = 0.f;
        for (int l = 0; l < NL; ++l) {
            acc += red[l * GS + gl][kk];
            if (MX) m = fmaxf(m, rmx[l * GS + gl][kk]);
        }
        const int c = (j * GS + gl) * 8 + (kk & 7), which = kk >> 3;
        part[((long)k * C + c) * 2 + which] = acc;
        if (MX && pmax) pmax[((long)k * C + c) * 2 + which] = m;
    }
}

template <class L>
__global__ __launch_bounds__(kB) void bn_stats_co_kernel(const uint8_t* __restrict__ y, long P,
                                                         int G, int GS, long cp,
                                                         double* __restrict__ part) {
    const int k = blockIdx.x, j = blockIdx.y, t = threadIdx.x;
    const int NL = kB / GS, g = j * GS + t % GS;
    const long p1 = min(P, (long)k * cp + cp);
    double s[8], q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.0;
    auto acc = [&](const G8& v) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            s[e] += (double)v.v[e];
            q[e] += (double)v.v[e] * (double)v.v[e];
        }
    };
    long p = (long)k * cp + t / GS;
    for (; p + NL < p1; p += 2 * NL) {
        const G8 a = L::load(y + (p * G + g) * L::GB), b = L::load(y + ((p + NL) * G + g) * L::GB);
        acc(a);
        acc(b);
    }
    if (p < p1) acc(L::load(y + (p * G + g) * L::GB));
    const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bn_fold_write<false>(s, q, z, z, GS, j, k, G * 8, part, nullptr);
}

template <class LG, class LA, bool MASKY>
__global__ __launch_bounds__(kB) void bn_bwd_partial_sc2_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, long P, int G, int GS, long cp, double* __restrict__ part,
    float* __restrict__ pmax) {
    const int k = blockIdx.x, j = blockIdx.y, t = threadIdx.x;
    const int NL = kB / GS, g = j * GS + t % GS;
    const long p1 = min(P, (long)k * cp + cp);
    double s[8], q[8];
    float mu[8], is[8], gm[8], bt[8], mg[8], mx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s[e] = q[e] = 0.0;
        mu[e] = mean[8 * g + e];
        is[e] = invstd[8 * g + e];
        gm[e] = gamma[8 * g + e];
        bt[e] = beta[8 * g + e];
        mg[e] = mx[e] = 0.f;
    }
    auto acc = [&](const G8& d, const G8& o, const G8& v) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float xh = (v.v[e] - mu[e]) * is[e];
            const float gg = bwd_g<LA, MASKY>(d.v[e], MASKY ? 0.f : o.v[e], xh, gm[e], bt[e]);
            s[e] += (double)gg;
            q[e] += (double)gg * (double)xh;
            mg[e] = fmaxf(mg[e], fabsf(gg));
            mx[e] = fmaxf(mx[e], fabsf(xh));
        }
    };
    long p = (long)k * cp + t / GS;
    G8 o0 = {}, o1 = {};
    for (; p + NL < p1; p += 2 * NL) {
        const long i0 = p * G + g, i1 = (p + NL) * G + g;
        const G8 d0 = LG::load(dout + i0 * LG::GB), v0 = LA::load(y + i0 * LA::GB);
        const G8 d1 = LG::load(dout + i1 * LG::GB), v1 = LA::load(y + i1 * LA::GB);
        if (!MASKY) {
            o0 = LA::load(out + i0 * LA::GB);
            o1 = LA::load(out + i1 * LA::GB);
        }
        acc(d0, o0, v0);
        acc(d1, o1, v1);
    }
    if (p < p1) {
        const long i0 = p * G + g;
        if (!MASKY) o0 = LA::load(out + i0 * LA::GB);
        acc(LG::load(dout + i0 * LG::GB), o0, LA::load(y + i0 * LA::GB));
    }
    bn_fold_write<true>(s, q, mg, mx, GS, j, k, G * 8, part, pmax);
}

// The fused backward's apply pass: dy = gamma invstd (g - mean g - xh mean(g xh)), written as
// dy3 (the gradients' layout) and / or its scaled S2 copy dy2, over a fixed grid whose stride
// is a multiple of G (kB % G == 0): the channel parameters read once per thread into registers
// (a per-element form issued seven waited-on parameter loads per element), two elements
// loaded before either is computed.
template <class LG, class LA, bool MASKY>
__global__ __launch_bounds__(kB) void bn_bwd_apply_sc2_kernel(
    const uint8_t* __restrict__ dout, const uint8_t* __restrict__ out,
    const uint8_t* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ coef,
    const float* __restrict__ scale, float inv_n, uint8_t* __restrict__ dy3,
    uint8_t* __restrict__ dy2, long total, int G) {
    const int g = (int)(threadIdx.x % (unsigned)G);
    float mu[8], is[8], gm[8], bt[8], k0[8], k1[8], sc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        mu[e] = mean[c];
        is[e] = invstd[c];
        gm[e] = gamma[c];
        bt[e] = beta[c];
        k0[e] = coef[2 * c];
        k1[e] = coef[2 * c + 1];
        sc[e] = scale ? scale[c] : 0.f;
    }
    auto apply = [&](long i, const G8& d, const G8& o, const G8& v) {
        G8 r, rs;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float xh = (v.v[e] - mu[e]) * is[e];
            const float gg = bwd_g<LA, MASKY>(d.v[e], MASKY ? 0.f : o.v[e], xh, gm[e], bt[e]);
            r.v[e] = gm[e] * is[e] * (gg - k0[e] * inv_n - xh * (k1[e] * inv_n));
            rs.v[e] = r.v[e] * sc[e];   // a power of two: exact
        }
        if (dy3) LG::store(dy3 + i * LG::GB, r);
        if (dy2) LayS2::store(dy2 + i * LayS2::GB, rs);
    };
    const long stride = (long)gridDim.x * kB;
    long i = (long)blockIdx.x * kB + threadIdx.x;
    G8 o0 = {}, o1 = {};
    for (; i + stride < total; i += 2 * stride) {
        const long i1 = i + stride;
        const G8 d0 = LG::load(dout + i * LG::GB), v0 = LA::load(y + i * LA::GB);
        const G8 d1 = LG::load(dout + i1 * LG::GB), v1 = LA::load(y + i1 * LA::GB);
        if (!MASKY) {
            o0 = LA::load(out + i * LA::GB);
            o1 = LA::load(out + i1 * LA::GB);
        }
        apply(i, d0, o0, v0);
        apply(i1, d1, o1, v1);
    }
    if (i < total) {
        if (!MASKY) o0 = LA::load(out + i * LA::GB);
        apply(i, LG::load(dout + i * LG::GB), o0, LA::load(y + i * LA::GB));
    }
}

// ------------------------------------------------------------ up2 bwd
template <class L>
__global__ __launch_bounds__(kB) void up2_bwd_kernel(const uint8_t* __restrict__ gu,
                                                     uint8_t* __restrict__ gx, int G, int H,
                                                     int W, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const long b = t / H;
    const int W2 = 2 * W;
    G8 acc;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc.v[e] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const G8 v =
                L::load(gu + ((((b * 2 * H) + 2 * y + dy) * W2 + 2 * x + dx) * G + g) * L::GB);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc.v[e] += v.v[e];
        }
    L::store(gx + i * L::GB, acc);
}

// -------------------------------------------------- up2 + resize bwd
// Adjoint of up2_resize_s3 (nearest x2 to (2H, 2W), then bilinear align_corners=True to
// (Ho, Wo); decoder.py:43-51) as a gather: low-res pixel (y, x) collects, for every output
// (oy, ox) whose bilinear taps hit its 2x2 upsampled block, g * wy * wx.  Deterministic.
__device__ __forceinline__ float up_weight(int o, int lowi, float sc, int Hu) {
    // weight with which output row o reads upsampled rows {2 lowi, 2 lowi + 1}
    const float r = sc * (float)o;
    const int u0 = (int)r;
    const int u1 = u0 + (u0 < Hu - 1 ? 1 : 0);
    const float l1 = fminf(fmaxf(r - (float)u0, 0.f), 1.f), l0 = 1.f - l1;
    float w = 0.f;
    if ((u0 >> 1) == lowi) w += l0;
    if ((u1 >> 1) == lowi) w += l1;
    return w;
}

template <class L>
__global__ __launch_bounds__(kB) void up2_resize_bwd_kernel(const uint8_t* __restrict__ g,
                                                            uint8_t* __restrict__ gx, int G,
                                                            int H, int W, int Ho, int Wo,
                                                            float sh, float sw, long total) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= total) return;
    const int gg = (int)(i % G);
    long t = i / G;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const long b = t / H;
    // outputs whose source coordinate lies within one upsampled pixel of this block
    const int oy0 = max(0, (int)floorf((2.f * y - 1.f) / fmaxf(sh, 1e-6f)) - 1);
    const int oy1 = min(Ho - 1, (int)ceilf((2.f * y + 2.f) / fmaxf(sh, 1e-6f)) + 1);
    const int ox0 = max(0, (int)floorf((2.f * x - 1.f) / fmaxf(sw, 1e-6f)) - 1);
    const int ox1 = min(Wo - 1, (int)ceilf((2.f * x + 2.f) / fmaxf(sw, 1e-6f)) + 1);
    G8 acc;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc.v[e] = 0.f;
    for (int oy = (sh > 0.f ? oy0 : 0); oy <= (sh > 0.f ? oy1 : Ho - 1); ++oy) {
        const float wy = up_weight(oy, y, sh, 2 * H);
        if (wy == 0.f) continue;
        for (int ox = (sw > 0.f ? ox0 : 0); ox <= (sw > 0.f ? ox1 : Wo - 1); ++ox) {
            const float wx = up_weight(ox, x, sw, 2 * W);
            if (wx == 0.f) continue;
            const G8 v = L::load(g + (((b * Ho + oy) * Wo + ox) * G + gg) * L::GB);
            const float w = wy * wx;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc.v[e] += w * v.v[e];
        }
    }
    L::store(gx + i * L::GB, acc);
}

// ------------------------------------------------------------- wgrad
struct WSrc {
    const uint8_t* p;
    int C, H, W, stride, up2, G;
};

struct WgArgs {
    WSrc s[2];
    int c0, Ctot;
    const uint8_t* dy;
    int Cout, Gout, Hout, Wout, KH, KW, pad_h, pad_w;
    long P;
    int ntm, nct, ntiles;
    long chunk;   // pixels per split (multiple of kWK)
    float* part;  // [split][tile][64][64]
};

constexpr int kWT = 64;   // tile (co) x (channels of one tap)
constexpr int kWK = 16;   // pixels per K-step
constexpr int kLP = kWT + 4;

template <class L, class LX = L>
__global__ __launch_bounds__(kB) void wgrad_kernel(WgArgs a) {
    __shared__ float As[kWK][kLP];
    __shared__ float Bs[kWK][kLP];
    const int tile = blockIdx.x;
    const int split = blockIdx.y;
    const int mt = tile % a.ntm;
    const int rest = tile / a.ntm;
    const int ct = rest % a.nct;
    const int tap = rest / a.nct;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const long p0 = (long)split * a.chunk;
    const long p1 = min(a.P, p0 + a.chunk);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int HWo = a.Hout * a.Wout;
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    // loader roles: tid < 128 -> A (dy), else B (x); item = (pixel, group)
    const int item = tid & 127;
    const int lp = item >> 3, lg = item & 7;
    const bool isA = tid < 128;
    for (long pb = p0; pb < p1; pb += kWK) {
        const long p = pb + lp;
        G8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v.v[e] = 0.f;
        if (p < p1) {
            if (isA) {
                const int co0 = mt * kWT + lg * 8;
                if (co0 < a.Cout) v = L::load(a.dy + (p * a.Gout + co0 / 8) * L::GB);
            } else {
                const int c = ct * kWT + lg * 8;
                if (c < a.Ctot) {
                    const int si = c < a.c0 ? 0 : 1;
                    const WSrc& s = a.s[si];
                    const int cl = c - (si ? a.c0 : 0);
                    const long b = p / HWo;
                    const int r = (int)(p - b * HWo);
                    const int oy = r / a.Wout, ox = r - oy * a.Wout;
                    int iy = oy * s.stride - a.pad_h + kh;
                    int ix = ox * s.stride - a.pad_w + kw;
                    const int Hs = s.up2 ? 2 * s.H : s.H, Ws = s.up2 ? 2 * s.W : s.W;
                    if ((unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws) {
                        if (s.up2) {
                            iy >>= 1;
                            ix >>= 1;
                        }
                        v = LX::load(s.p + (((b * s.H + iy) * s.W + ix) * s.G + cl / 8) *
                                     LX::GB);
                    }
                }
            }
        }
        float* dst = isA ? &As[lp][lg * 8] : &Bs[lp][lg * 8];
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = v.v[e];
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kWK; kk += 2) {
            const float av = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
            const float bv = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    float* out = a.part + ((long)split * a.ntiles + tile) * (kWT * kWT);
    const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int m = wm * 32 + 8 * (j >> 2) + 4 * h + (j & 3);
        const int n = wn * 32 + r32;
        out[m * kWT + n] = acc[j];
    }
}

// ---- wgrad for 3x3 / stride 1 / pad 1 (every trainable decoder conv and the seg head):
// spatial patches of 2 rows x 32 columns; the x halo (4 x 34 pixels x 32 channels) and the
// dy patch (64 pixels x 32*MSUB channels) are staged in LDS once per patch and all nine
// taps read the halo shifted, so each x element is fetched from memory once per tile
// instead of nine times.  Wave (msub, kh) owns the three taps (kh, 0..2) of one 32-row
// M subtile: 3 x 16 fp32 accumulators, v_mfma_f32_32x32x2_f32.
constexpr int kPR = 2, kPC = 32, kPX = kPC + 2, kPY = kPR + 2, kXCP = 33;

struct W33Args {
    WSrc s[2];
    int c0, Ctot;
    const uint8_t* dy;
    int Cout, Gout, H, W;
    long npatch;
    int prow, pcol;        // patches per frame: rows, columns
    int ntm, ncb, ntiles;
    long ppb;              // patches per split
    float* part;           // [split][tile][32 MSUB][288]
    const float* dscale;   // WgF3: per-dy-channel power-of-two scale (dy is then S2 scaled)
    int* oflow;            // WgF3: set when an x value leaves the fp16 range (or null)
};

template <int MSUB>
__global__ __launch_bounds__(192 * MSUB) void wgrad33_kernel(W33Args a) {
    constexpr int NT = 192 * MSUB;
    constexpr int MT = 32 * MSUB;
    constexpr int DP = MT + 1;
    __shared__ float xs[kPY][kPX][kXCP];
    __shared__ float ds[kPR * kPC][DP];
    const int tile = blockIdx.x;
    const int mt = tile % a.ntm, cb = tile / a.ntm;
    const long q0 = (long)blockIdx.y * a.ppb;
    const long q1 = min(a.npatch, q0 + a.ppb);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int msub = wave / 3, kh = wave % 3;
    floatx16 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    const int per_frame = a.prow * a.pcol;
    for (long q = q0; q < q1; ++q) {
        const long b = q / per_frame;
        const int r = (int)(q - b * per_frame);
        const int y0 = (r / a.pcol) * kPR, x0 = (r % a.pcol) * kPC;
        // x halo: rows y0-1 .. y0+2, cols x0-1 .. x0+32, 4 channel groups of block cb
        for (int it = tid; it < kPY * kPX * 4; it += NT) {
            const int g = it & 3, pix = it >> 2;
            const int hy = pix / kPX, hx = pix - hy * kPX;
            const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
            const int c = cb * 32 + g * 8;
            G8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e) v.v[e] = 0.f;
            if (c < a.Ctot && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
                const int si = c < a.c0 ? 0 : 1;
                const WSrc& sx = a.s[si];
                const int cl = c - (si ? a.c0 : 0);
                const int sy = sx.up2 ? iy >> 1 : iy, sxx = sx.up2 ? ix >> 1 : ix;
                v = load_g8(sx.p + (((b * sx.H + sy) * sx.W + sxx) * sx.G + cl / 8) * 48);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) xs[hy][hx][g * 8 + e] = v.v[e];
        }
        // dy patch: 64 pixels x MT channels
        for (int it = tid; it < kPR * kPC * (MT / 8); it += NT) {
            const int g = it % (MT / 8), pix = it / (MT / 8);
            const int py = pix / kPC, px = pix - py * kPC;
            const int oy = y0 + py, ox = x0 + px;
            const int co = mt * MT + g * 8;
            G8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e) v.v[e] = 0.f;
            if (co < a.Cout && oy < a.H && ox < a.W)
                v = load_g8(a.dy + (((b * a.H + oy) * a.W + ox) * a.Gout + co / 8) * 48);
#pragma unroll
            for (int e = 0; e < 8; ++e) ds[pix][g * 8 + e] = v.v[e];
        }
        __syncthreads();
#pragma unroll 4
        for (int k0 = 0; k0 < kPR * kPC; k0 += 2) {
            const int k = k0 + (lane >> 5);
            const int py = k / kPC, px = k - py * kPC;
            const float av = ds[k][msub * 32 + (lane & 31)];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const float bv = xs[py + kh][px + kw][lane & 31];
                acc[kw] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[kw], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float* out = a.part + ((long)blockIdx.y * a.ntiles + tile) * (MT * 288);
    const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int m = msub * 32 + 8 * (j >> 2) + 4 * h + (j & 3);
            out[m * 288 + tap * 32 + r32] = acc[kw][j];
        }
    }
}

// ---- the same 3x3 wgrad on the bf16 MFMA at fp32 accuracy ("x6", as conv_x6.hip): dy
// and x are S3 (each value = hi + mid + lo, three bf16 parts), and every product keeps
// the six cross terms of order <= 2, accumulated in fp32 by v_mfma_f32_32x32x16_bf16.
// The reduction runs over pixels, which are not the contiguous axis of S3, so the LDS
// images stay pixel-major ([part][pixel][channel], as loaded) and the MFMA operands are
// gathered with ds_read_b64_tr_b16: a 16-lane group reads a 4-pixel x 16-channel block
// and lane i receives channel i of the 4 pixels, i.e. 4 consecutive K of one row/column.
// Two such reads make a 32x32x16 fragment.  x rows are halo pixels, so the tap shift
// (kh, kw) is only a row offset.  Wave kh owns MSUB 32-row subtiles x the three taps
// (kh, 0..2); partial slabs and their reduction are wgrad33's.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));

typedef _Float16 halfx8w __attribute__((ext_vector_type(8)));

// Operand formats of the 3x3 wgrad: x6 (S3, three bf16 parts, six cross terms on the bf16
// MFMA), H1 (S1, the AMP path: one fp16 part, one product on the fp16 MFMA) and F3 (S3
// operands as two fp16 parts, three terms on the fp16 MFMA: f16x3).  NP = parts per value in
// LDS, XPIN / DPIN = parts per x / dy value in memory.
struct WgX6 {
    static constexpr int NP = 3, XPIN = 3, DPIN = 3, NTERM = 6;
    using V8 = bf16x8w;
    // term t multiplies dy part ta(t) by x part tb(t): small terms first, hi*hi last
    static constexpr int ta(int t) { return t == 0 ? 2 : (t == 2 || t == 3) ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 2 : (t == 2 || t == 4) ? 1 : 0; }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
struct WgH1 {
    static constexpr int NP = 1, XPIN = 1, DPIN = 1, NTERM = 1;
    using V8 = halfx8w;
    static constexpr int ta(int) { return 0; }
    static constexpr int tb(int) { return 0; }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};
// f16x3 on the fp32-accurate (S3) training tensors: each value v (x unscaled, dy times its
// channel's power-of-two scale s, max|dy| s in [2^14, 2^15): the activation gradients are
// ~1e-7, far below fp16's normal range) is split as conv_x6.hip's S2, h = rne_f16(v),
// l = rne_f16(v - h), and a product keeps dl*xh + dh*xl + dh*xh (the dropped dl*xl
// < 2^-22 |dy x|); the reduction divides by s exactly.  dy is re-split once into a scaled
// S2 copy (it is read once per 32-channel block of x); x (S3) is re-split on load.
struct WgF3 {
    static constexpr int NP = 2, XPIN = 3, DPIN = 2, NTERM = 3;
    using V8 = halfx8w;
    static constexpr int ta(int t) { return t == 0 ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 1 : 0; }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

// f16x3 on S2 operands (the f16x3 training step): x is S2 (the forward's activations), dy
// the caller's per-channel scaled S2 copy (tcam_dy_scaled_s2); no re-split on load.
struct WgF2 {
    static constexpr int NP = 2, XPIN = 2, DPIN = 2, NTERM = 3;
    using V8 = halfx8w;
    static constexpr int ta(int t) { return t == 0 ? 1 : 0; }
    static constexpr int tb(int t) { return t == 1 ? 1 : 0; }
    static __device__ __forceinline__ floatx16 mfma32(V8 a, V8 b, floatx16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

// one S3 group (three 16-B bf16 parts) -> the S2 parts (h, l) of its 8 values, each times
// sc[e] when SCALED; returns whether a value falls outside fp16's range
template <bool SCALED>
__device__ __forceinline__ bool s3_resplit(const uint4* p, const float* sc, uint4& h,
                                           uint4& l) {
    const uint32_t hw[4] = {p[0].x, p[0].y, p[0].z, p[0].w};
    const uint32_t mw[4] = {p[1].x, p[1].y, p[1].z, p[1].w};
    const uint32_t lw[4] = {p[2].x, p[2].y, p[2].z, p[2].w};
    uint32_t ho[4], lo[4];
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t hh[2], ll[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float v = e ? (s3::bf_hi(hw[i]) + s3::bf_hi(mw[i])) + s3::bf_hi(lw[i])
                        : (s3::bf_lo(hw[i]) + s3::bf_lo(mw[i])) + s3::bf_lo(lw[i]);
            if (SCALED) v *= sc[2 * i + e];
            bad |= fabsf(v) >= 65520.f;   // rounds to fp16 infinity
            s2::split2(v, hh[e], ll[e]);
        }
        ho[i] = hh[0] | (hh[1] << 16);
        lo[i] = ll[0] | (ll[1] << 16);
    }
    h = make_uint4(ho[0], ho[1], ho[2], ho[3]);
    l = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    return bad;
}

template <class F, int MSUB>
struct W33X6 {
    static constexpr int MT = 32 * MSUB;
    static constexpr int NT = 192;                       // 3 waves (kh)
    static constexpr int NP = F::NP;
    static constexpr int XGB = 16 * F::XPIN;             // bytes per 8-channel group (memory)
    static constexpr int DGB = 16 * F::DPIN;
    static constexpr int XROW = 64;                      // bytes per halo pixel (32 ch)
    static constexpr int XPART = kPY * kPX * XROW;       // 8704 B per part
    // dy row stride: MT channels, padded so that 4 consecutive rows fall in distinct
    // quarters of the 64 banks (stride = 64 mod 128 bytes): conflict-free tr reads
    static constexpr int DROW = MT * 2 + ((MT * 2) % 128 == 0 ? 64 : 0);
    static constexpr int DPART = kPR * kPC * DROW;
    static constexpr int LDS_BYTES = NP * XPART + NP * DPART;
};

__device__ __forceinline__ v4i16 tr_read(const uint8_t* lds, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(lds + off));
}

template <class V8>
__device__ __forceinline__ V8 frag(v4i16 a, v4i16 b) {
    const v8i16 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(V8, v);
}

template <class F, int MSUB, bool PIPE = false>
__global__ __launch_bounds__(192) void wgrad33x6_kernel(W33Args a) {
    using C = W33X6<F, MSUB>;
    constexpr int NP = F::NP;
    using V8 = typename F::V8;
    constexpr int MT = C::MT;
    __shared__ __attribute__((aligned(16))) uint8_t lds[C::LDS_BYTES];
    uint8_t* ximg = lds;
    uint8_t* dimg = lds + NP * C::XPART;
    const int tile = blockIdx.x;
    const int mt = tile % a.ntm, cb = tile / a.ntm;
    const long q0 = (long)blockIdx.y * a.ppb;
    const long q1 = min(a.npatch, q0 + a.ppb);
    const int tid = threadIdx.x, lane = tid & 63;
    const int kh = __builtin_amdgcn_readfirstlane(tid >> 6);
    // transposed-read lane roles (see the header comment)
    const int g16 = lane >> 4, i16 = lane & 15;
    const int rq = i16 >> 2, cp = i16 & 3;
    const int hh = g16 >> 1;
    const int colb = 16 * (g16 & 1) + 4 * cp;   // first of the 4 columns this lane addresses
    floatx16 acc[MSUB][3];
#pragma unroll
    for (int m = 0; m < MSUB; ++m)
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][t][r] = 0.f;
    const int per_frame = a.prow * a.pcol;
    const int c = cb * 32;
    constexpr int XPIN = F::XPIN, DPIN = F::DPIN;
    bool bad = false;
    // the global loads of a patch: the x halo (rows y0-1 .. y0+2, cols x0-1 .. x0+32, 4 groups
    // of channel block cb) and the dy patch (64 pixels x MT channels)
    constexpr int XIT = (kPY * kPX * 4 + C::NT - 1) / C::NT;
    constexpr int DIT = (kPR * kPC * (MT / 8) + C::NT - 1) / C::NT;
    uint4 xv[XIT][XPIN];
    uint4 dv[DIT][DPIN];
    auto load_patch = [&](long q) {
        const long b = q / per_frame;
        const int r = (int)(q - b * per_frame);
        const int y0 = (r / a.pcol) * kPR, x0 = (r % a.pcol) * kPC;
#pragma unroll
        for (int j = 0; j < XIT; ++j) {
            const int it = tid + j * C::NT;
            const int g = it & 3, pix = it >> 2;
            const int hy = pix / kPX, hx = pix - hy * kPX;
            const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
            const int cg = c + g * 8;
            for (int pp = 0; pp < XPIN; ++pp) xv[j][pp] = make_uint4(0, 0, 0, 0);
            if (it < kPY * kPX * 4 && cg < a.Ctot && (unsigned)iy < (unsigned)a.H &&
                (unsigned)ix < (unsigned)a.W) {
                const bool s1 = cg >= a.c0;
                const uint8_t* sp = s1 ? a.s[1].p : a.s[0].p;
                const int sH = s1 ? a.s[1].H : a.s[0].H, sW = s1 ? a.s[1].W : a.s[0].W;
                const int sG = s1 ? a.s[1].G : a.s[0].G, up = s1 ? a.s[1].up2 : a.s[0].up2;
                const int cl = cg - (s1 ? a.c0 : 0);
                const uint8_t* src = sp + (((b * sH + (iy >> up)) * sW + (ix >> up)) * sG +
                                           cl / 8) * C::XGB;
#pragma unroll
                for (int pp = 0; pp < XPIN; ++pp)
                    xv[j][pp] = *reinterpret_cast<const uint4*>(src + 16 * pp);
            }
        }
#pragma unroll
        for (int j = 0; j < DIT; ++j) {
            const int it = tid + j * C::NT;
            const int g = it % (MT / 8), pix = it / (MT / 8);
            const int py = pix / kPC, px = pix - py * kPC;
            const int oy = y0 + py, ox = x0 + px;
            const int co = mt * MT + g * 8;
            for (int pp = 0; pp < DPIN; ++pp) dv[j][pp] = make_uint4(0, 0, 0, 0);
            if (it < kPR * kPC * (MT / 8) && co < a.Cout && oy < a.H && ox < a.W) {
                const uint8_t* src = a.dy + (((b * a.H + oy) * a.W + ox) * a.Gout + co / 8) * C::DGB;
#pragma unroll
                for (int pp = 0; pp < DPIN; ++pp)
                    dv[j][pp] = *reinterpret_cast<const uint4*>(src + 16 * pp);
            }
        }
    };
    // PIPE: software pipeline — patch q+1's loads are issued before patch q's MFMAs, so they
    // land while the matrix pipe works (costs the registers of one patch in flight); else each
    // patch's loads are issued at the top of its iteration
    if (PIPE && q0 < q1) load_patch(q0);
    for (long q = q0; q < q1; ++q) {
        if (!PIPE) load_patch(q);
        // (WgF3) x: S3 -> the S2 split, in registers
        uint4 xs[XIT][NP];
#pragma unroll
        for (int j = 0; j < XIT; ++j) {
            if constexpr (XPIN == NP) {
#pragma unroll
                for (int pp = 0; pp < NP; ++pp) xs[j][pp] = xv[j][pp];
            } else {
                bad |= s3_resplit<false>(xv[j], nullptr, xs[j][0], xs[j][1]);
            }
        }
        __syncthreads();   // the previous patch's readers are done
#pragma unroll
        for (int j = 0; j < XIT; ++j) {
            const int it = tid + j * C::NT;
            if (it < kPY * kPX * 4) {
                const int g = it & 3, pix = it >> 2;
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    *reinterpret_cast<uint4*>(ximg + pp * C::XPART + pix * C::XROW + g * 16) =
                        xs[j][pp];
            }
        }
#pragma unroll
        for (int j = 0; j < DIT; ++j) {
            const int it = tid + j * C::NT;
            if (it < kPR * kPC * (MT / 8)) {
                const int g = it % (MT / 8), pix = it / (MT / 8);
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    *reinterpret_cast<uint4*>(dimg + pp * C::DPART + pix * C::DROW + g * 16) =
                        dv[j][pp];
            }
        }
        __syncthreads();
        if (PIPE && q + 1 < q1) load_patch(q + 1);
        // 4 K-steps of 16 pixels: K-step ks covers patch row ks/2, columns 16(ks%2) ..
#pragma unroll
        for (int ks = 0; ks < kPR * kPC / 16; ++ks) {
            V8 fa[MSUB][NP], fb[3][NP];
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) {
#pragma unroll
                for (int m = 0; m < MSUB; ++m) {
                    const int base = pp * C::DPART + (m * 32 + colb) * 2;
                    const int k0 = 16 * ks + 8 * hh + rq;
                    fa[m][pp] = frag<V8>(tr_read(dimg, base + k0 * C::DROW),
                                     tr_read(dimg, base + (k0 + 4) * C::DROW));
                }
                const int py = ks >> 1;
                const int px0 = 16 * (ks & 1) + 8 * hh + rq;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const int base = pp * C::XPART + colb * 2 +
                                     ((py + kh) * kPX + px0 + kw) * C::XROW;
                    fb[kw][pp] = frag<V8>(tr_read(ximg, base), tr_read(ximg, base + 4 * C::XROW));
                }
            }
#pragma unroll
            for (int t = 0; t < F::NTERM; ++t)
#pragma unroll
                for (int m = 0; m < MSUB; ++m)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw)
                        acc[m][kw] = F::mfma32(fa[m][F::ta(t)], fb[kw][F::tb(t)], acc[m][kw]);
        }
    }
    if constexpr (XPIN != NP) {
        // one store per wave that saw an out-of-range value (the flag only goes 0 -> 1)
        const unsigned long long msk = __ballot(bad);
        if (msk && a.oflow && lane == __builtin_ctzll(msk)) *a.oflow = 1;
    }
    // partial slab, wgrad33's layout: [split][tile][MT][288 = tap * 32 + c]
    float* out = a.part + ((long)blockIdx.y * a.ntiles + tile) * (MT * 288);
    const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int m = 0; m < MSUB; ++m)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int tap = kh * 3 + kw;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int row = m * 32 + 8 * (j >> 2) + 4 * h + (j & 3);
                out[row * 288 + tap * 32 + r32] = acc[m][kw][j];
            }
        }
}

// WgF3: per-channel max |dy| of an S3 tensor (P pixels x G 8-channel groups, G <= 256),
// as the bit patterns of the non-negative floats (which order as the values)
__global__ __launch_bounds__(kB) void dy_amax_kernel(const uint8_t* __restrict__ dy, long P,
                                                     int G, uint32_t* __restrict__ amax) {
    __shared__ uint32_t red[2048];
    const int tid = threadIdx.x;
    for (int i = tid; i < G * 8; i += kB) red[i] = 0u;
    __syncthreads();
    const int per = kB / G;   // threads per group (consecutive groups of one pixel: coalesced)
    const int g = tid % G, r = tid / G;
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (r < per) {
        for (long p = (long)blockIdx.x * per + r; p < P; p += (long)gridDim.x * per) {
            const s3::G8 v = s3::load_g8(dy + (p * G + g) * 48);
#pragma unroll
            for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], fabsf(v.v[e]));
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicMax(&red[g * 8 + e], __float_as_uint(m[e]));
    }
    __syncthreads();
    for (int i = tid; i < G * 8; i += kB)
        if (red[i]) atomicMax(&amax[i], red[i]);
}

// WgF3: dy (S3) -> its per-channel scaled S2 copy, one 8-channel group per thread
__global__ __launch_bounds__(kB) void dy_to_s2_kernel(const uint8_t* __restrict__ dy,
                                                      const float* __restrict__ scale, long n,
                                                      int G, uint8_t* __restrict__ out) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over P x G groups
    if (i >= n) return;
    const int g = (int)(i % G);
    s3::G8 v = s3::load_g8(dy + i * 48);
    const float4 s0 = *reinterpret_cast<const float4*>(scale + g * 8);
    const float4 s1 = *reinterpret_cast<const float4*>(scale + g * 8 + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v.v[e] *= sc[e];
    s2::store_g8(out + i * 32, v);
}

// scale[c] = 2^k with amax[c] 2^k in [2^14, 2^15) (1 for an all-zero or non-finite channel)
__global__ __launch_bounds__(kB) void dy_scale_kernel(const uint32_t* __restrict__ amax,
                                                      float* __restrict__ scale, int n) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const float a = __uint_as_float(amax[i]);
    int k = 0;
    if (a > 0.f && isfinite(a)) {
        int ex = 0;
        frexpf(a, &ex);   // a in [2^(ex-1), 2^ex)
        k = max(-126, min(126, 15 - ex));
    }
    scale[i] = ldexpf(1.f, k);
}

// The split reduction of the 3x3 weight gradient, in two passes over the partial slabs in their
// own (coalesced) order.  A pass-1 thread sums kRedChunk consecutive splits of one slab
// element; the final pass sums the chunk sums (or, with <= kRedChunk splits, the splits) in
// order, undoes the dy scale and writes the PyTorch (Cout, Ctot, 3, 3) element.  Before, one
// thread per output summed every split with strided loads: on the Cout <= 32 decoder layers
// (one tile, ~1500 splits) that was a few dozen blocks of 1500-long load chains.
constexpr int kRedChunk = 16;

template <int MSUB>
__global__ __launch_bounds__(kB) void wgrad33_chunk_kernel(W33Args a, int splits,
                                                           float* __restrict__ out) {
    const long slab = (long)a.ntiles * (32 * MSUB) * 288;
    const long j = (long)blockIdx.x * kB + threadIdx.x;
    if (j >= slab) return;
    const int k0 = blockIdx.y * kRedChunk, k1 = min(splits, k0 + kRedChunk);
    float s = 0.f;
    for (int k = k0; k < k1; ++k) s += a.part[(long)k * slab + j];
    out[(long)blockIdx.y * slab + j] = s;
}

template <int MSUB>
__global__ __launch_bounds__(kB) void wgrad33_reduce_kernel(W33Args a, const float* __restrict__ src,
                                                            int nsum, int cout_store,
                                                            float* __restrict__ dw, int r16) {
    constexpr int MT = 32 * MSUB;
    const long slab = (long)a.ntiles * MT * 288;
    const long j = (long)blockIdx.x * kB + threadIdx.x;   // slab order: tile, m, n
    if (j >= slab) return;
    const int tile = (int)(j / (MT * 288));
    const int rem = (int)(j - (long)tile * (MT * 288));
    const int m = rem / 288, n = rem - m * 288;
    const int co = (tile % a.ntm) * MT + m;
    const int c = (tile / a.ntm) * 32 + (n & 31), tap = n >> 5;
    if (co >= cout_store || c >= a.Ctot) return;
    float s = 0.f;
    for (int k = 0; k < nsum; ++k) s += src[(long)k * slab + j];
    if (a.dscale) s /= a.dscale[co];   // a power of two: exact
    dw[((long)co * a.Ctot + c) * 9 + tap] = r16 ? (float)(_Float16)s : s;
}

__global__ __launch_bounds__(kB) void wgrad_reduce_kernel(WgArgs a, int splits, int cout_store,
                                                          float* __restrict__ dw, int r16) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over cout_store * Ctot * KH * KW
    const long total = (long)cout_store * a.Ctot * a.KH * a.KW;
    if (i >= total) return;
    const int taps = a.KH * a.KW;
    const int tap = (int)(i % taps);
    const long t = i / taps;
    const int c = (int)(t % a.Ctot);
    const int co = (int)(t / a.Ctot);
    const int tile = ((tap * a.nct + c / kWT) * a.ntm) + co / kWT;
    const int m = co % kWT, n = c % kWT;
    float s = 0.f;
    for (int k = 0; k < splits; ++k)
        s += a.part[((long)k * a.ntiles + tile) * (kWT * kWT) + m * kWT + n];
    dw[i] = r16 ? (float)(_Float16)s : s;   // PyTorch layout (Cout, Ctot, KH, KW)
}

// ------------------------------------------------------- weight pack
// packed[kt][g][part][m][e] = part of Wsel[32 kt + 8 g + e][m], k = tap * Cin' + c'.
// mode 0: Wsel[k][m] = W[m][c'][kh][kw] (W = (Cout, Ctot, KH, KW), Cin' = Ctot)
// mode 1 (dgrad): outputs m over channels [c0, c0 + Cout') of W's inputs, inputs c' over
//   W's outputs: Wsel[k][m] = W[c'][c0 + m][KH-1-kh][KW-1-kw]   (Cin' = W's Cout)
__global__ __launch_bounds__(kB) void pack_kernel(const float* __restrict__ w,
                                                  uint16_t* __restrict__ out, int mode,
                                                  int CoutW, int CtotW, int KH, int KW, int c0,
                                                  int Coutp, int Cinp, int Kpad, int Mpad,
                                                  int h1) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over Kpad * Mpad
    if (i >= (long)Kpad * Mpad) return;
    const int m = (int)(i % Mpad);
    const int k = (int)(i / Mpad);
    const int K = KH * KW * Cinp;
    float v = 0.f;
    if (k < K && m < Coutp) {
        const int tap = k / Cinp, c = k - tap * Cinp;
        const int kh = tap / KW, kw = tap - kh * KW;
        if (mode == 0) {
            if (c < CtotW) v = w[(((long)m * CtotW + c) * KH + kh) * KW + kw];
        } else if (c < CoutW) {   // inputs c' >= CoutW: zero padding of a padded dy
            v = w[(((long)c * CtotW + c0 + m) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
        }
    }
    const int kt = k / 32, g = (k / 8) & 3, e = k & 7;
    if (h1) {   // FmtH1: (Kpad/32, 4, 1, Mpad, 8) fp16, the autocast cast of the weight
        out[(((long)kt * 4 + g) * Mpad + m) * 8 + e] = (uint16_t)s2::hbits(v);
        return;
    }
    const uint32_t hb = s3::bfbits(v);
    const float r1 = v - __uint_as_float(hb << 16);
    const uint32_t mb = s3::bfbits(r1);
    const uint32_t lb = s3::bfbits(r1 - __uint_as_float(mb << 16));
    const long base = ((((long)kt * 4 + g) * 3) * Mpad + m) * 8 + e;
    out[base] = (uint16_t)hb;
    out[base + (long)Mpad * 8] = (uint16_t)mb;
    out[base + 2l * Mpad * 8] = (uint16_t)lb;
}

// The split f16x3 operand of a trainable conv (conv_x6.hip FmtF16, as ops.pack_conv_weight_f16
// on the host): v = Wsel[k][m] / kdiv[c'] (kdiv: a power of two per input channel c' of the
// selected conv, or none) over a per-column power-of-two scale s_m with max_k |v| / s_m in
// [2^14, 2^15); parts h = rne_f16(v / s_m), l = rne_f16(v / s_m - h), layout
// (Kpad/32, 4, 2, Mpad, 8).  Mode 1 with kdiv = dy's channel scales is the data-gradient
// operand of the f16x3 step: the scales that put dy into fp16's range divide out exactly.
__device__ __forceinline__ float pack_sel(const float* __restrict__ w, int mode, int CoutW,
                                          int CtotW, int KH, int KW, int c0, int Coutp,
                                          int Cinp, const float* __restrict__ kdiv, int k,
                                          int m) {
    const int K = KH * KW * Cinp;
    if (k >= K || m >= Coutp) return 0.f;
    const int tap = k / Cinp, c = k - tap * Cinp;
    const int kh = tap / KW, kw = tap - kh * KW;
    float v = 0.f;
    if (mode == 0) {
        if (c < CtotW) v = w[(((long)m * CtotW + c) * KH + kh) * KW + kw];
    } else if (c < CoutW) {
        v = w[(((long)c * CtotW + c0 + m) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
    }
    if (kdiv && c < (mode == 0 ? CtotW : CoutW)) v = v / kdiv[c];   // a power of two: exact
    return v;
}

// one block per output column m: its power-of-two scale
__global__ __launch_bounds__(kB) void pack_f16_scale_kernel(const float* __restrict__ w, int mode,
                                                            int CoutW, int CtotW, int KH, int KW,
                                                            int c0, int Coutp, int Cinp, int Kpad,
                                                            const float* __restrict__ kdiv,
                                                            float* __restrict__ wscale) {
    const int m = blockIdx.x;
    float a = 0.f;
    for (int k = threadIdx.x; k < Kpad; k += kB)
        a = fmaxf(a, fabsf(pack_sel(w, mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp, kdiv, k, m)));
    for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
    __shared__ float red[kB / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int i = 0; i < kB / 64; ++i) t = fmaxf(t, red[i]);
        float sc = 1.f;
        if (t > 0.f && isfinite(t)) {
            int ex = 0;
            frexpf(t, &ex);              // t in [2^(ex-1), 2^ex)
            sc = ldexpf(1.f, ex - 1 - 14);
        }
        wscale[m] = sc;
    }
}

__global__ __launch_bounds__(kB) void pack_f16x3_kernel(const float* __restrict__ w, int mode,
                                                        int CoutW, int CtotW, int KH, int KW,
                                                        int c0, int Coutp, int Cinp, int Kpad,
                                                        int Mpad, const float* __restrict__ kdiv,
                                                        const float* __restrict__ wscale,
                                                        uint16_t* __restrict__ out) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;   // over Kpad * Mpad
    if (i >= (long)Kpad * Mpad) return;
    const int m = (int)(i % Mpad);
    const int k = (int)(i / Mpad);
    const float u = pack_sel(w, mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp, kdiv, k, m) /
                    wscale[m];
    uint32_t h, l;
    s2::split2(u, h, l);
    const int kt = k / 32, g = (k / 8) & 3, e = k & 7;
    const long base = ((((long)kt * 4 + g) * 2) * Mpad + m) * 8 + e;
    out[base] = (uint16_t)h;
    out[base + (long)Mpad * 8] = (uint16_t)l;
}

// ---- batched weight packs (tcam_pack_weights): a trainer's repack after every optimizer
// step is one (fp16) or two (f16x3: column scales, then parts) launches over a table of
// items instead of one or two launches per conv.  Each block finds its item by binary search
// over the items' first blocks; the per-item arithmetic is the kernels' above.
struct PackDesc {
    const float* w;
    uint16_t* out;
    float* wscale;
    const float* kdiv;
    int mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp, Kpad, Mpad;
    int sb0, pb0;   // the item's first block in the scale / pack launch
};

__device__ __forceinline__ int pack_item(const PackDesc* __restrict__ t, int n, int blk,
                                         bool scale) {
    int lo = 0, hi = n - 1;   // the last item whose first block is <= blk
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((scale ? t[mid].sb0 : t[mid].pb0) <= blk) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(kB) void pack_multi_scale_kernel(const PackDesc* __restrict__ t,
                                                              int n) {
    const PackDesc& d = t[pack_item(t, n, blockIdx.x, true)];
    const int m = blockIdx.x - d.sb0;
    float a = 0.f;
    for (int k = threadIdx.x; k < d.Kpad; k += kB)
        a = fmaxf(a, fabsf(pack_sel(d.w, d.mode, d.CoutW, d.CtotW, d.KH, d.KW, d.c0, d.Coutp,
                                    d.Cinp, d.kdiv, k, m)));
    for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
    __shared__ float red[kB / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        float v = 0.f;
        for (int i = 0; i < kB / 64; ++i) v = fmaxf(v, red[i]);
        float sc = 1.f;
        if (v > 0.f && isfinite(v)) {
            int ex = 0;
            frexpf(v, &ex);
            sc = ldexpf(1.f, ex - 1 - 14);
        }
        d.wscale[m] = sc;
    }
}

template <bool F16X3>
__global__ __launch_bounds__(kB) void pack_multi_kernel(const PackDesc* __restrict__ t, int n) {
    const PackDesc& d = t[pack_item(t, n, blockIdx.x, false)];
    const long i = (long)(blockIdx.x - d.pb0) * kB + threadIdx.x;   // over Kpad * Mpad
    if (i >= (long)d.Kpad * d.Mpad) return;
    const int m = (int)(i % d.Mpad);
    const int k = (int)(i / d.Mpad);
    const float v = pack_sel(d.w, d.mode, d.CoutW, d.CtotW, d.KH, d.KW, d.c0, d.Coutp, d.Cinp,
                             d.kdiv, k, m);
    const int kt = k / 32, g = (k / 8) & 3, e = k & 7;
    if (!F16X3) {   // FmtH1: (Kpad/32, 4, 1, Mpad, 8) fp16
        d.out[(((long)kt * 4 + g) * d.Mpad + m) * 8 + e] = (uint16_t)s2::hbits(v);
        return;
    }
    uint32_t h, l;
    s2::split2(v / d.wscale[m], h, l);
    const long base = ((((long)kt * 4 + g) * 2) * d.Mpad + m) * 8 + e;
    d.out[base] = (uint16_t)h;
    d.out[base + (long)d.Mpad * 8] = (uint16_t)l;
}

// ------------------------------------------------------------ chansum
__global__ __launch_bounds__(kB) void chansum_partial_kernel(const float* __restrict__ x,
                                                             int C, long HW, long chunk,
                                                             double* __restrict__ part,
                                                             int nchunks) {
    // grid (nchunks, B * C): sum over a chunk of one plane
    const long plane = blockIdx.y;
    const long h0 = (long)blockIdx.x * chunk, h1 = min(HW, h0 + chunk);
    double s = 0.0;
    for (long j = h0 + threadIdx.x; j < h1; j += kB) s += (double)x[plane * HW + j];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double red[kB / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < kB / 64; ++i) t += red[i];
        part[plane * nchunks + blockIdx.x] = t;
    }
}

__global__ void chansum_final_kernel(const double* __restrict__ part, int B, int C, int nchunks,
                                     float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s = 0.0;
    for (int b = 0; b < B; ++b)
        for (int k = 0; k < nchunks; ++k) s += part[((long)b * C + c) * nchunks + k];
    out[c] = (float)s;
}

// ------------------------------------------------------------- losses
// Per-(frame, block) partials over pixels: sum S0, sum S1, CE sum, valid count, sum S.AS.
constexpr int kLossPix = 4096;

__device__ __forceinline__ void softmax2(float f0, float f1, float& s0, float& s1) {
    const float m = fmaxf(f0, f1);
    const float e0 = expf(f0 - m), e1 = expf(f1 - m);
    const float z = e0 + e1;
    s0 = e0 / z;
    s1 = e1 / z;
}

__global__ __launch_bounds__(kB) void softmax2_kernel(const float* __restrict__ f,
                                                      float* __restrict__ S, int B, long HW) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= (long)B * HW) return;
    const long b = i / HW, j = i - b * HW;
    float s0, s1;
    softmax2(f[(b * 2) * HW + j], f[(b * 2 + 1) * HW + j], s0, s1);
    S[(b * 2) * HW + j] = s0;
    S[(b * 2 + 1) * HW + j] = s1;
}

__global__ __launch_bounds__(kB) void loss_partial_kernel(const float* __restrict__ f,
                                                          const float* __restrict__ S,
                                                          const int32_t* __restrict__ seeds,
                                                          const float* __restrict__ AS, long HW,
                                                          int nchunks, double* __restrict__ part) {
    const int b = blockIdx.y;
    const long j0 = (long)blockIdx.x * kLossPix, j1 = min(HW, j0 + kLossPix);
    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};   // S0, S1, CE, valid, S.AS
    for (long j = j0 + threadIdx.x; j < j1; j += kB) {
        const long o0 = (long)(b * 2) * HW + j, o1 = o0 + HW;
        const float s0 = S[o0], s1 = S[o1];
        acc[0] += s0;
        acc[1] += s1;
        if (seeds) {
            const int sd = seeds[(long)b * HW + j];
            if (sd == 0 || sd == 1) {
                // cross entropy = logsumexp(f) - f[seed]
                const float f0 = f[o0], f1 = f[o1];
                const float m = fmaxf(f0, f1);
                const float lse = m + logf(expf(f0 - m) + expf(f1 - m));
                acc[2] += (double)(lse - (sd ? f1 : f0));
                acc[3] += 1.0;
            }
        }
        if (AS) acc[4] += (double)s0 * AS[o0] + (double)s1 * AS[o1];
    }
    __shared__ double red[kB / 64][5];
#pragma unroll
    for (int q = 0; q < 5; ++q)
        for (int o = 32; o > 0; o >>= 1) acc[q] += __shfl_xor(acc[q], o, 64);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 5; ++q) red[threadIdx.x >> 6][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < 5) {
        double t = 0.0;
        for (int w = 0; w < kB / 64; ++w) t += red[w][threadIdx.x];
        part[((long)b * nchunks + blockIdx.x) * 5 + threadIdx.x] = t;
    }
}

struct LossCfg {
    float lam_sl, lam_crf, lam_size, elb_t;
    int use_sl, use_crf, use_size;
};

// One thread: the scalar losses and per-(b, c) size gradients.
//   sl   = lam_sl * CE mean over valid seeds
//   crf  = lam_crf * -(sum S.AS) / B
//   size = lam_size * 0.5 * sum_c ELB(-sum_hw S_c)  (ELB mean over b, elb.py:119-137)
// coef: [0] = lam_sl / n_valid; [2 + 2b + c] = d size / d S[b, c, :] (constant per plane).
// extra (optional): one more term's value already on the device (RgbJointConRanFieldTcams),
// added to the total and stored as losses[4].
// One block: thread i takes frames i, i + 256, ... (its chunks in order), then thread 0 adds
// the 256 thread partials in order — a fixed summation order, so the result is
// deterministic (a single thread over B * nchunks dependent fp64 adds took ~0.6 ms at B = 256).
constexpr int kFinBlock = 256;
__global__ __launch_bounds__(kFinBlock) void loss_finalize_kernel(
    const double* __restrict__ part, int B, int nchunks, LossCfg cfg,
    const float* __restrict__ extra, float* __restrict__ losses, float* __restrict__ coef) {
    __shared__ double red[4][kFinBlock];
    double ce = 0.0, nv = 0.0, sas = 0.0, size = 0.0;
    const double t = cfg.elb_t, ct = -1.0 / (t * t);
    for (int b = threadIdx.x; b < B; b += kFinBlock) {
        double bl[2] = {0.0, 0.0};
        for (int k = 0; k < nchunks; ++k) {
            const double* p = part + ((long)b * nchunks + k) * 5;
            bl[0] += p[0];
            bl[1] += p[1];
            ce += p[2];
            nv += p[3];
            sas += p[4];
        }
        for (int c = 0; c < 2; ++c) {
            // ELB.forward on fx = -bl, elementwise (fx <= ct: -log(-fx)/t, else t fx - log(1/t^2)/t + 1/t)
            const float fx = (float)(-bl[c]);
            float l, dl;
            if (fx <= (float)ct) {
                l = -(1.f / (float)t) * logf(-fx);
                dl = -(1.f / (float)t) / fx;
            } else {
                l = (float)t * fx - (1.f / (float)t) * logf(1.f / ((float)t * (float)t)) +
                    1.f / (float)t;
                dl = (float)t;
            }
            size += (double)l;
            // loss = lam * 0.5 * sum_c mean_b ELB(fx);  d fx / d S = -1
            coef[2 + 2 * b + c] = cfg.use_size ? -cfg.lam_size * 0.5f * dl / (float)B : 0.f;
        }
    }
    red[0][threadIdx.x] = ce;
    red[1][threadIdx.x] = nv;
    red[2][threadIdx.x] = sas;
    red[3][threadIdx.x] = size;
    __syncthreads();
    if (threadIdx.x != 0) return;
    ce = nv = sas = size = 0.0;
    for (int i = 0; i < kFinBlock; ++i) {
        ce += red[0][i];
        nv += red[1][i];
        sas += red[2][i];
        size += red[3][i];
    }
    const float sl = (cfg.use_sl && nv > 0) ? (float)(cfg.lam_sl * ce / nv) : 0.f;
    const float crf = cfg.use_crf ? (float)(cfg.lam_crf * -sas / B) : 0.f;
    const float sz = cfg.use_size ? (float)(cfg.lam_size * 0.5 * size / B) : 0.f;
    const float ex = extra ? extra[0] : 0.f;
    losses[0] = extra ? ((sl + crf) + sz) + ex : (sl + crf) + sz;
    losses[1] = sl;
    losses[2] = crf;
    losses[3] = sz;
    if (extra) losses[4] = ex;
    coef[0] = (cfg.use_sl && nv > 0) ? (float)(cfg.lam_sl / nv) : 0.f;
    coef[1] = cfg.use_crf ? -2.f * cfg.lam_crf / (float)B : 0.f;
}

// d loss / d fcams per pixel:
//   gS_c = coef1 * AS_c + size[b, c] + gx_c    (CRF: -2 lam AS / B; size: constant;
//                                               gx: an extra term's d loss / d S, or NULL)
//   gf_c = S_c (gS_c - sum_j S_j gS_j)          (softmax backward)
//        + coef0 (S_c - [seed == c])            (CE, valid seeds only)
__global__ __launch_bounds__(kB) void loss_grad_kernel(const float* __restrict__ S,
                                                       const int32_t* __restrict__ seeds,
                                                       const float* __restrict__ AS,
                                                       const float* __restrict__ gx,
                                                       const float* __restrict__ coef, int B,
                                                       long HW, float* __restrict__ gf) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= (long)B * HW) return;
    const long b = i / HW, j = i - b * HW;
    const long o0 = (b * 2) * HW + j, o1 = o0 + HW;
    const float s0 = S[o0], s1 = S[o1];
    float g0 = coef[2 + 2 * b], g1 = coef[2 + 2 * b + 1];
    if (AS) {
        g0 += coef[1] * AS[o0];
        g1 += coef[1] * AS[o1];
    }
    if (gx) {
        g0 += gx[o0];
        g1 += gx[o1];
    }
    const float dot = s0 * g0 + s1 * g1;
    float r0 = s0 * (g0 - dot), r1 = s1 * (g1 - dot);
    if (seeds) {
        const int sd = seeds[b * HW + j];
        if (sd == 0 || sd == 1) {
            r0 += coef[0] * (s0 - (sd == 0 ? 1.f : 0.f));
            r1 += coef[0] * (s1 - (sd == 1 ? 1.f : 0.f));
        }
    }
    gf[o0] = r0;
    gf[o1] = r1;
}

// ------------------------------------------------- RgbJoint frame mosaics
// RgbJointConRanFieldTcams.pair_samples (losses/tcam.py:207-232): the frames of one group,
// in frame order, concatenated along the width.  idx (G, L): frame of group g at
// position p.  out (G, C, H, L*W) from src (B, C, H, W); 4 consecutive x per thread
// when W % 4 == 0 (16-B loads and stores), else one.
template <int V>
__global__ __launch_bounds__(kB) void mosaic_gather_kernel(const float* __restrict__ src,
                                                           const int32_t* __restrict__ idx,
                                                           int G, int L, int C, int H, int W,
                                                           float* __restrict__ out) {
    const int Wv = W / V;
    const long n = (long)G * L * C * H * Wv;
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const int xv = (int)(i % Wv);
    long r = i / Wv;
    const int y = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    r /= C;
    const int p = (int)(r % L);
    const int g = (int)(r / L);
    const int b = idx[g * L + p];
    const float* s = src + (((long)b * C + c) * H + y) * W + (long)xv * V;
    float* d = out + (((long)g * C + c) * H + y) * ((long)L * W) + (long)p * W + (long)xv * V;
    if constexpr (V == 4)
        *reinterpret_cast<float4*>(d) = *reinterpret_cast<const float4*>(s);
    else
        *d = *s;
}

// The adjoint: dst[b, c, y, x] (+)= coef * sum over the occurrences k of frame b (in
// occ[occ_start[b] .. occ_start[b+1]), each g * L + p, fixed order) of
// mosaic[g, c, y, p*W + x].  A frame repeated by _fill_minibatch sums its copies.
__global__ __launch_bounds__(kB) void mosaic_scatter_kernel(const float* __restrict__ mosaic,
                                                            const int32_t* __restrict__ occ_start,
                                                            const int32_t* __restrict__ occ,
                                                            int B, int L, int C, int H, int W,
                                                            float coef, int accumulate,
                                                            float* __restrict__ dst) {
    const long n = (long)B * C * H * W;
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % W);
    long r = i / W;
    const int y = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    const int b = (int)(r / C);
    const int k0 = occ_start[b], k1 = occ_start[b + 1];
    if (k0 == k1 && accumulate) return;
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) {
        const int gp = occ[k], g = gp / L, p = gp - g * L;
        acc += mosaic[(((long)g * C + c) * H + y) * ((long)L * W) + (long)p * W + x];
    }
    dst[i] = accumulate ? dst[i] + coef * acc : coef * acc;
}

// ------------------------------------------------------------------ SGD
__global__ __launch_bounds__(kB) void sgd_kernel(float* __restrict__ p,
                                                 const float* __restrict__ g,
                                                 float* __restrict__ buf, long n, float lr,
                                                 float momentum, float dampening, float wd,
                                                 int nesterov, int first, float gscale) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    float d = gscale == 1.f ? g[i] : g[i] * gscale;
    if (wd != 0.f) d = d + wd * p[i];
    if (momentum != 0.f) {
        float b;
        if (first)
            b = d;
        else
            b = momentum * buf[i] + (1.f - dampening) * d;
        buf[i] = b;
        d = nesterov ? d + momentum * b : b;
    }
    p[i] = p[i] - lr * d;
}

// The same step, skipped on the device when *gate (the all-reduced loss) is not finite
// (learning/train_wsol.py:1181: ``if loss.requires_grad and torch.isfinite(loss)``): no
// host sync, and every rank reads the same all-reduced value.  *steps counts the applied
// steps; the first applied one initialises the momentum buffer (torch SGD's
// ``momentum_buffer is None``).
__global__ __launch_bounds__(kB) void sgd_gated_kernel(float* __restrict__ p,
                                                       const float* __restrict__ g,
                                                       float* __restrict__ buf, long n, float lr,
                                                       float momentum, float dampening, float wd,
                                                       int nesterov, float gscale,
                                                       const float* __restrict__ gate,
                                                       const int* __restrict__ steps) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= n || !isfinite(*gate)) return;
    float d = gscale == 1.f ? g[i] : g[i] * gscale;
    if (wd != 0.f) d = d + wd * p[i];
    if (momentum != 0.f) {
        float b;
        if (*steps == 0)
            b = d;
        else
            b = momentum * buf[i] + (1.f - dampening) * d;
        buf[i] = b;
        d = nesterov ? d + momentum * b : b;
    }
    p[i] = p[i] - lr * d;
}

__global__ void sgd_count_kernel(const float* __restrict__ gate, int* __restrict__ steps,
                                 int* __restrict__ skipped) {
    if (threadIdx.x == 0) {
        if (isfinite(*gate))
            steps[0] += 1;
        else if (skipped)
            skipped[0] += 1;
    }
}

// ------------------------------------------------------------------ AMP
// torch.cuda.amp.GradScaler on the device (learning/train_wsol.py:1077, 1180-1183:
// scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()).
// unscale_: g *= 1 / scale (a power of two: exact), found_inf = any non-finite g.
__global__ __launch_bounds__(kB) void amp_unscale_kernel(float* __restrict__ g, long n,
                                                         const float* __restrict__ scale,
                                                         float* __restrict__ found_inf) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    const float inv = 1.0f / *scale;
    bool bad = false;
    if (i < n) {
        const float v = g[i];
        bad = !isfinite(v);
        g[i] = v * inv;
    }
    // one store per wave that saw a non-finite value (the flag only ever goes 0 -> 1)
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) *found_inf = 1.f;
}

// scaler.step + the reference's loss gate: the SGD step runs only when the all-reduced loss
// is finite AND no rank found a non-finite gradient (found_inf summed over ranks == 0)
__global__ __launch_bounds__(kB) void sgd_amp_kernel(float* __restrict__ p,
                                                     const float* __restrict__ g,
                                                     float* __restrict__ buf, long n, float lr,
                                                     float momentum, float dampening, float wd,
                                                     int nesterov, float gscale,
                                                     const float* __restrict__ gate,
                                                     const int* __restrict__ steps) {
    const long i = (long)blockIdx.x * kB + threadIdx.x;
    if (i >= n || !isfinite(gate[0]) || gate[1] != 0.f) return;
    float d = gscale == 1.f ? g[i] : g[i] * gscale;
    if (wd != 0.f) d = d + wd * p[i];
    if (momentum != 0.f) {
        float b;
        if (*steps == 0)
            b = d;
        else
            b = momentum * buf[i] + (1.f - dampening) * d;
        buf[i] = b;
        d = nesterov ? d + momentum * b : b;
    }
    p[i] = p[i] - lr * d;
}

// step counters + scaler.update(): a non-finite loss skips backward, step and update alike
// (train_wsol.py:1180); otherwise found_inf backs the scale off and resets the growth
// tracker, and growth_interval clean steps in a row grow it (torch GradScaler semantics)
__global__ void amp_update_kernel(const float* __restrict__ gate, int* __restrict__ steps,
                                  int* __restrict__ skipped, float* __restrict__ scale,
                                  int* __restrict__ tracker, float growth, float backoff,
                                  int interval) {
    if (threadIdx.x != 0) return;
    if (!isfinite(gate[0])) {
        if (skipped) skipped[0] += 1;
        return;
    }
    if (gate[1] != 0.f) {
        if (skipped) skipped[0] += 1;
        *scale = *scale * backoff;
        *tracker = 0;
        return;
    }
    steps[0] += 1;
    if (++*tracker >= interval) {
        *scale = *scale * growth;
        *tracker = 0;
    }
}

}  // namespace

// ================================================================== C ABI
extern "C" size_t tcam_bn_ws_bytes(long P, int C) {
    // the finest of the chunkings: kBwdChunkPix (bn_bwd_partial_co_kernel) and bn_plan's
    const long nchunks = std::max<long>((P + kBwdChunkPix - 1) / kBwdChunkPix,
                                        P > 0 && C > 0 ? bn_plan(P, C / 8).nchunks : 0);
    return (size_t)(nchunks * C * 2 * sizeof(double) + 2 * C * sizeof(float) + 256);
}

template <class L>
static int bn_stats(const void* y, long P, int C, float eps, float momentum,
                                float* mean, float* invstd, float* run_mean, float* run_var,
                                void* ws, void* stream) {
    TCAM_REQUIRE(y && P > 0 && C > 0 && C % 8 == 0 && mean && invstd && ws);
    hipStream_t st = as_stream(stream);
    const BnPlan pl = bn_plan(P, C / 8);
    const int nchunks = pl.nchunks;
    double* part = (double*)ws;
    bn_stats_co_kernel<L><<<dim3(nchunks, C / 8 / pl.GS), kB, 0, st>>>(
        (const uint8_t*)y, P, C / 8, pl.GS, pl.cp, part);
    TCAM_CHECK_LAUNCH();
    bn_finalize_kernel<<<C, kB, 0, st>>>(part, nchunks, C, P, eps, momentum, mean, invstd,
                                         run_mean, run_var);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int bn_relu(const void* y, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, void* out, long P, int C,
                               void* stream) {
    TCAM_REQUIRE(y && out && mean && invstd && gamma && beta && P > 0 && C % 8 == 0);
    const long total = P * (C / 8);
    bn_relu_kernel<L><<<cdiv(total, kB), kB, 0, as_stream(stream)>>>(
        (const uint8_t*)y, mean, invstd, gamma, beta, (uint8_t*)out, total, C / 8);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L, class LA = L>
static int bn_relu_bwd(const void* dout, const void* out, const void* y,
                                   const float* mean, const float* invstd, const float* gamma,
                                   void* dy, float* dgamma, float* dbeta, long P, int C, void* ws,
                                   void* stream, uint32_t* amax = nullptr) {
    TCAM_REQUIRE(dout && out && y && mean && invstd && gamma && dy && dgamma && dbeta && ws);
    TCAM_REQUIRE(P > 0 && C > 0 && C % 8 == 0);
    hipStream_t st = as_stream(stream);
    const bool co = kB % (C / 8) == 0;
    const int chunk = co ? kBwdChunkPix : kChunkPix;
    const int nchunks = (int)((P + chunk - 1) / chunk);
    double* part = (double*)ws;
    float* coef = (float*)((char*)ws + (size_t)nchunks * C * 2 * sizeof(double));
    if (co)
        bn_bwd_partial_co_kernel<L, LA><<<nchunks, kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, P,
            C / 8, part);
    else
        bn_bwd_partial_kernel<L, LA><<<dim3(nchunks, C / 8), kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, P,
            C / 8, part);
    TCAM_CHECK_LAUNCH();
    bn_bwd_finalize_kernel<<<C, kB, 0, st>>>(part, nchunks, C, dgamma, dbeta, coef);
    TCAM_CHECK_LAUNCH();
    const long total = P * (C / 8);
    if (amax) {
        TCAM_REQUIRE(kB % (C / 8) == 0 && C <= 2048);
        TCAM_REQUIRE(hipMemsetAsync(amax, 0, (size_t)C * sizeof(uint32_t), st) == hipSuccess);
        const long nb = std::min<long>(1024, cdiv(total, kB));
        bn_bwd_apply_amax_kernel<L, LA><<<(int)nb, kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, gamma,
            coef, 1.0f / (float)P, (uint8_t*)dy, total, C / 8, amax);
    } else {
        bn_bwd_apply_kernel<L, LA><<<cdiv(total, kB), kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, gamma,
            coef, 1.0f / (float)P, (uint8_t*)dy, total, C / 8);
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int up2_bwd(const void* gup, void* gx, int B, int C, int H, int W,
                               void* stream) {
    TCAM_REQUIRE(gup && gx && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    const long total = (long)B * H * W * (C / 8);
    up2_bwd_kernel<L><<<cdiv(total, kB), kB, 0, as_stream(stream)>>>(
        (const uint8_t*)gup, (uint8_t*)gx, C / 8, H, W, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int up2_resize_bwd(const void* g, void* gx, int B, int C, int H, int W,
                                      int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(g && gx && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0);
    const float sh = Ho > 1 ? (float)(2 * H - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(2 * W - 1) / (float)(Wo - 1) : 0.f;
    const long total = (long)B * H * W * (C / 8);
    up2_resize_bwd_kernel<L><<<cdiv(total, kB), kB, 0, as_stream(stream)>>>(
        (const uint8_t*)g, (uint8_t*)gx, C / 8, H, W, Ho, Wo, sh, sw, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

#define TCAM_TRAIN_LAYOUT_ENTRIES(SUF, L)                                                     \
    extern "C" int tcam_bn_stats_##SUF(const void* y, long P, int C, float eps, float momentum,  \
                                       float* mean, float* invstd, float* run_mean,             \
                                       float* run_var, void* ws, void* stream) {               \
        return bn_stats<L>(y, P, C, eps, momentum, mean, invstd, run_mean, run_var, ws,         \
                           stream);                                                             \
    }                                                                                           \
    extern "C" int tcam_bn_relu_##SUF(const void* y, const float* mean, const float* invstd,     \
                                      const float* gamma, const float* beta, void* out, long P,  \
                                      int C, void* stream) {                                    \
        return bn_relu<L>(y, mean, invstd, gamma, beta, out, P, C, stream);                     \
    }                                                                                           \
    extern "C" int tcam_bn_relu_bwd_##SUF(const void* dout, const void* out, const void* y,      \
                                          const float* mean, const float* invstd,               \
                                          const float* gamma, void* dy, float* dgamma,          \
                                          float* dbeta, long P, int C, void* ws, void* stream) { \
        return bn_relu_bwd<L>(dout, out, y, mean, invstd, gamma, dy, dgamma, dbeta, P, C, ws,   \
                              stream);                                                          \
    }                                                                                           \
    extern "C" int tcam_up2_bwd_##SUF(const void* gup, void* gx, int B, int C, int H, int W,     \
                                      void* stream) {                                           \
        return up2_bwd<L>(gup, gx, B, C, H, W, stream);                                         \
    }                                                                                           \
    extern "C" int tcam_up2_resize_bwd_##SUF(const void* g, void* gx, int B, int C, int H,      \
                                             int W, int Ho, int Wo, void* stream) {             \
        return up2_resize_bwd<L>(g, gx, B, C, H, W, Ho, Wo, stream);                            \
    }

TCAM_TRAIN_LAYOUT_ENTRIES(s3, LayS3)
TCAM_TRAIN_LAYOUT_ENTRIES(s1, LayS1)

// The f16x3 training step: BN statistics / affine on S2 activations, and the backward of
// bn_relu with S3 gradients (dout, dy) over S2 activations (out, y), optionally with the
// per-channel max |dy| (amax: C uint32 bit patterns, zeroed here) for the dy scales.
extern "C" int tcam_bn_stats_s2(const void* y, long P, int C, float eps, float momentum,
                                float* mean, float* invstd, float* run_mean, float* run_var,
                                void* ws, void* stream) {
    return bn_stats<LayS2>(y, P, C, eps, momentum, mean, invstd, run_mean, run_var, ws, stream);
}
extern "C" int tcam_bn_relu_s2(const void* y, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, void* out, long P, int C,
                               void* stream) {
    return bn_relu<LayS2>(y, mean, invstd, gamma, beta, out, P, C, stream);
}
extern "C" int tcam_bn_relu_bwd_s3s2(const void* dout, const void* out, const void* y,
                                     const float* mean, const float* invstd, const float* gamma,
                                     void* dy, float* dgamma, float* dbeta, long P, int C,
                                     void* ws, uint32_t* amax, void* stream) {
    return bn_relu_bwd<LayS3, LayS2>(dout, out, y, mean, invstd, gamma, dy, dgamma, dbeta, P, C,
                                     ws, stream, amax);
}

// dy (S3, P pixels x C channels) -> scale[c] (the power of two with amax[c] scale in
// [2^14, 2^15), 1 for an all-zero channel) and dy2, its scaled S2 copy.  amax from
// tcam_bn_relu_bwd_s3s2, or computed here when `compute` is set (amax zeroed first).
extern "C" int tcam_dy_scaled_s2(const void* dy, long P, int C, uint32_t* amax, int compute,
                                 float* scale, void* dy2, void* stream) {
    TCAM_REQUIRE(dy && amax && scale && dy2 && P > 0 && C > 0 && C % 8 == 0 && C <= 2048);
    hipStream_t st = as_stream(stream);
    const int G = C / 8;
    if (compute) {
        TCAM_REQUIRE(kB % G == 0);
        TCAM_REQUIRE(hipMemsetAsync(amax, 0, (size_t)C * sizeof(uint32_t), st) == hipSuccess);
        const int per = kB / G;
        const long nb = std::min<long>(1024, (P + per - 1) / per);
        dy_amax_kernel<<<(int)nb, kB, 0, st>>>((const uint8_t*)dy, P, G, amax);
        TCAM_CHECK_LAUNCH();
    }
    dy_scale_kernel<<<cdiv(C, kB), kB, 0, st>>>(amax, scale, C);
    TCAM_CHECK_LAUNCH();
    dy_to_s2_kernel<<<cdiv(P * G, kB), kB, 0, st>>>((const uint8_t*)dy, scale, P * G, G,
                                                     (uint8_t*)dy2);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

// The fused f16x3 BN-ReLU backward (the kernels above): dout S3, y (and out unless the
// mask is recomputed: out == NULL) S2 -> dy2 (the scaled S2 copy) + scale (+ dy3 S3 if
// given), dgamma, dbeta.  C / 8 must divide 256.  ws: tcam_bn_bwd_scaled_ws_bytes(P, C) =
// tcam_bn_ws_bytes(P, C) + the per-chunk maxima of |g| and |xh| (the scale's bound: reduced
// in the finalize, so no zeroed buffer and no atomics).
extern "C" size_t tcam_bn_bwd_scaled_ws_bytes(long P, int C) {
    const long nch = P > 0 && C > 0 ? bn_plan(P, C / 8).nchunks : 0;
    return tcam_bn_ws_bytes(P, C) + (size_t)nch * C * 2 * sizeof(float) + 256;
}

template <class LG, class LA>
static int bn_relu_bwd_fused(const void* dout, const void* out, const void* y, const float* mean,
                             const float* invstd, const float* gamma, const float* beta,
                             void* dy3, void* dy2, float* scale, float* dgamma, float* dbeta,
                             long P, int C, void* ws, void* stream) {
    TCAM_REQUIRE(dout && y && mean && invstd && gamma && beta && dgamma && dbeta && ws &&
                 P > 0 && C > 0 && C % 8 == 0 && kB % (C / 8) == 0);
    TCAM_REQUIRE((dy2 != nullptr) == (scale != nullptr) && (dy2 || dy3));
    hipStream_t st = as_stream(stream);
    const int G = C / 8;
    const BnPlan pl = bn_plan(P, G);
    const int nchunks = pl.nchunks;
    double* part = (double*)ws;
    float* coef = (float*)((char*)ws + (size_t)nchunks * C * 2 * sizeof(double));
    float* pmax = scale ? (float*)((char*)ws + tcam_bn_ws_bytes(P, C)) : nullptr;
    const dim3 pgrid(nchunks, G / pl.GS);
    if (out)
        bn_bwd_partial_sc2_kernel<LG, LA, false><<<pgrid, kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, gamma,
            beta, P, G, pl.GS, pl.cp, part, pmax);
    else
        bn_bwd_partial_sc2_kernel<LG, LA, true><<<pgrid, kB, 0, st>>>(
            (const uint8_t*)dout, nullptr, (const uint8_t*)y, mean, invstd, gamma, beta, P, G,
            pl.GS, pl.cp, part, pmax);
    TCAM_CHECK_LAUNCH();
    bn_bwd_finalize_sc_kernel<<<C, kB, 0, st>>>(part, nchunks, C, P, gamma, invstd, pmax, dgamma,
                                                dbeta, coef, scale);
    TCAM_CHECK_LAUNCH();
    const long total = P * G;
    // a few elements per thread over a grid whose stride is a multiple of G (kB % G == 0)
    const int nb = (int)std::min<long>(cdiv(total, 4L * kB), 8192);
    if (out)
        bn_bwd_apply_sc2_kernel<LG, LA, false><<<nb, kB, 0, st>>>(
            (const uint8_t*)dout, (const uint8_t*)out, (const uint8_t*)y, mean, invstd, gamma,
            beta, coef, scale, 1.0f / (float)P, (uint8_t*)dy3, (uint8_t*)dy2, total, G);
    else
        bn_bwd_apply_sc2_kernel<LG, LA, true><<<nb, kB, 0, st>>>(
            (const uint8_t*)dout, nullptr, (const uint8_t*)y, mean, invstd, gamma, beta, coef,
            scale, 1.0f / (float)P, (uint8_t*)dy3, (uint8_t*)dy2, total, G);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_bn_relu_bwd_scaled_s3s2(const void* dout, const void* out, const void* y,
                                            const float* mean, const float* invstd,
                                            const float* gamma, const float* beta, void* dy3,
                                            void* dy2, float* scale, float* dgamma,
                                            float* dbeta, long P, int C, void* ws,
                                            void* stream) {
    TCAM_REQUIRE(dy2 && scale);
    return bn_relu_bwd_fused<LayS3, LayS2>(dout, out, y, mean, invstd, gamma, beta, dy3, dy2,
                                           scale, dgamma, dbeta, P, C, ws, stream);
}

// The AMP step's BN-ReLU backward in the same two passes: S1 everywhere, dy written as S1
// (fp16, autocast's gradient), the mask recomputed from y when out == NULL.
extern "C" int tcam_bn_relu_bwd_fused_s1(const void* dout, const void* out, const void* y,
                                         const float* mean, const float* invstd,
                                         const float* gamma, const float* beta, void* dy,
                                         float* dgamma, float* dbeta, long P, int C, void* ws,
                                         void* stream) {
    TCAM_REQUIRE(dy);
    return bn_relu_bwd_fused<LayS1, LayS1>(dout, out, y, mean, invstd, gamma, beta, dy, nullptr,
                                           nullptr, dgamma, dbeta, P, C, ws, stream);
}

namespace {
bool make_wg(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout, int Hout,
             int Wout, int KH, int KW, int pad_h, int pad_w, WgArgs* a, int* splits) {
    if (!srcs || nsrc < 1 || nsrc > 2 || B <= 0 || !dy || Cout <= 0 || Cout % 8) return false;
    if (KH < 1 || KW < 1 || KH > 7 || KW > 7 || pad_h < 0 || pad_w < 0) return false;
    int ctot = 0;
    for (int i = 0; i < nsrc; ++i) {
        const tcam_conv_src& s = srcs[i];
        if (!s.ptr || s.C <= 0 || s.C % 8 || s.stride < 1) return false;
        a->s[i] = WSrc{(const uint8_t*)s.ptr, s.C, s.H, s.W, s.stride, s.up2 ? 1 : 0, s.C / 8};
        ctot += s.C;
    }
    if (nsrc == 1) a->s[1] = a->s[0];
    a->c0 = nsrc == 2 ? srcs[0].C : ctot;
    a->Ctot = ctot;
    a->dy = (const uint8_t*)dy;
    a->Cout = Cout;
    a->Gout = Cout / 8;
    a->Hout = Hout;
    a->Wout = Wout;
    a->KH = KH;
    a->KW = KW;
    a->pad_h = pad_h;
    a->pad_w = pad_w;
    a->P = (long)B * Hout * Wout;
    a->ntm = (Cout + kWT - 1) / kWT;
    a->nct = (ctot + kWT - 1) / kWT;
    a->ntiles = a->ntm * a->nct * KH * KW;
    // pixel splits: ~2048 blocks in flight, >= 64 K-steps per split
    long s = (2048 + a->ntiles - 1) / a->ntiles;
    const long maxs = (a->P + 64 * kWK - 1) / (64 * kWK);
    s = std::max(1l, std::min(s, maxs));
    a->chunk = ((a->P + s - 1) / s + kWK - 1) / kWK * kWK;
    *splits = (int)((a->P + a->chunk - 1) / a->chunk);
    return true;
}
}  // namespace

namespace {
// The 3x3 / stride-1 / pad-1 fast path (every source at the output size, up2 allowed).
bool make_w33(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout, int Hout,
              int Wout, int KH, int KW, int pad_h, int pad_w, W33Args* a, int* splits,
              int* msub) {
    if (KH != 3 || KW != 3 || pad_h != 1 || pad_w != 1) return false;
    if (!srcs || nsrc < 1 || nsrc > 2 || B <= 0 || !dy || Cout <= 0 || Cout % 8) return false;
    int ctot = 0;
    for (int i = 0; i < nsrc; ++i) {
        const tcam_conv_src& s = srcs[i];
        if (!s.ptr || s.C <= 0 || s.C % 8 || s.stride != 1) return false;
        const int h = s.up2 ? 2 * s.H : s.H, w = s.up2 ? 2 * s.W : s.W;
        if (h != Hout || w != Wout) return false;
        a->s[i] = WSrc{(const uint8_t*)s.ptr, s.C, s.H, s.W, 1, s.up2 ? 1 : 0, s.C / 8};
        ctot += s.C;
    }
    if (nsrc == 2 && srcs[0].C % 32) return false;   // a 32-channel block within one source
    if (nsrc == 1) a->s[1] = a->s[0];
    a->c0 = nsrc == 2 ? srcs[0].C : ctot;
    a->Ctot = ctot;
    a->dy = (const uint8_t*)dy;
    a->Cout = Cout;
    a->Gout = Cout / 8;
    a->H = Hout;
    a->W = Wout;
    a->prow = (Hout + kPR - 1) / kPR;
    a->pcol = (Wout + kPC - 1) / kPC;
    a->npatch = (long)B * a->prow * a->pcol;
    *msub = Cout <= 32 ? 1 : 2;
    const int MT = 32 * *msub;
    a->ntm = (Cout + MT - 1) / MT;
    a->ncb = (ctot + 31) / 32;
    a->ntiles = a->ntm * a->ncb;
    // ~1536 blocks; partial slabs bounded to ~256 MB
    long s = (1536 + a->ntiles - 1) / a->ntiles;
    const long slab = (long)a->ntiles * MT * 288 * 4;
    s = std::max(1l, std::min(s, std::min(a->npatch, (256l << 20) / slab)));
    a->ppb = (a->npatch + s - 1) / s;
    *splits = (int)((a->npatch + a->ppb - 1) / a->ppb);
    return true;
}
}  // namespace

// 3x3 wgrad arithmetic: 0 = bf16-split MFMA (x6, default), 1 = fp32 MFMA (A/B, tests)
static int g_wgrad_fp32 = 0;
extern "C" int tcam_wgrad_force_fp32(int on) {
    g_wgrad_fp32 = on ? 1 : 0;
    return TCAM_OK;
}

// workspace of the 3x3 path: the partial slabs, then (WgF3) the dy channel maxima and scales
static size_t w33_slab_bytes(const W33Args& a, int splits, int msub) {
    return ((size_t)splits * a.ntiles * (32 * msub) * 288 * sizeof(float) + 255) / 256 * 256;
}
// (+ the scaled S2 copy of dy: 4 B per element, WgF3)
static size_t w33_chunk_offset(const W33Args& a, int splits, int msub) {
    return (w33_slab_bytes(a, splits, msub) + (size_t)a.Cout * 2 * sizeof(float) +
            (size_t)a.npatch / ((size_t)a.prow * a.pcol) * a.H * a.W * a.Cout * 4 + 255) /
           256 * 256;
}
static int w33_nchunk(int splits) {
    return splits > kRedChunk ? (splits + kRedChunk - 1) / kRedChunk : 0;
}
// (+ the chunk sums of the two-pass split reduction)
static size_t w33_ws_bytes(const W33Args& a, int splits, int msub) {
    return w33_chunk_offset(a, splits, msub) +
           (size_t)w33_nchunk(splits) * a.ntiles * (32 * msub) * 288 * sizeof(float);
}

template <int MSUB>
static void reduce33(const W33Args& a, int splits, int cout_store, float* dw, int r16, void* ws,
                     hipStream_t st) {
    const long slab = (long)a.ntiles * (32 * MSUB) * 288;
    const int nch = w33_nchunk(splits);
    const float* src = a.part;
    int nsum = splits;
    if (nch) {
        float* cs = reinterpret_cast<float*>((char*)ws + w33_chunk_offset(a, splits, MSUB));
        wgrad33_chunk_kernel<MSUB><<<dim3(cdiv(slab, kB), nch), kB, 0, st>>>(a, splits, cs);
        src = cs;
        nsum = nch;
    }
    wgrad33_reduce_kernel<MSUB><<<cdiv(slab, kB), kB, 0, st>>>(a, src, nsum, cout_store, dw, r16);
}

extern "C" size_t tcam_conv_wgrad_ws_bytes(const tcam_conv_src* srcs, int nsrc, int B,
                                           int Cout, int Hout, int Wout, int KH, int KW) {
    int dummy = 0;
    {
        W33Args a{};
        int splits = 0, msub = 0;
        if (make_w33(srcs, nsrc, B, &dummy, Cout, Hout, Wout, KH, KW, 1, 1, &a, &splits, &msub))
            return w33_ws_bytes(a, splits, msub);
    }
    WgArgs a{};
    int splits = 0;
    if (!make_wg(srcs, nsrc, B, &dummy, Cout, Hout, Wout, KH, KW, 0, 0, &a, &splits)) return 0;
    return (size_t)splits * a.ntiles * kWT * kWT * sizeof(float);
}

template <class L, class F>
static int conv_wgrad(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout,
                      int Hout, int Wout, int KH, int KW, int pad_h, int pad_w, int cout_store,
                      float* dw, void* ws, size_t ws_bytes, int r16, void* stream,
                      int* oflow = nullptr, const float* dscale_in = nullptr) {
    TCAM_REQUIRE(dw && ws && cout_store > 0 && cout_store <= Cout);
    constexpr bool PRESCALED = std::is_same<F, WgF2>::value;   // dy: a scaled S2 copy
    {
        W33Args a{};
        int splits = 0, msub = 0;
        if (make_w33(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w, &a, &splits,
                     &msub) && ws_bytes >= w33_ws_bytes(a, splits, msub)) {
            a.part = (float*)ws;
            hipStream_t st = as_stream(stream);
            if constexpr (F::DPIN != F::XPIN) {
                // WgF3: the per-channel power-of-two scales of dy (max |dy| s in [2^14, 2^15))
                TCAM_REQUIRE(Cout <= 2048);
                uint32_t* amax = reinterpret_cast<uint32_t*>((char*)ws + w33_slab_bytes(a, splits,
                                                                                         msub));
                float* scale = reinterpret_cast<float*>(amax + Cout);
                TCAM_REQUIRE(hipMemsetAsync(amax, 0, (size_t)Cout * sizeof(uint32_t), st) ==
                             hipSuccess);
                const long P = (long)B * Hout * Wout;
                const int per = kB / a.Gout;
                const long nb = std::min<long>(1024, (P + per - 1) / per);
                dy_amax_kernel<<<(int)nb, kB, 0, st>>>((const uint8_t*)dy, P, a.Gout, amax);
                TCAM_CHECK_LAUNCH();
                dy_scale_kernel<<<cdiv(Cout, kB), kB, 0, st>>>(amax, scale, Cout);
                TCAM_CHECK_LAUNCH();
                uint8_t* dy2 = reinterpret_cast<uint8_t*>(scale + Cout);
                dy_to_s2_kernel<<<cdiv(P * a.Gout, kB), kB, 0, st>>>((const uint8_t*)dy, scale,
                                                                      P * a.Gout, a.Gout, dy2);
                TCAM_CHECK_LAUNCH();
                a.dy = dy2;
                a.dscale = scale;
                a.oflow = oflow;
            }
            if constexpr (PRESCALED) {
                TCAM_REQUIRE(dscale_in);
                a.dscale = dscale_in;
            }
            if (g_wgrad_fp32 == 0 || F::NP != 3) {
                // TCAM_WGRAD_PIPE=1: the software-pipelined patch loads (A/B)
                static const bool pipe = getenv("TCAM_WGRAD_PIPE") &&
                                         atoi(getenv("TCAM_WGRAD_PIPE")) == 1;
                if (msub == 1 && pipe)
                    wgrad33x6_kernel<F, 1, true><<<dim3(a.ntiles, splits), 192, 0, st>>>(a);
                else if (msub == 1)
                    wgrad33x6_kernel<F, 1><<<dim3(a.ntiles, splits), 192, 0, st>>>(a);
                else if (pipe)
                    wgrad33x6_kernel<F, 2, true><<<dim3(a.ntiles, splits), 192, 0, st>>>(a);
                else
                    wgrad33x6_kernel<F, 2><<<dim3(a.ntiles, splits), 192, 0, st>>>(a);
                TCAM_CHECK_LAUNCH();
                if (msub == 1) reduce33<1>(a, splits, cout_store, dw, r16, ws, st);
                else reduce33<2>(a, splits, cout_store, dw, r16, ws, st);
            } else if constexpr (F::NP == 3) {
                // fp32 MFMA (tcam_wgrad_force_fp32: A/B and tests; S3 only)
                if (msub == 1) {
                    wgrad33_kernel<1><<<dim3(a.ntiles, splits), 192, 0, st>>>(a);
                    TCAM_CHECK_LAUNCH();
                    reduce33<1>(a, splits, cout_store, dw, r16, ws, st);
                } else {
                    wgrad33_kernel<2><<<dim3(a.ntiles, splits), 384, 0, st>>>(a);
                    TCAM_CHECK_LAUNCH();
                    reduce33<2>(a, splits, cout_store, dw, r16, ws, st);
                }
            }
            TCAM_CHECK_LAUNCH();
            return TCAM_OK;
        }
    }
    if constexpr (PRESCALED) return TCAM_E_ARG;   // 3x3 / stride 1 / pad 1 only
    WgArgs a{};
    int splits = 0;
    TCAM_REQUIRE(make_wg(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w, &a, &splits));
    TCAM_REQUIRE(ws_bytes >= (size_t)splits * a.ntiles * kWT * kWT * sizeof(float));
    a.part = (float*)ws;
    hipStream_t st = as_stream(stream);
    wgrad_kernel<L><<<dim3(a.ntiles, splits), kB, 0, st>>>(a);
    TCAM_CHECK_LAUNCH();
    const long total = (long)cout_store * a.Ctot * KH * KW;
    wgrad_reduce_kernel<<<cdiv(total, kB), kB, 0, st>>>(a, splits, cout_store, dw, r16);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_conv_wgrad_s3(const tcam_conv_src* srcs, int nsrc, int B, const void* dy,
                                  int Cout, int Hout, int Wout, int KH, int KW, int pad_h,
                                  int pad_w, int cout_store, float* dw, void* ws,
                                  size_t ws_bytes, void* stream) {
    return conv_wgrad<LayS3, WgX6>(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w,
                                   cout_store, dw, ws, ws_bytes, 0, stream);
}

extern "C" int tcam_conv_wgrad_s3_f16x3(const tcam_conv_src* srcs, int nsrc, int B,
                                        const void* dy, int Cout, int Hout, int Wout, int KH,
                                        int KW, int pad_h, int pad_w, int cout_store, float* dw,
                                        void* ws, size_t ws_bytes, int* oflow, void* stream) {
    return conv_wgrad<LayS3, WgF3>(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w,
                                   cout_store, dw, ws, ws_bytes, 0, stream, oflow);
}

// The f16x3 training step's 3x3 weight gradient: S2 sources x, dy2 = the per-channel
// scaled S2 copy of dy with its scales dscale (tcam_dy_scaled_s2); three fp16 products per
// MAC, the reduction divides by dscale exactly.  3x3 / stride 1 / pad 1 only.
extern "C" int tcam_conv_wgrad_s2_f16x3(const tcam_conv_src* srcs, int nsrc, int B,
                                        const void* dy2, const float* dscale, int Cout, int Hout,
                                        int Wout, int KH, int KW, int pad_h, int pad_w,
                                        int cout_store, float* dw, void* ws, size_t ws_bytes,
                                        void* stream) {
    return conv_wgrad<LayS2, WgF2>(srcs, nsrc, B, dy2, Cout, Hout, Wout, KH, KW, pad_h, pad_w,
                                   cout_store, dw, ws, ws_bytes, 0, stream, nullptr, dscale);
}

extern "C" int tcam_conv_wgrad_s1(const tcam_conv_src* srcs, int nsrc, int B, const void* dy,
                                  int Cout, int Hout, int Wout, int KH, int KW, int pad_h,
                                  int pad_w, int cout_store, float* dw, void* ws,
                                  size_t ws_bytes, void* stream) {
    return conv_wgrad<LayS1, WgH1>(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w,
                                   cout_store, dw, ws, ws_bytes, 1, stream);
}

// The encoder step's other weight gradients (the 7x7 / stride-2 stem, the 3x3 / stride-2
// conv2 of layer2.0; encoders/resnet.py:85, 206): dy S3 (the exact gradient), x S2 (the
// forward's activations, read at the source's stride), any KH x KW / pad, fp32 MFMA
// (v_mfma_f32_32x32x2_f32: exact products, fp32 sums), deterministic split reduction.
extern "C" size_t tcam_conv_wgrad_generic_ws_bytes(const tcam_conv_src* srcs, int nsrc, int B,
                                                   int Cout, int Hout, int Wout, int KH, int KW) {
    WgArgs a{};
    int splits = 0, dummy = 0;
    if (!make_wg(srcs, nsrc, B, &dummy, Cout, Hout, Wout, KH, KW, 0, 0, &a, &splits)) return 0;
    return (size_t)splits * a.ntiles * kWT * kWT * sizeof(float);
}

extern "C" int tcam_conv_wgrad_s3s2(const tcam_conv_src* srcs, int nsrc, int B, const void* dy,
                                    int Cout, int Hout, int Wout, int KH, int KW, int pad_h,
                                    int pad_w, int cout_store, float* dw, void* ws,
                                    size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(dw && ws && cout_store > 0 && cout_store <= Cout);
    WgArgs a{};
    int splits = 0;
    TCAM_REQUIRE(make_wg(srcs, nsrc, B, dy, Cout, Hout, Wout, KH, KW, pad_h, pad_w, &a, &splits));
    TCAM_REQUIRE(ws_bytes >= (size_t)splits * a.ntiles * kWT * kWT * sizeof(float));
    a.part = (float*)ws;
    hipStream_t st = as_stream(stream);
    wgrad_kernel<LayS3, LayS2><<<dim3(a.ntiles, splits), kB, 0, st>>>(a);
    TCAM_CHECK_LAUNCH();
    const long total = (long)cout_store * a.Ctot * KH * KW;
    wgrad_reduce_kernel<<<cdiv(total, kB), kB, 0, st>>>(a, splits, cout_store, dw, 0);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

static int pack_weight(const float* w, void* out, int mode, int CoutW, int CtotW, int KH,
                       int KW, int c0, int cout_sel, int cin_pad, int h1, void* stream) {
    TCAM_REQUIRE(w && out && CoutW > 0 && CtotW > 0 && KH > 0 && KW > 0);
    int Coutp, Cinp;
    if (mode == 0) {   // cin_pad: zero input channels beyond CtotW (the stem's 8-channel image)
        Coutp = CoutW;
        Cinp = cin_pad > CtotW ? cin_pad : CtotW;
    } else {
        TCAM_REQUIRE(mode == 1 && c0 >= 0 && cout_sel > 0 && c0 + cout_sel <= CtotW);
        Coutp = cout_sel;
        Cinp = cin_pad > CoutW ? cin_pad : CoutW;
    }
    int Kpad, Mpad;
    TCAM_REQUIRE(tcam_conv_x6_weight_dims(KH * KW * Cinp, Coutp, &Kpad, &Mpad) == TCAM_OK);
    pack_kernel<<<cdiv((long)Kpad * Mpad, kB), kB, 0, as_stream(stream)>>>(
        w, (uint16_t*)out, mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp, Kpad, Mpad, h1);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_pack_weight_x6(const float* w, void* out, int mode, int CoutW, int CtotW,
                                   int KH, int KW, int c0, int cout_sel, int cin_pad,
                                   void* stream) {
    return pack_weight(w, out, mode, CoutW, CtotW, KH, KW, c0, cout_sel, cin_pad, 0, stream);
}

extern "C" int tcam_pack_weight_f16(const float* w, void* out, int mode, int CoutW, int CtotW,
                                    int KH, int KW, int c0, int cout_sel, int cin_pad,
                                    void* stream) {
    return pack_weight(w, out, mode, CoutW, CtotW, KH, KW, c0, cout_sel, cin_pad, 1, stream);
}

extern "C" int tcam_pack_weight_f16x3(const float* w, void* out, float* wscale, int mode,
                                      int CoutW, int CtotW, int KH, int KW, int c0, int cout_sel,
                                      int cin_pad, const float* kdiv, void* stream) {
    TCAM_REQUIRE(w && out && wscale && CoutW > 0 && CtotW > 0 && KH > 0 && KW > 0);
    int Coutp, Cinp;
    if (mode == 0) {   // cin_pad: zero input channels beyond CtotW (the stem's 8-channel image)
        Coutp = CoutW;
        Cinp = cin_pad > CtotW ? cin_pad : CtotW;
    } else {
        TCAM_REQUIRE(mode == 1 && c0 >= 0 && cout_sel > 0 && c0 + cout_sel <= CtotW);
        Coutp = cout_sel;
        Cinp = cin_pad > CoutW ? cin_pad : CoutW;
    }
    int Kpad, Mpad;
    TCAM_REQUIRE(tcam_conv_x6_weight_dims(KH * KW * Cinp, Coutp, &Kpad, &Mpad) == TCAM_OK);
    hipStream_t st = as_stream(stream);
    pack_f16_scale_kernel<<<Mpad, kB, 0, st>>>(w, mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp,
                                               Kpad, kdiv, wscale);
    TCAM_CHECK_LAUNCH();
    pack_f16x3_kernel<<<cdiv((long)Kpad * Mpad, kB), kB, 0, st>>>(
        w, mode, CoutW, CtotW, KH, KW, c0, Coutp, Cinp, Kpad, Mpad, kdiv, wscale,
        (uint16_t*)out);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

// The batched packs.  Items as tcam_pack_weight_f16 (f16x3 == 0: wscale, kdiv unused) or
// tcam_pack_weight_f16x3; the descriptor table goes to `table` (tcam_pack_table_bytes(n) of
// device memory), copied only when it differs from the one last copied there.
extern "C" size_t tcam_pack_table_bytes(int n) { return (size_t)(n > 0 ? n : 0) * sizeof(PackDesc); }

extern "C" int tcam_pack_weights(const tcam_pack_item* items, int n, int f16x3, void* table,
                                 void* stream) {
    TCAM_REQUIRE(items && table && n > 0);
    std::vector<PackDesc> t((size_t)n);
    long sb = 0, pb = 0;
    for (int i = 0; i < n; ++i) {
        const tcam_pack_item& it = items[i];
        TCAM_REQUIRE(it.w && it.out && it.CoutW > 0 && it.CtotW > 0 && it.KH > 0 && it.KW > 0);
        TCAM_REQUIRE(!f16x3 || it.wscale);
        PackDesc& d = t[i];
        d.w = it.w;
        d.out = (uint16_t*)it.out;
        d.wscale = it.wscale;
        d.kdiv = f16x3 ? it.kdiv : nullptr;
        d.mode = it.mode;
        d.CoutW = it.CoutW;
        d.CtotW = it.CtotW;
        d.KH = it.KH;
        d.KW = it.KW;
        d.c0 = it.c0;
        if (it.mode == 0) {
            d.Coutp = it.CoutW;
            d.Cinp = it.cin_pad > it.CtotW ? it.cin_pad : it.CtotW;
        } else {
            TCAM_REQUIRE(it.mode == 1 && it.c0 >= 0 && it.cout_sel > 0 &&
                         it.c0 + it.cout_sel <= it.CtotW);
            d.Coutp = it.cout_sel;
            d.Cinp = it.cin_pad > it.CoutW ? it.cin_pad : it.CoutW;
        }
        TCAM_REQUIRE(tcam_conv_x6_weight_dims(d.KH * d.KW * d.Cinp, d.Coutp, &d.Kpad, &d.Mpad) ==
                     TCAM_OK);
        d.sb0 = (int)sb;
        d.pb0 = (int)pb;
        sb += d.Mpad;
        pb += cdiv((long)d.Kpad * d.Mpad, kB);
        TCAM_REQUIRE(sb < (1L << 31) && pb < (1L << 31));
    }
    hipStream_t st = as_stream(stream);
    // the table: copied when it differs from the last one copied to this address
    static std::mutex mu;
    static std::map<void*, std::vector<PackDesc>> last;
    {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<PackDesc>& prev = last[table];
        if (prev.size() != t.size() ||
            memcmp(prev.data(), t.data(), t.size() * sizeof(PackDesc)) != 0) {
            prev = t;   // (the copy's source outlives the call)
            TCAM_REQUIRE(hipMemcpyAsync(table, prev.data(), prev.size() * sizeof(PackDesc),
                                        hipMemcpyHostToDevice, st) == hipSuccess);
        }
    }
    const PackDesc* dt = (const PackDesc*)table;
    if (f16x3) {
        pack_multi_scale_kernel<<<(int)sb, kB, 0, st>>>(dt, n);
        TCAM_CHECK_LAUNCH();
        pack_multi_kernel<true><<<(int)pb, kB, 0, st>>>(dt, n);
    } else {
        pack_multi_kernel<false><<<(int)pb, kB, 0, st>>>(dt, n);
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" size_t tcam_chansum_ws_bytes(int B, int C, long HW) {
    const long chunk = 16384;
    const long nchunks = (HW + chunk - 1) / chunk;
    return (size_t)B * C * nchunks * sizeof(double);
}

extern "C" int tcam_chansum_nchw(const float* x, int B, int C, long HW, float* out, void* ws,
                                 void* stream) {
    TCAM_REQUIRE(x && out && ws && B > 0 && C > 0 && HW > 0);
    const long chunk = 16384;
    const int nchunks = (int)((HW + chunk - 1) / chunk);
    hipStream_t st = as_stream(stream);
    chansum_partial_kernel<<<dim3(nchunks, B * C), kB, 0, st>>>(x, C, HW, chunk, (double*)ws,
                                                                nchunks);
    TCAM_CHECK_LAUNCH();
    chansum_final_kernel<<<cdiv(C, 64), 64, 0, st>>>((const double*)ws, B, C, nchunks, out);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_softmax2(const float* fcams, float* S, int B, long HW, void* stream) {
    TCAM_REQUIRE(fcams && S && B > 0 && HW > 0);
    softmax2_kernel<<<cdiv((long)B * HW, kB), kB, 0, as_stream(stream)>>>(fcams, S, B, HW);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" size_t tcam_tcam_loss_ws_bytes(int B, long HW) {
    const long nchunks = (HW + kLossPix - 1) / kLossPix;
    return (size_t)B * nchunks * 5 * sizeof(double) + (size_t)(2 + 2 * B) * sizeof(float) + 256;
}

extern "C" int tcam_tcam_losses_ex(const float* fcams, const float* S, const int32_t* seeds,
                                   const float* AS, const float* gx, const float* extra,
                                   int B, long HW, float lam_sl, float lam_crf,
                                   float lam_size, float elb_t, float* losses, float* dfcams,
                                   void* ws, void* stream) {
    TCAM_REQUIRE(fcams && S && losses && dfcams && ws && B > 0 && HW > 0 && elb_t > 0.f);
    TCAM_REQUIRE((gx == nullptr) == (extra == nullptr));
    hipStream_t st = as_stream(stream);
    const int nchunks = (int)((HW + kLossPix - 1) / kLossPix);
    double* part = (double*)ws;
    float* coef = (float*)((char*)ws + (size_t)B * nchunks * 5 * sizeof(double));
    loss_partial_kernel<<<dim3(nchunks, B), kB, 0, st>>>(fcams, S, seeds, AS, HW, nchunks, part);
    TCAM_CHECK_LAUNCH();
    LossCfg cfg{lam_sl, lam_crf, lam_size, elb_t, seeds != nullptr, AS != nullptr,
                lam_size != 0.f};
    loss_finalize_kernel<<<1, kFinBlock, 0, st>>>(part, B, nchunks, cfg, extra, losses, coef);
    TCAM_CHECK_LAUNCH();
    loss_grad_kernel<<<cdiv((long)B * HW, kB), kB, 0, st>>>(S, seeds, AS, gx, coef, B, HW,
                                                             dfcams);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_tcam_losses(const float* fcams, const float* S, const int32_t* seeds,
                                const float* AS, int B, long HW, float lam_sl, float lam_crf,
                                float lam_size, float elb_t, float* losses, float* dfcams,
                                void* ws, void* stream) {
    return tcam_tcam_losses_ex(fcams, S, seeds, AS, nullptr, nullptr, B, HW, lam_sl, lam_crf,
                               lam_size, elb_t, losses, dfcams, ws, stream);
}

extern "C" int tcam_mosaic_gather(const float* src, const int32_t* idx, int G, int L, int C,
                                  int H, int W, float* out, void* stream) {
    TCAM_REQUIRE(src && idx && out && G > 0 && L > 0 && C > 0 && H > 0 && W > 0);
    hipStream_t st = as_stream(stream);
    if (W % 4 == 0) {
        const long n = (long)G * L * C * H * (W / 4);
        mosaic_gather_kernel<4><<<cdiv(n, kB), kB, 0, st>>>(src, idx, G, L, C, H, W, out);
    } else {
        const long n = (long)G * L * C * H * W;
        mosaic_gather_kernel<1><<<cdiv(n, kB), kB, 0, st>>>(src, idx, G, L, C, H, W, out);
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_mosaic_scatter(const float* mosaic, const int32_t* occ_start,
                                   const int32_t* occ, int B, int L, int C, int H, int W,
                                   float coef, int accumulate, float* dst, void* stream) {
    TCAM_REQUIRE(mosaic && occ_start && occ && dst && B > 0 && L > 0 && C > 0 && H > 0 &&
                 W > 0);
    const long n = (long)B * C * H * W;
    mosaic_scatter_kernel<<<cdiv(n, kB), kB, 0, as_stream(stream)>>>(
        mosaic, occ_start, occ, B, L, C, H, W, coef, accumulate, dst);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_sgd_step(float* p, const float* g, float* buf, long n, float lr,
                             float momentum, float dampening, float weight_decay, int nesterov,
                             int first, float grad_scale, void* stream) {
    TCAM_REQUIRE(p && g && n > 0 && (momentum == 0.f || buf));
    sgd_kernel<<<cdiv(n, kB), kB, 0, as_stream(stream)>>>(p, g, buf, n, lr, momentum, dampening,
                                                          weight_decay, nesterov, first,
                                                          grad_scale);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_sgd_step_gated(float* p, const float* g, float* buf, long n, float lr,
                                   float momentum, float dampening, float weight_decay,
                                   int nesterov, float grad_scale, const float* gate,
                                   int* steps, int* skipped, void* stream) {
    TCAM_REQUIRE(p && g && gate && steps && n > 0 && (momentum == 0.f || buf));
    hipStream_t st = as_stream(stream);
    sgd_gated_kernel<<<cdiv(n, kB), kB, 0, st>>>(p, g, buf, n, lr, momentum, dampening,
                                                 weight_decay, nesterov, grad_scale, gate, steps);
    TCAM_CHECK_LAUNCH();
    sgd_count_kernel<<<1, 64, 0, st>>>(gate, steps, skipped);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_amp_unscale(float* g, long n, const float* scale, float* found_inf,
                                void* stream) {
    TCAM_REQUIRE(g && scale && found_inf && n > 0);
    amp_unscale_kernel<<<cdiv(n, kB), kB, 0, as_stream(stream)>>>(g, n, scale, found_inf);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_sgd_step_amp(float* p, const float* g, float* buf, long n, float lr,
                                 float momentum, float dampening, float weight_decay,
                                 int nesterov, float grad_scale, const float* gate, int* steps,
                                 int* skipped, float* scale, int* tracker, float growth_factor,
                                 float backoff_factor, int growth_interval, void* stream) {
    TCAM_REQUIRE(p && g && gate && steps && scale && tracker && n > 0 &&
                 (momentum == 0.f || buf) && growth_interval > 0);
    hipStream_t st = as_stream(stream);
    sgd_amp_kernel<<<cdiv(n, kB), kB, 0, st>>>(p, g, buf, n, lr, momentum, dampening,
                                               weight_decay, nesterov, grad_scale, gate, steps);
    TCAM_CHECK_LAUNCH();
    amp_update_kernel<<<1, 64, 0, st>>>(gate, steps, skipped, scale, tracker, growth_factor,
                                        backoff_factor, growth_interval);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
