// Kernels over the S3 activation layout used by the x6 convolution path
// (conv_x6.hip): NHWC, channels in groups of 8 stored as [hi x8][mid x8]
// [lo x8] bf16 (48 B per group), value = (hi + mid) + lo exactly.
//
//   image (NCHW fp32) -> S3 with channel padding      (stem input)
//   S3 -> NCHW fp32                                    (feature export, tests)
//   MaxPool2d(3, 2, 1)                                 (resnet.py:99)
//   nearest x2 + bilinear(align_corners=True) resample (decoder.py:43-51)
//   AdaptiveAvgPool2d(1) + Linear (WGAP)               (poolings/core.py:96-115)
//   SegmentationHead conv3x3 + SegmentationCam + u8    (heads.py:19-36,
//                                                        builtincam.py:201-225)
//   STD_CL CAM                                          (cams/core.py:139-193)
// All are HBM-bound: one pass over their input, 6 B per element.
#include "common.h"
#include "s3_util.h"

namespace {

using s3::G8;
using s3::bf_lo;
using s3::bf_hi;
using s3::bfbits;

// ---------------------------------------------------------------- layout
// thread per (pixel, group)
template <class L>
__global__ void from_nchw_kernel(const float* __restrict__ in, uint8_t* __restrict__ out, int C,
                                 int HW, int G, long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    const long pix = i / G;
    const long b = pix / HW;
    const int hw = (int)(pix - b * HW);
    G8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = 8 * g + e;
        v.v[e] = c < C ? in[(b * C + c) * HW + hw] : 0.f;
    }
    L::store(out + i * L::GB, v);
}

template <class L>
__global__ void to_nchw_kernel(const uint8_t* __restrict__ in, float* __restrict__ out, int C,
                               int HW, int G, long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    const long pix = i / G;
    const long b = pix / HW;
    const int hw = (int)(pix - b * HW);
    const G8 v = L::load(in + i * L::GB);
#pragma unroll
    for (int e = 0; e < 8; ++e) out[(b * C + 8 * g + e) * HW + hw] = v.v[e];
}

// ------------------------------------------------------------- max-pool
template <class L>
__global__ void maxpool_s3_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                  int G, int H, int W, int Ho, int Wo, long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int ox = (int)(t % Wo);
    t /= Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    // window taps outside the frame are clamped onto its nearest in-frame row / column, which
    // lies in the same window (the centre 2oy, 2ox is always inside): a duplicate leaves the
    // max unchanged, and the nine loads carry no branches, so they are all in flight at once
    G8 v[9];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        const int y = min(max(2 * oy - 1 + dy, 0), H - 1);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int x = min(max(2 * ox - 1 + dx, 0), W - 1);
            v[3 * dy + dx] = L::load(in + (((b * H + y) * W + x) * G + g) * L::GB);
        }
    }
    G8 m;
#pragma unroll
    for (int e = 0; e < 8; ++e) m.v[e] = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            m.v[e] = (v[k].v[e] > m.v[e] || v[k].v[e] != v[k].v[e]) ? v[k].v[e] : m.v[e];
    L::store(out + i * L::GB, m);
}

// General KHxKW / stride / pad pooling (torch max_pool2d / avg_pool2d semantics; the
// caller gives Ho, Wo, which encode ceil_mode).  mode 0: max (NaN propagates);
// mode 1: average with count_include_pad=True — divisor (hend - hstart)(wend - wstart)
// with hend = min(hstart + K, H + pad) before clipping to the input, summed row-major
// as ATen's CPU kernel does.  Output written into groups [ogo, ogo + G) of a tensor with
// ogs groups per pixel (fused channel concat: InceptionB's pool branch,
// wsol_backbones/inceptionv3.py:127-132).
template <class L>
__global__ void pool_s3_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                               int G, int H, int W, int Ho, int Wo, int KH, int KW, int st,
                               int pad, int mode, int ogs, int ogo, long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int ox = (int)(t % Wo);
    t /= Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    const int hs = oy * st - pad, ws = ox * st - pad;
    const int he = min(hs + KH, H + pad), we = min(ws + KW, W + pad);
    const int div = (he - hs) * (we - ws);
    G8 m;
#pragma unroll
    for (int e = 0; e < 8; ++e) m.v[e] = mode ? 0.f : -INFINITY;
    for (int y = max(hs, 0); y < min(he, H); ++y) {
        for (int x = max(ws, 0); x < min(we, W); ++x) {
            const G8 v = L::load(in + (((b * H + y) * W + x) * G + g) * L::GB);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (mode)
                    m.v[e] += v.v[e];
                else
                    m.v[e] = (v.v[e] > m.v[e] || v.v[e] != v.v[e]) ? v.v[e] : m.v[e];
            }
        }
    }
    if (mode) {
#pragma unroll
        for (int e = 0; e < 8; ++e) m.v[e] = m.v[e] / (float)div;
    }
    L::store(out + ((((b * Ho + oy) * Wo + ox) * ogs) + ogo + g) * L::GB, m);
}

// ------------------------------------------------------ up2 + bilinear
template <class L>
__global__ void up2_resize_s3_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                     int G, int H, int W, int Ho, int Wo, float sh, float sw,
                                     long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int g = (int)(i % G);
    long t = i / G;
    const int ox = (int)(t % Wo);
    t /= Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    const int Hu = 2 * H, Wu = 2 * W;
    const float ry = sh * (float)oy, rx = sw * (float)ox;
    const int y0 = (int)ry, x0 = (int)rx;
    const int y1 = y0 + (y0 < Hu - 1 ? 1 : 0);
    const int x1 = x0 + (x0 < Wu - 1 ? 1 : 0);
    const float ly1 = fminf(fmaxf(ry - (float)y0, 0.f), 1.f), ly0 = 1.f - ly1;
    const float lx1 = fminf(fmaxf(rx - (float)x0, 0.f), 1.f), lx0 = 1.f - lx1;
    auto at = [&](int y, int x) {
        return L::load(in + (((b * H + (y >> 1)) * W + (x >> 1)) * G + g) * L::GB);
    };
    const G8 v00 = at(y0, x0), v01 = at(y0, x1), v10 = at(y1, x0), v11 = at(y1, x1);
    G8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        r.v[e] = ly0 * (lx0 * v00.v[e] + lx1 * v01.v[e]) + ly1 * (lx0 * v10.v[e] + lx1 * v11.v[e]);
    L::store(out + i * L::GB, r);
}

// ------------------------------------------------------------------ WGAP
// Partial channel sums over a chunk of pixels: grid (chunks, B), thread per group.  The
// pixels' group rows (48 G contiguous bytes each) are read as consecutive 16-B pieces per
// lane, POOL_PX pixels at a time, into LDS; each thread then sums its group's 8 channels
// over the pixels in pixel order (the per-group loop's exact arithmetic).  Reading each
// group's 48 B straight from global put lanes 48 B apart: every 16-B load touched a
// third of the lines of three such loads, ~1 TB/s.
template <class L>
__global__ __launch_bounds__(1024) void pool_partial_kernel(const uint8_t* __restrict__ x,
                                                            float* __restrict__ part, int G,
                                                            int HW, int chunk, int nchunks) {
    // a thread per 8-channel group sums its chunk's pixels in order, straight from memory
    // (consecutive threads read consecutive groups of a pixel: coalesced; the loads of
    // successive pixels do not depend on the sums and pipeline)
    const int b = blockIdx.y, ch = blockIdx.x;
    const int p0 = ch * chunk, p1 = min(HW, p0 + chunk);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int g = threadIdx.x;         // blockDim >= G (host)
    if (g < G) {
        const uint8_t* src = x + (((long)b * HW + p0) * G + g) * L::GB;
#pragma unroll 8
        for (int p = p0; p < p1; ++p, src += (long)G * L::GB) {
            const G8 v = L::load(src);
#pragma unroll
            for (int e = 0; e < 8; ++e) s[e] += v.v[e];
        }
    }
    if (threadIdx.x < G) {
        float* dst = part + ((long)b * nchunks + ch) * G * 8 + 8 * threadIdx.x;
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = s[e];
    }
}

// mean = sum over chunks / HW; logits = Linear(mean).  Block per frame.
__global__ void pool_linear_kernel(const float* __restrict__ part, const float* __restrict__ w,
                                   const float* __restrict__ bias, float* __restrict__ logits,
                                   float* __restrict__ mean_out, int C, int HW, int nchunks,
                                   int classes) {
    extern __shared__ float mean[];
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int ch = 0; ch < nchunks; ++ch) s += part[((long)b * nchunks + ch) * C + c];
        mean[c] = s / (float)HW;
        if (mean_out) mean_out[(long)b * C + c] = mean[c];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int k = wid; k < classes; k += nw) {
        float s = 0.f;
        for (int c = lane; c < C; c += 64) s += mean[c] * w[(long)k * C + c];
        s = wave_sum(s);
        if (lane == 0) logits[(long)b * classes + k] = s + bias[k];
    }
}

// ------------------------------------------------- segmentation head + CAM
// conv3x3 (Cin -> 2, pad 1, bias) -> softmax[:, 1] (or argmax) -> nan_to_num
// -> uint8(cam * 255).  A block owns a 16x16 output tile of one frame: its 18x18 input
// halo is read once (each pixel's 48-B groups contiguous, whole halo rows per wave) and
// kept as fp32 in LDS, channel-major; a thread per output pixel then accumulates its
// 9 taps x Cin from LDS in the order (kh, kw, channel) with fmaf, skipping taps outside
// the frame — the per-pixel kernel's exact arithmetic.
constexpr int SEG_MAX_G = 8;  // Cin <= 64
constexpr int SEG_T = 16, SEG_H = SEG_T + 2, SEG_PX = SEG_H * SEG_H;
template <class L>
__global__ __launch_bounds__(256) void seghead_s3_kernel(
    const uint8_t* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ fcams, float* __restrict__ cam, uint8_t* __restrict__ cam_u8, int G,
    int H, int W, int argmax) {
    __shared__ float ws[2][9][SEG_MAX_G * 8];  // [o][tap][c]
    extern __shared__ float hx[];                 // [c][halo pixel], Cin x SEG_PX
    const int Cin = 8 * G;
    for (int i = threadIdx.x; i < 2 * Cin * 9; i += blockDim.x) {
        const int o = i / (Cin * 9), r = i % (Cin * 9), c = r / 9, tap = r % 9;
        ws[o][tap][c] = w[i];  // PyTorch (2, Cin, 3, 3)
    }
    const int tx = (W + SEG_T - 1) / SEG_T, ty = (H + SEG_T - 1) / SEG_T;
    const int b = blockIdx.x / (tx * ty), tr = blockIdx.x % (tx * ty);
    const int oy0 = (tr / tx) * SEG_T, ox0 = (tr % tx) * SEG_T;
    // the halo in batches of SEG_AHEAD items per thread: the batch's loads issued together
    // (one memory latency per batch; a load-store loop waits on each load before its store)
    constexpr int SEG_AHEAD = 4;
    for (int it0 = 0; it0 < SEG_PX * G; it0 += SEG_AHEAD * (int)blockDim.x) {
        G8 v[SEG_AHEAD];
#pragma unroll
        for (int u = 0; u < SEG_AHEAD; ++u) {
            const int it = it0 + u * blockDim.x + threadIdx.x;
            const int hp = it / G, g = it - hp * G;
            const int y = oy0 - 1 + hp / SEG_H, xx = ox0 - 1 + hp % SEG_H;
            if (it < SEG_PX * G && (unsigned)y < (unsigned)H && (unsigned)xx < (unsigned)W) {
                v[u] = L::load(x + ((((long)b * H + y) * W + xx) * G + g) * L::GB);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[u].v[e] = 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < SEG_AHEAD; ++u) {
            const int it = it0 + u * blockDim.x + threadIdx.x;
            if (it >= SEG_PX * G) continue;
            const int hp = it / G, g = it - hp * G;
#pragma unroll
            for (int e = 0; e < 8; ++e) hx[(8 * g + e) * SEG_PX + hp] = v[u].v[e];
        }
    }
    __syncthreads();
    const int ly = threadIdx.x / SEG_T, lx = threadIdx.x % SEG_T;
    const int py = oy0 + ly, px = ox0 + lx;
    if (py >= H || px >= W) return;
    float a0 = 0.f, a1 = 0.f;
    for (int kh = 0; kh < 3; ++kh) {
        if ((unsigned)(py + kh - 1) >= (unsigned)H) continue;
        for (int kw = 0; kw < 3; ++kw) {
            if ((unsigned)(px + kw - 1) >= (unsigned)W) continue;
            const int tap = kh * 3 + kw, hp = (ly + kh) * SEG_H + lx + kw;
            for (int c = 0; c < Cin; ++c) {
                const float v = hx[c * SEG_PX + hp];
                a0 = fmaf(ws[0][tap][c], v, a0);
                a1 = fmaf(ws[1][tap][c], v, a1);
            }
        }
    }
    a0 += bias[0];
    a1 += bias[1];
    const int HW = H * W;
    const long pix = (long)py * W + px;
    if (fcams) {
        fcams[((long)b * 2 + 0) * HW + pix] = a0;
        fcams[((long)b * 2 + 1) * HW + pix] = a1;
    }
    float c1;
    if (argmax) {
        c1 = (a1 > a0) ? 1.f : 0.f;  // torch.argmax: first max wins ties
    } else {
        const float m = fmaxf(a0, a1);
        const float e0 = expf(a0 - m), e1 = expf(a1 - m);
        c1 = e1 / (e0 + e1);
    }
    if (c1 != c1) c1 = 0.f;  // nan_to_num(nan=0, posinf=1, neginf=0)
    if (isinf(c1)) c1 = c1 > 0.f ? 1.f : 0.f;
    if (cam) cam[(long)b * HW + pix] = c1;
    if (cam_u8) cam_u8[(long)b * HW + pix] = (uint8_t)(int)((double)c1 * 255.0);
}

// fcams resized to the input size when the decoder output differs from it
// (FCAMModel.forward, base/model.py:148-154: bilinear, align_corners=True — InceptionV3 at
// 299 decodes to 300), then SegmentationCam + u8 as seghead_s3_kernel.
__global__ void resize_cam_kernel(const float* __restrict__ fin, float* __restrict__ fout,
                                  float* __restrict__ cam, uint8_t* __restrict__ cam_u8, int Hi,
                                  int Wi, int Ho, int Wo, float sh, float sw, long total,
                                  int argmax) {
#pragma clang fp contract(off)   // ATen's fp32 tap positions: ly1 = rounded(sh * oy) - y0
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int ox = (int)(i % Wo);
    const long t = i / Wo;
    const int oy = (int)(t % Ho);
    const long b = t / Ho;
    // ATen upsample_bilinear2d, align_corners=True: src = scale * dst
    const float ry = sh * (float)oy, rx = sw * (float)ox;
    const int y0 = (int)ry, x0 = (int)rx;
    const int y1 = y0 + (y0 < Hi - 1 ? 1 : 0);
    const int x1 = x0 + (x0 < Wi - 1 ? 1 : 0);
    const float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
    const float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
    float a[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float* f = fin + (b * 2 + c) * (long)Hi * Wi;
        a[c] = ly0 * (lx0 * f[y0 * Wi + x0] + lx1 * f[y0 * Wi + x1]) +
               ly1 * (lx0 * f[y1 * Wi + x0] + lx1 * f[y1 * Wi + x1]);
    }
    const long HW = (long)Ho * Wo;
    const long pix = (long)oy * Wo + ox;
    if (fout) {
        fout[(b * 2 + 0) * HW + pix] = a[0];
        fout[(b * 2 + 1) * HW + pix] = a[1];
    }
    float c1;
    if (argmax) {
        c1 = (a[1] > a[0]) ? 1.f : 0.f;
    } else {
        const float m = fmaxf(a[0], a[1]);
        const float e0 = expf(a[0] - m), e1 = expf(a[1] - m);
        c1 = e1 / (e0 + e1);
    }
    if (c1 != c1) c1 = 0.f;
    if (isinf(c1)) c1 = c1 > 0.f ? 1.f : 0.f;
    if (cam) cam[b * HW + pix] = c1;
    if (cam_u8) cam_u8[b * HW + pix] = (uint8_t)(int)((double)c1 * 255.0);
}

// Adjoint of resize_cam_kernel's bilinear (align_corners=True) resize for the training
// backward (InceptionV3 decodes 300 for a 299 input): din[y][x] = sum over the output
// pixels whose taps touch (y, x) of tap weight * dout, gathered per input pixel (no
// atomics: deterministic), with the forward's fp32 tap positions and weights.
__global__ void resize_ac_bwd_kernel(const float* __restrict__ dout, float* __restrict__ din,
                                     int Hi, int Wi, int Ho, int Wo, float sh, float sw,
                                     long total) {
#pragma clang fp contract(off)   // the forward's fp32 tap positions (no fma into ly1 / lx1)
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int x = (int)(i % Wi);
    const long t = i / Wi;
    const int y = (int)(t % Hi);
    const long bc = t / Hi;
    const float* g = dout + bc * (long)Ho * Wo;
    int oy0 = 0, oy1 = Ho - 1, ox0 = 0, ox1 = Wo - 1;
    if (sh > 0.f) {
        oy0 = max(0, (int)floorf((float)(y - 1) / sh) - 1);
        oy1 = min(Ho - 1, (int)ceilf((float)(y + 1) / sh) + 1);
    }
    if (sw > 0.f) {
        ox0 = max(0, (int)floorf((float)(x - 1) / sw) - 1);
        ox1 = min(Wo - 1, (int)ceilf((float)(x + 1) / sw) + 1);
    }
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
        const float ry = sh * (float)oy;
        const int y0 = (int)ry;
        const int y1 = y0 + (y0 < Hi - 1 ? 1 : 0);
        const float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
        const float wy = (y0 == y ? ly0 : 0.f) + (y1 == y ? ly1 : 0.f);
        if (wy == 0.f) continue;
        for (int ox = ox0; ox <= ox1; ++ox) {
            const float rx = sw * (float)ox;
            const int x0 = (int)rx;
            const int x1 = x0 + (x0 < Wi - 1 ? 1 : 0);
            const float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
            const float wx = (x0 == x ? lx0 : 0.f) + (x1 == x ? lx1 : 0.f);
            if (wx != 0.f) acc += (wy * wx) * g[(long)oy * Wo + ox];
        }
    }
    din[i] = acc;
}

// ---------------------------------------------------------- STD_CL CAM
// One workgroup per frame; a wave per position (lanes over channel groups):
//   low = nansum_c w[cls, c] * A[c]; min-max normalise; nan_to_num;
//   bilinear(align_corners=False) to (Ho, Wo).
constexpr int STD_MAX_HW = 4096;
template <class L>
__global__ __launch_bounds__(1024) void std_cam_s3_kernel(
    const uint8_t* __restrict__ A, const float* __restrict__ fcw, const int32_t* __restrict__ cls,
    float* __restrict__ low_out, float* __restrict__ cam, uint8_t* __restrict__ cam_u8, int G,
    int h, int w, int Ho, int Wo) {
    __shared__ float low[STD_MAX_HW];
    __shared__ float red[32];
    const int b = blockIdx.x;
    const int hw = h * w;
    const int C = 8 * G;
    const float* wr = fcw + (long)cls[b] * C;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int p = wid; p < hw; p += nw) {
        const uint8_t* src = A + ((long)b * hw + p) * G * L::GB;
        float s = 0.f;
        for (int g = lane; g < G; g += 64) {
            const G8 v = L::load(src + g * L::GB);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float t = wr[8 * g + e] * v.v[e];
                if (t == t) s += t;  // nansum
            }
        }
        s = wave_sum(s);
        if (lane == 0) low[p] = s;
    }
    __syncthreads();
    float mn = INFINITY;
    for (int p = threadIdx.x; p < hw; p += blockDim.x) mn = fminf(mn, low[p]);
    mn = wave_min(mn);
    if (lane == 0) red[wid] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = red[0];
        for (int i = 1; i < nw; ++i) m = fminf(m, red[i]);
        red[31] = m;
    }
    __syncthreads();
    mn = red[31];
    __syncthreads();
    float mx = -INFINITY;
    for (int p = threadIdx.x; p < hw; p += blockDim.x) {
        const float v = low[p] - mn;
        low[p] = v;
        mx = fmaxf(mx, v);
    }
    mx = wave_max(mx);
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = red[0];
        for (int i = 1; i < nw; ++i) m = fmaxf(m, red[i]);
        red[30] = m;
    }
    __syncthreads();
    mx = red[30];
    for (int p = threadIdx.x; p < hw; p += blockDim.x) {
        float v = low[p] / mx;
        if (v != v) v = 0.f;
        if (isinf(v)) v = v > 0.f ? 1.f : 0.f;
        low[p] = v;
        if (low_out) low_out[(long)b * hw + p] = v;
    }
    __syncthreads();
    const float sh = (float)h / (float)Ho, sw = (float)w / (float)Wo;
    for (int p = threadIdx.x; p < Ho * Wo; p += blockDim.x) {
        const int oy = p / Wo, ox = p % Wo;
        const float ry = fmaxf(sh * ((float)oy + 0.5f) - 0.5f, 0.f);
        const float rx = fmaxf(sw * ((float)ox + 0.5f) - 0.5f, 0.f);
        const int y0 = (int)ry, x0 = (int)rx;
        const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
        const float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
        const float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
        const float v = ly0 * (lx0 * low[y0 * w + x0] + lx1 * low[y0 * w + x1]) +
                         ly1 * (lx0 * low[y1 * w + x0] + lx1 * low[y1 * w + x1]);
        if (cam) cam[(long)b * Ho * Wo + p] = v;
        if (cam_u8) cam_u8[(long)b * Ho * Wo + p] = (uint8_t)(int)((double)v * 255.0);
    }
}

constexpr int POOL_CHUNK = 32;

}  // namespace

template <class L>
static int from_nchw(const float* in, void* out, int B, int C, int H, int W, int Cpad,
                     void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && H > 0 && W > 0 && Cpad >= C && Cpad % 8 == 0);
    const long total = (long)B * H * W * (Cpad / 8);
    from_nchw_kernel<L><<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        in, (uint8_t*)out, C, H * W, Cpad / 8, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int to_nchw(const void* in, float* out, int B, int C, int H, int W, void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    const long total = (long)B * H * W * (C / 8);
    to_nchw_kernel<L><<<cdiv(total, 256), 256, 0, as_stream(stream)>>>((const uint8_t*)in, out, C,
                                                                    H * W, C / 8, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int maxpool3x3s2(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                        void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0);
    TCAM_REQUIRE(Ho == (H + 2 - 3) / 2 + 1 && Wo == (W + 2 - 3) / 2 + 1);
    const long total = (long)B * Ho * Wo * (C / 8);
    maxpool_s3_kernel<L><<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        (const uint8_t*)in, (uint8_t*)out, C / 8, H, W, Ho, Wo, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int pool2d(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo, int KH,
                  int KW, int stride, int pad, int mode, int out_cstride, int out_coff,
                  void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && Ho > 0 &&
                 Wo > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0 && (mode == 0 || mode == 1));
    TCAM_REQUIRE(2 * pad <= KH && 2 * pad <= KW);   // torch's pad <= kernel / 2 rule
    if (out_cstride == 0) out_cstride = C;
    TCAM_REQUIRE(out_cstride % 8 == 0 && out_coff % 8 == 0 && out_coff >= 0 &&
                 out_coff + C <= out_cstride);
    // every window must start inside the padded input (torch's ceil_mode rule)
    TCAM_REQUIRE((Ho - 1) * stride - pad < H && (Wo - 1) * stride - pad < W);
    const long total = (long)B * Ho * Wo * (C / 8);
    pool_s3_kernel<L><<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        (const uint8_t*)in, (uint8_t*)out, C / 8, H, W, Ho, Wo, KH, KW, stride, pad, mode,
        out_cstride / 8, out_coff / 8, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int up2_resize(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                      void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && Ho > 0 &&
                 Wo > 0);
    const float sh = Ho > 1 ? (float)(2 * H - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(2 * W - 1) / (float)(Wo - 1) : 0.f;
    const long total = (long)B * Ho * Wo * (C / 8);
    up2_resize_s3_kernel<L><<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        (const uint8_t*)in, (uint8_t*)out, C / 8, H, W, Ho, Wo, sh, sw, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" size_t tcam_wgap_s3_ws_bytes(int B, int C, int HW) {
    const int nchunks = (HW + POOL_CHUNK - 1) / POOL_CHUNK;
    return (size_t)B * nchunks * C * sizeof(float);
}

template <class L>
static int wgap(const void* x, const float* fc_w, const float* fc_b, float* logits, float* mean,
                float* ws, int B, int C, int HW, int classes, void* stream) {
    TCAM_REQUIRE(x && fc_w && fc_b && logits && ws && B > 0 && C > 0 && C % 8 == 0 && HW > 0 &&
                 classes > 0 && C <= 8192);
    hipStream_t st = as_stream(stream);
    const int nchunks = (HW + POOL_CHUNK - 1) / POOL_CHUNK;
    const int threads = std::max(64, (C / 8 + 63) / 64 * 64);   // a thread per group
    pool_partial_kernel<L><<<dim3(nchunks, B), threads, 0, st>>>(
        (const uint8_t*)x, ws, C / 8, HW, POOL_CHUNK, nchunks);
    TCAM_CHECK_LAUNCH();
    pool_linear_kernel<<<B, 1024, C * sizeof(float), st>>>(ws, fc_w, fc_b, logits, mean, C, HW,
                                                           nchunks, classes);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int seghead_cam(const void* x, const float* w, const float* b, float* fcams, float* cam,
                       uint8_t* cam_u8, int B, int Cin, int H, int W, int argmax, void* stream) {
    TCAM_REQUIRE(x && w && b && B > 0 && Cin > 0 && Cin % 8 == 0 && Cin <= 8 * SEG_MAX_G &&
                 H > 0 && W > 0);
    const long blocks = (long)B * ((H + SEG_T - 1) / SEG_T) * ((W + SEG_T - 1) / SEG_T);
    seghead_s3_kernel<L><<<(unsigned)blocks, 256, sizeof(float) * Cin * SEG_PX,
                        as_stream(stream)>>>(
        (const uint8_t*)x, w, b, fcams, cam, cam_u8, Cin / 8, H, W, argmax);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_resize_cam(const float* fcams_in, float* fcams_out, float* cam,
                               uint8_t* cam_u8, int B, int Hi, int Wi, int Ho, int Wo, int argmax,
                               void* stream) {
    TCAM_REQUIRE(fcams_in && B > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0);
    const float sh = Ho > 1 ? (float)(Hi - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(Wi - 1) / (float)(Wo - 1) : 0.f;
    const long total = (long)B * Ho * Wo;
    resize_cam_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        fcams_in, fcams_out, cam, cam_u8, Hi, Wi, Ho, Wo, sh, sw, total, argmax);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_resize_ac_bwd(const float* dout, float* din, int BC, int Hi, int Wi,
                                  int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(dout && din && BC > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0);
    const float sh = Ho > 1 ? (float)(Hi - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(Wi - 1) / (float)(Wo - 1) : 0.f;
    const long total = (long)BC * Hi * Wi;
    resize_ac_bwd_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(dout, din, Hi, Wi, Ho,
                                                                          Wo, sh, sw, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <class L>
static int std_cam(const void* A, const float* fc_w, const int32_t* cls, float* low, float* cam,
                   uint8_t* cam_u8, int B, int C, int h, int w, int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(A && fc_w && cls && B > 0 && C > 0 && C % 8 == 0 && h > 0 && w > 0 &&
                 h * w <= STD_MAX_HW && Ho > 0 && Wo > 0);
    std_cam_s3_kernel<L><<<B, 1024, 0, as_stream(stream)>>>((const uint8_t*)A, fc_w, cls, low, cam,
                                                         cam_u8, C / 8, h, w, Ho, Wo);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

// ---- entry points: S3 (bf16 x3, the x6 path) and S2 (fp16 x2, the f16x3 path) ----
// Re-layout between S2 and S3: one thread per 8-channel group; S2 -> S3 is exact (22 <= 24
// bits), S3 -> S2 rounds to the 22-bit pair (and overflows beyond 65504).
template <class LI, class LO>
__global__ void relayout_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                long groups) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= groups) return;
    LO::store(out + i * LO::GB, LI::load(in + i * LI::GB));
}

extern "C" int tcam_s2_to_s3(const void* in, void* out, long groups, void* stream) {
    TCAM_REQUIRE(in && out && groups >= 0);
    if (groups == 0) return TCAM_OK;
    relayout_kernel<LayS2, LayS3><<<cdiv(groups, 256), 256, 0, as_stream(stream)>>>(
        (const uint8_t*)in, (uint8_t*)out, groups);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_s3_to_s2(const void* in, void* out, long groups, void* stream) {
    TCAM_REQUIRE(in && out && groups >= 0);
    if (groups == 0) return TCAM_OK;
    relayout_kernel<LayS3, LayS2><<<cdiv(groups, 256), 256, 0, as_stream(stream)>>>(
        (const uint8_t*)in, (uint8_t*)out, groups);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

#define TCAM_LAYOUT_ENTRIES(SUF, L)                                                           \
    extern "C" int tcam_##SUF##_from_nchw(const float* in, void* out, int B, int C, int H,      \
                                          int W, int Cpad, void* stream) {                     \
        return from_nchw<L>(in, out, B, C, H, W, Cpad, stream);                                \
    }                                                                                          \
    extern "C" int tcam_##SUF##_to_nchw(const void* in, float* out, int B, int C, int H, int W, \
                                        void* stream) {                                        \
        return to_nchw<L>(in, out, B, C, H, W, stream);                                        \
    }                                                                                          \
    extern "C" int tcam_maxpool3x3s2_##SUF(const void* in, void* out, int B, int C, int H,      \
                                           int W, int Ho, int Wo, void* stream) {              \
        return maxpool3x3s2<L>(in, out, B, C, H, W, Ho, Wo, stream);                           \
    }                                                                                          \
    extern "C" int tcam_pool2d_##SUF(const void* in, void* out, int B, int C, int H, int W,     \
                                     int Ho, int Wo, int KH, int KW, int stride, int pad,      \
                                     int mode, int out_cstride, int out_coff, void* stream) {  \
        return pool2d<L>(in, out, B, C, H, W, Ho, Wo, KH, KW, stride, pad, mode, out_cstride,  \
                         out_coff, stream);                                                    \
    }                                                                                          \
    extern "C" int tcam_up2_resize_##SUF(const void* in, void* out, int B, int C, int H, int W, \
                                         int Ho, int Wo, void* stream) {                       \
        return up2_resize<L>(in, out, B, C, H, W, Ho, Wo, stream);                             \
    }                                                                                          \
    extern "C" int tcam_wgap_##SUF(const void* x, const float* fc_w, const float* fc_b,         \
                                   float* logits, float* mean, float* ws, int B, int C, int HW, \
                                   int classes, void* stream) {                                \
        return wgap<L>(x, fc_w, fc_b, logits, mean, ws, B, C, HW, classes, stream);            \
    }                                                                                          \
    extern "C" int tcam_seghead_cam_##SUF(const void* x, const float* w, const float* b,        \
                                          float* fcams, float* cam, uint8_t* cam_u8, int B,    \
                                          int Cin, int H, int W, int argmax, void* stream) {   \
        return seghead_cam<L>(x, w, b, fcams, cam, cam_u8, B, Cin, H, W, argmax, stream);      \
    }                                                                                          \
    extern "C" int tcam_std_cam_##SUF(const void* A, const float* fc_w, const int32_t* cls,     \
                                      float* low, float* cam, uint8_t* cam_u8, int B, int C,   \
                                      int h, int w, int Ho, int Wo, void* stream) {            \
        return std_cam<L>(A, fc_w, cls, low, cam, cam_u8, B, C, h, w, Ho, Wo, stream);         \
    }

TCAM_LAYOUT_ENTRIES(s3, LayS3)
TCAM_LAYOUT_ENTRIES(s2, LayS2)
TCAM_LAYOUT_ENTRIES(s1, LayS1)
