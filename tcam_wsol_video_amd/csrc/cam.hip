// CAM kernels: the TCAM segmentation head fused with SegmentationCam and the
// eval-time uint8 quantisation, the STD_CL CAM (weighted sum of the hooked
// layer4 activations + min-max normalise + bilinear resize), the temporal
// max over neighbour-frame CAMs, and the top-1/top-5 rank of the target.
#include "common.h"

namespace {

// conv3x3(Cin -> 2, pad 1, bias) -> softmax(dim=1)[:, 1] (or argmax) ->
// nan_to_num -> uint8(cam * 255).
//   base/heads.py:19-36; cams/builtincam.py:201-225;
//   learning/inference_wsol.py:323 (nan_to_num), wsol_metrics.py:153 (u8).
// One thread per output pixel; weights in LDS.  HBM traffic per pixel:
// Cin*4 B read (taps re-read through L1/L2) + (8 + 4 + 1) B written.
constexpr int SEG_MAX_CIN = 64;
__global__ void seghead_cam_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                   const float* __restrict__ bias, float* __restrict__ fcams,
                                   float* __restrict__ cam, uint8_t* __restrict__ cam_u8,
                                   int Cin, int H, int W, long total, int argmax) {
    __shared__ float ws[2 * SEG_MAX_CIN * 9];
    for (int i = threadIdx.x; i < 2 * Cin * 9; i += blockDim.x) ws[i] = w[i];
    __syncthreads();
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int HW = H * W;
    int px = (int)(i % W);
    long t = i / W;
    int py = (int)(t % H);
    long b = t / H;
    const float* xb = x + b * Cin * HW;
    float a0 = 0.f, a1 = 0.f;
    for (int c = 0; c < Cin; ++c) {
        const float* xc = xb + (long)c * HW;
        const float* w0 = ws + c * 9;
        const float* w1 = ws + (Cin + c) * 9;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            int y = py + kh - 1;
            if ((unsigned)y >= (unsigned)H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                int xx = px + kw - 1;
                if ((unsigned)xx >= (unsigned)W) continue;
                float v = xc[y * W + xx];
                a0 = fmaf(w0[kh * 3 + kw], v, a0);
                a1 = fmaf(w1[kh * 3 + kw], v, a1);
            }
        }
    }
    a0 += bias[0];
    a1 += bias[1];
    const long pix = (long)py * W + px;
    if (fcams) {
        fcams[(b * 2 + 0) * HW + pix] = a0;
        fcams[(b * 2 + 1) * HW + pix] = a1;
    }
    float c1;
    if (argmax) {
        c1 = (a1 > a0) ? 1.f : 0.f;  // torch.argmax: first max wins ties
    } else {
        float m = fmaxf(a0, a1);
        float e0 = expf(a0 - m), e1 = expf(a1 - m);
        c1 = e1 / (e0 + e1);
    }
    if (c1 != c1) c1 = 0.f;  // nan_to_num(nan=0, posinf=1, neginf=0)
    if (isinf(c1)) c1 = c1 > 0.f ? 1.f : 0.f;
    if (cam) cam[b * HW + pix] = c1;
    if (cam_u8) cam_u8[b * HW + pix] = (uint8_t)(int)((double)c1 * 255.0);
}

// STD_CL CAM, one workgroup per frame.
//   low = nansum_c w[cls, c] * A[c]          (cams/core.py:176-182)
//   low = (low - min) / max(low - min)       (core.py:105-111, in place)
//   nan_to_num                                (inference_wsol.py:323)
//   cam = bilinear(low -> Ho x Wo, align_corners=False) (inference_wsol.py:342-346)
constexpr int STD_MAX_HW = 4096;
__global__ __launch_bounds__(1024) void std_cam_kernel(
    const float* __restrict__ A, const float* __restrict__ fcw, const int32_t* __restrict__ cls,
    float* __restrict__ low_out, float* __restrict__ cam, uint8_t* __restrict__ cam_u8, int C,
    int h, int w, int Ho, int Wo) {
    __shared__ float low[STD_MAX_HW];
    __shared__ float red[32];
    const int b = blockIdx.x;
    const int hw = h * w;
    const float* Ab = A + (long)b * C * hw;
    const float* wr = fcw + (long)cls[b] * C;
    for (int p = threadIdx.x; p < hw; p += blockDim.x) {
        float s = 0.f;
        for (int c = 0; c < C; ++c) {
            float v = wr[c] * Ab[(long)c * hw + p];
            if (v == v) s += v;  // nansum
        }
        low[p] = s;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
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
        float v = low[p] - mn;
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
    // align_corners=False: src = scale * (dst + 0.5) - 0.5, clamped at 0.
    const float sh = (float)h / (float)Ho, sw = (float)w / (float)Wo;
    for (int p = threadIdx.x; p < Ho * Wo; p += blockDim.x) {
        int oy = p / Wo, ox = p % Wo;
        float ry = fmaxf(sh * ((float)oy + 0.5f) - 0.5f, 0.f);
        float rx = fmaxf(sw * ((float)ox + 0.5f) - 0.5f, 0.f);
        int y0 = (int)ry, x0 = (int)rx;
        int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
        float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
        float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
        float v = ly0 * (lx0 * low[y0 * w + x0] + lx1 * low[y0 * w + x1]) +
                  ly1 * (lx0 * low[y1 * w + x0] + lx1 * low[y1 * w + x1]);
        if (cam) cam[(long)b * Ho * Wo + p] = v;
        if (cam_u8) cam_u8[(long)b * Ho * Wo + p] = (uint8_t)(int)((double)v * 255.0);
    }
}

// Temporal max over neighbour-frame CAMs, one workgroup per output.
//   datasets/wsol_loader.py:591-601 (torch.maximum accumulation, NaN-propagating)
//   wsol_loader.py:630-635 re_normalize_cam(cam, h=t): exp(t (c + 1e-6)) / max.
constexpr int TMP_MAX_HW = 8192;
__global__ __launch_bounds__(256) void temporal_max_kernel(const float* __restrict__ cams,
                                                           const int32_t* __restrict__ idx,
                                                           float* __restrict__ out, int k1,
                                                           int hw, float t) {
    __shared__ float red[4];
    const int o = blockIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float* dst = out + (long)o * hw;
    bool first = true;
    for (int j = 0; j < k1; ++j) {
        int f = idx[o * k1 + j];
        if (f < 0) continue;
        const float* src = cams + (long)f * hw;
        float scale = 1.f;
        if (t > 0.f) {
            float mx = -INFINITY;
            for (int p = threadIdx.x; p < hw; p += blockDim.x)
                mx = fmaxf(mx, expf((src[p] + 1e-6f) * t));
            mx = wave_max(mx);
            if (lane == 0) red[wid] = mx;
            __syncthreads();
            mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
            __syncthreads();
            scale = mx;
        }
        for (int p = threadIdx.x; p < hw; p += blockDim.x) {
            float v = src[p];
            if (t > 0.f) {
                v = expf((v + 1e-6f) * t) / scale;
                if (v != v) v = 0.f;
                if (isinf(v)) v = v > 0.f ? 1.f : 0.f;
            }
            if (first) {
                dst[p] = v;
            } else {
                float a = dst[p];
                dst[p] = (a != a || v != v) ? NAN : fmaxf(a, v);
            }
        }
        first = false;
        __syncthreads();
    }
}

// Full-resolution temporal CAM (CAM-TMP over a sharded clip, BASELINE configs[4]).
// Same arithmetic as temporal_max_kernel, laid out for big frames: the
// re_normalize_cam denominators max_p exp(t (c_f[p] + 1e-6)) are computed once per
// source frame (frame_expmax_kernel), then a 2-D grid (pixel chunk, output frame)
// streams the k+1 source frames with 16-byte loads and writes the fp32 CAM and its
// uint8(double(cam) * 255) quantisation (wsol_metrics.py:153) in one pass.
// HBM bytes per output pixel: 4 (k1 reads, mostly L2 hits for neighbours) + 5 written.
__global__ __launch_bounds__(1024) void frame_expmax_kernel(const float* __restrict__ cams,
                                                            float* __restrict__ scale, int hw,
                                                            float t) {
    __shared__ float red[16];
    const float* src = cams + (long)blockIdx.x * hw;
    float mx = -INFINITY;
    for (int p = threadIdx.x; p < hw; p += blockDim.x) mx = fmaxf(mx, expf((src[p] + 1e-6f) * t));
    mx = wave_max(mx);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = red[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
        scale[blockIdx.x] = m;
    }
}

__device__ __forceinline__ float renorm_cam(float v, float t, float s) {
    v = expf((v + 1e-6f) * t) / s;
    if (v != v) v = 0.f;
    if (isinf(v)) v = v > 0.f ? 1.f : 0.f;
    return v;
}

__global__ __launch_bounds__(256) void temporal_cam_kernel(
    const float* __restrict__ cams, const int32_t* __restrict__ idx,
    const float* __restrict__ scale, float* __restrict__ out, uint8_t* __restrict__ out_u8,
    int N, int k1, int hw, float t) {
    const int o = blockIdx.y;
    const long p0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (p0 >= hw) return;
    const bool vec = (hw & 3) == 0 && p0 + 4 <= hw;
    float acc[4];
    bool first = true;
    for (int j = 0; j < k1; ++j) {
        const int f = idx[o * k1 + j];
        if (f < 0 || f >= N) continue;   // absent neighbour (or out of range: ignored)
        const float* src = cams + (long)f * hw;
        float v[4];
        if (vec) {
            float4 q = *reinterpret_cast<const float4*>(src + p0);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = p0 + i < hw ? src[p0 + i] : 0.f;
        }
        if (t > 0.f) {
            const float s = scale[f];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = renorm_cam(v[i], t, s);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc[i] = first ? v[i] : ((acc[i] != acc[i] || v[i] != v[i]) ? NAN : fmaxf(acc[i], v[i]));
        first = false;
    }
    float a[4];
    uint32_t u = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = first ? 0.f : acc[i];
        const uint32_t q = a[i] == a[i] ? (uint32_t)(uint8_t)(int)((double)a[i] * 255.0) : 0u;
        u |= q << (8 * i);
    }
    float* dst = out ? out + (long)o * hw + p0 : nullptr;
    uint8_t* du = out_u8 ? out_u8 + (long)o * hw + p0 : nullptr;
    if (vec) {
        if (dst) *reinterpret_cast<float4*>(dst) = make_float4(a[0], a[1], a[2], a[3]);
        if (du) *reinterpret_cast<uint32_t*>(du) = u;
    } else {
        for (int i = 0; i < 4 && p0 + i < hw; ++i) {
            if (dst) dst[i] = a[i];
            if (du) du[i] = (uint8_t)(u >> (8 * i));
        }
    }
}

// preds_ordered = torch.sort(logits, descending=True, stable=True)
// (inference_wsol.py:368-369); top1 = target == preds[0], top5 = target in preds[:5].
__global__ void topk_kernel(const float* __restrict__ logits, const int32_t* __restrict__ target,
                            int32_t* __restrict__ top1, int32_t* __restrict__ top5, int B,
                            int C) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int t = target[b];
    const float* l = logits + (long)b * C;
    float lt = l[t];
    int rank = 0;
    for (int c = 0; c < C; ++c) rank += (l[c] > lt) || (l[c] == lt && c < t);
    top1[b] = rank == 0;
    top5[b] = rank < 5;
}

}  // namespace

extern "C" int tcam_seghead_cam(const float* x, const float* w, const float* b, float* fcams,
                                float* cam, uint8_t* cam_u8, int B, int Cin, int H, int W,
                                int argmax, void* stream) {
    TCAM_REQUIRE(x && w && b && B > 0 && Cin > 0 && Cin <= SEG_MAX_CIN && H > 0 && W > 0);
    long total = (long)B * H * W;
    seghead_cam_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        x, w, b, fcams, cam, cam_u8, Cin, H, W, total, argmax);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_std_cam(const float* A, const float* fc_w, const int32_t* cls, float* low,
                            float* cam, uint8_t* cam_u8, int B, int C, int h, int w, int Ho,
                            int Wo, void* stream) {
    TCAM_REQUIRE(A && fc_w && cls && B > 0 && C > 0 && h > 0 && w > 0 && h * w <= STD_MAX_HW);
    TCAM_REQUIRE(Ho > 0 && Wo > 0);
    std_cam_kernel<<<B, 1024, 0, as_stream(stream)>>>(A, fc_w, cls, low, cam, cam_u8, C, h, w,
                                                      Ho, Wo);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_temporal_max(const float* cams, const int32_t* idx, float* out, int M,
                                 int k1, int hw, float t, void* stream) {
    TCAM_REQUIRE(cams && idx && out && M > 0 && k1 > 0 && hw > 0);
    temporal_max_kernel<<<M, 256, 0, as_stream(stream)>>>(cams, idx, out, k1, hw, t);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_temporal_cam(const float* cams, int N, const int32_t* idx, float* out,
                                 uint8_t* out_u8, int M, int k1, int hw, float t, float* scale_ws,
                                 void* stream) {
    TCAM_REQUIRE(cams && idx && (out || out_u8) && N > 0 && M > 0 && k1 > 0 && hw > 0);
    TCAM_REQUIRE(!(t > 0.f) || scale_ws);
    hipStream_t s = as_stream(stream);
    if (t > 0.f) {
        frame_expmax_kernel<<<N, 1024, 0, s>>>(cams, scale_ws, hw, t);
        TCAM_CHECK_LAUNCH();
    }
    dim3 grid((unsigned)cdiv((long)hw, 1024), (unsigned)M);
    temporal_cam_kernel<<<grid, 256, 0, s>>>(cams, idx, t > 0.f ? scale_ws : nullptr, out,
                                             out_u8, N, k1, hw, t);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_topk_flags(const float* logits, const int32_t* target, int32_t* top1,
                               int32_t* top5, int B, int C, void* stream) {
    TCAM_REQUIRE(logits && target && top1 && top5 && B > 0 && C > 0);
    topk_kernel<<<cdiv(B, 256), 256, 0, as_stream(stream)>>>(logits, target, top1, top5, B, C);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
