// Small HBM-bound kernels around the convolutions: stem max-pool, the
// decoder's nearest-x2 + bilinear(align_corners=True) resample, and the WGAP
// classification head.
#include "common.h"

namespace {

// nn.MaxPool2d(kernel_size=3, stride=2, padding=1) (encoders/resnet.py:99).
__global__ void maxpool3x3s2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                    int C, int H, int W, int Ho, int Wo, long total) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int ox = (int)(i % Wo);
    long t = i / Wo;
    int oy = (int)(t % Ho);
    long bc = t / Ho;
    const float* src = in + bc * H * W;
    float m = -INFINITY;
    int y0 = oy * 2 - 1, x0 = ox * 2 - 1;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        int y = y0 + dy;
        if ((unsigned)y >= (unsigned)H) continue;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            int x = x0 + dx;
            if ((unsigned)x >= (unsigned)W) continue;
            float v = src[y * W + x];
            // PyTorch max-pool propagates NaN.
            m = (v > m || v != v) ? v : m;
        }
    }
    out[i] = m;
}

// F.interpolate(x, scale_factor=2, mode="nearest") followed by
// F.interpolate(size=(Ho, Wo), mode="bilinear", align_corners=True)
// (unet/decoder.py:43-51).  The nearest map U has size (2H, 2W) and
// U[y][x] = in[y >> 1][x >> 1].  Bilinear source index follows ATen
// (area_pixel_compute_scale / compute_indices_weights_linear).
__global__ void up2_resize_kernel(const float* __restrict__ in, float* __restrict__ out,
                                  int H, int W, int Ho, int Wo, float sh, float sw,
                                  long total) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int ox = (int)(i % Wo);
    long t = i / Wo;
    int oy = (int)(t % Ho);
    long bc = t / Ho;
    const int Hu = 2 * H, Wu = 2 * W;
    float ry = sh * (float)oy;
    float rx = sw * (float)ox;
    int y0 = (int)ry, x0 = (int)rx;
    int y1 = y0 + (y0 < Hu - 1 ? 1 : 0);
    int x1 = x0 + (x0 < Wu - 1 ? 1 : 0);
    float ly1 = fminf(fmaxf(ry - (float)y0, 0.f), 1.f), ly0 = 1.f - ly1;
    float lx1 = fminf(fmaxf(rx - (float)x0, 0.f), 1.f), lx0 = 1.f - lx1;
    const float* src = in + bc * H * W;
    float v00 = src[(y0 >> 1) * W + (x0 >> 1)];
    float v01 = src[(y0 >> 1) * W + (x1 >> 1)];
    float v10 = src[(y1 >> 1) * W + (x0 >> 1)];
    float v11 = src[(y1 >> 1) * W + (x1 >> 1)];
    out[i] = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
}

// AdaptiveAvgPool2d(1): one wave per (b, c) plane.
__global__ void plane_mean_kernel(const float* __restrict__ x, float* __restrict__ mean,
                                  int HW, long planes) {
    long wid = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    if (wid >= planes) return;
    const float* src = x + wid * HW;
    float s = 0.f;
    for (int i = lane; i < HW; i += 64) s += src[i];
    s = wave_sum(s);
    if (lane == 0) mean[wid] = s / (float)HW;
}

// Linear(C -> classes): one wave per (b, class).
__global__ void linear_kernel(const float* __restrict__ feat, const float* __restrict__ w,
                              const float* __restrict__ bias, float* __restrict__ out,
                              int C, int classes, int B) {
    int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    if (wid >= B * classes) return;
    int b = wid / classes, k = wid % classes;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += feat[(long)b * C + c] * w[(long)k * C + c];
    s = wave_sum(s);
    if (lane == 0) out[wid] = s + bias[k];
}

}  // namespace

extern "C" int tcam_maxpool3x3s2(const float* in, float* out, int B, int C, int H,
                                 int W, int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && H > 0 && W > 0);
    TCAM_REQUIRE(Ho == (H + 2 - 3) / 2 + 1 && Wo == (W + 2 - 3) / 2 + 1);
    long total = (long)B * C * Ho * Wo;
    maxpool3x3s2_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(in, out, C, H, W,
                                                                         Ho, Wo, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_up2_resize(const float* in, float* out, int B, int C, int H, int W,
                               int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(in && out && B > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0);
    // align_corners=True: scale = (in - 1) / (out - 1), 0 for a 1-pixel output.
    float sh = Ho > 1 ? (float)(2 * H - 1) / (float)(Ho - 1) : 0.f;
    float sw = Wo > 1 ? (float)(2 * W - 1) / (float)(Wo - 1) : 0.f;
    long total = (long)B * C * Ho * Wo;
    up2_resize_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(in, out, H, W, Ho, Wo,
                                                                       sh, sw, total);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_wgap(const float* x, const float* fc_w, const float* fc_b,
                         float* logits, float* ws, int B, int C, int HW, int classes,
                         void* stream) {
    TCAM_REQUIRE(x && fc_w && fc_b && logits && ws && B > 0 && C > 0 && HW > 0 && classes > 0);
    hipStream_t st = as_stream(stream);
    long planes = (long)B * C;
    plane_mean_kernel<<<cdiv(planes * 64, 256), 256, 0, st>>>(x, ws, HW, planes);
    TCAM_CHECK_LAUNCH();
    linear_kernel<<<cdiv((long)B * classes * 64, 256), 256, 0, st>>>(ws, fc_w, fc_b, logits, C,
                                                                    classes, B);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
