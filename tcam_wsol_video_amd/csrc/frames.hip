// Frame preprocessing on the device (the data path): the reference's
// eval / train transforms (datasets/wsol_loader.py:903-908 get_eval_tranforms, :960-970
// the train Compose: Resize -> RandomCrop -> RandomHorizontalFlip -> ToTensor ->
// Normalize) for a batch of decoded uint8 RGB frames already in HBM.
//
// Resize is torchvision 0.12's TF.resize on a PIL image = Pillow's Image.resize(size,
// BILINEAR): a separable two-pass fixed-point resample (Pillow src/libImaging/Resample.c,
// precompute_coeffs + normalize_coeffs_8bpc + ImagingResampleHorizontal/Vertical_8bpc):
// per output coordinate a window [xmin, xmin + n) of the triangle filter scaled by
// max(1, in/out), weights normalised in double and rounded to int32 with 22 fraction bits;
// the horizontal pass is stored as uint8 (rounded, clipped), the vertical pass reads it.
// The coefficients are computed once on the host (tcam_resample_coeffs, double arithmetic
// exactly as Pillow's); the kernel does the integer arithmetic, so the resized pixels are
// bit-identical to Pillow's.  ToTensor / Normalize: x / 255.f, then (x - mean) / std in
// fp32 (torchvision's div / sub_ / div_), also bit-identical; raw_img (the CRF input) is the
// resized uint8 as float (wsol_loader.py:603-606).
#include <cmath>
#include <vector>

#include "common.h"

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;  // Pillow's PRECISION_BITS

__device__ __forceinline__ int clip8(int ss) {
    const int v = ss >> kPrecisionBits;  // arithmetic shift: floor, as Pillow's lookup
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

struct FrameArgs {
    const uint8_t* in;      // (B, Hin, Win, 3)
    int Hin, Win;
    const int* bh;          // horizontal bounds (Rw, 2): xmin, n
    const int* kh;          // horizontal weights (Rw, ksh)
    int ksh;
    const int* bv;          // vertical bounds (Rh, 2)
    const int* kv;          // vertical weights (Rh, ksv)
    int ksv;
    const int* crop;        // (B, 2): top, left in the resized frame, or null (0, 0)
    const uint8_t* flip;    // (B,): horizontal flip after the crop, or null
    int B, th, tw;
    float mean[3], stdv[3];
    float* norm;            // (B, 3, th, tw) or null
    float* raw;             // (B, 3, th, tw) or null
    uint8_t* u8;            // (B, th, tw, 3) or null
};

__global__ __launch_bounds__(256) void frames_kernel(FrameArgs a) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long hw = (long)a.th * a.tw;
    if (i >= (long)a.B * hw) return;
    const int b = (int)(i / hw);
    const int r = (int)(i - (long)b * hw);
    const int y = r / a.tw, x = r - y * a.tw;
    const int top = a.crop ? a.crop[2 * b] : 0, left = a.crop ? a.crop[2 * b + 1] : 0;
    const int xx = (a.flip && a.flip[b]) ? a.tw - 1 - x : x;
    const int ry = top + y, rx = left + xx;
    const int ymin = a.bv[2 * ry], yn = a.bv[2 * ry + 1];
    const int xmin = a.bh[2 * rx], xn = a.bh[2 * rx + 1];
    const int* kv = a.kv + (long)ry * a.ksv;
    const int* kh = a.kh + (long)rx * a.ksh;
    const uint8_t* src = a.in + (long)b * a.Hin * a.Win * 3;
    const int half = 1 << (kPrecisionBits - 1);
    int sv0 = half, sv1 = half, sv2 = half;
    for (int t = 0; t < yn; ++t) {
        const uint8_t* row = src + ((long)(ymin + t) * a.Win + xmin) * 3;
        int s0 = half, s1 = half, s2 = half;
        for (int s = 0; s < xn; ++s) {
            const int k = kh[s];
            s0 += (int)row[3 * s] * k;
            s1 += (int)row[3 * s + 1] * k;
            s2 += (int)row[3 * s + 2] * k;
        }
        // the horizontal pass is an 8-bit image in Pillow
        const int k = kv[t];
        sv0 += clip8(s0) * k;
        sv1 += clip8(s1) * k;
        sv2 += clip8(s2) * k;
    }
    const int v[3] = {clip8(sv0), clip8(sv1), clip8(sv2)};
    if (a.u8) {
        uint8_t* o = a.u8 + i * 3;
        o[0] = (uint8_t)v[0];
        o[1] = (uint8_t)v[1];
        o[2] = (uint8_t)v[2];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma clang fp contract(off)
        const long o = ((long)b * 3 + c) * hw + r;
        if (a.raw) a.raw[o] = (float)v[c];
        if (a.norm) a.norm[o] = ((float)v[c] / 255.0f - a.mean[c]) / a.stdv[c];
    }
}

double bilinear_filter(double x) {
    if (x < 0.0) x = -x;
    if (x < 1.0) return 1.0 - x;
    return 0.0;
}

}  // namespace

// Pillow's precompute_coeffs (BILINEAR, support 1, box = [0, in_size)) followed by
// normalize_coeffs_8bpc.  bounds: (out_size, 2) = (xmin, n); kk: (out_size, ksize) int32,
// zero past n.  Returns ksize, or a negative error code; with kk == NULL only ksize.
extern "C" int tcam_resample_coeffs(int in_size, int out_size, int* bounds, int* kk) {
    if (in_size <= 0 || out_size <= 0) return TCAM_E_ARG;
    const float in0 = 0.f, in1 = (float)in_size;
    double scale = (double)(in1 - in0) / out_size;
    double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * filterscale;
    const int ksize = (int)std::ceil(support) * 2 + 1;
    if (!bounds || !kk) return ksize;
    std::vector<double> k(ksize);
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        int x = 0;
        for (; x < xmax; ++x) {
            const double w = bilinear_filter((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; ++x) k[x] = 0;
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = xmax;
        for (x = 0; x < ksize; ++x) {
            const double v = k[x] * (1 << kPrecisionBits);
            kk[(long)xx * ksize + x] = k[x] < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
        }
    }
    return ksize;
}

extern "C" int tcam_frames_preprocess(const uint8_t* frames, int B, int Hin, int Win,
                                      const int* bh, const int* kh, int ksh, int Rw,
                                      const int* bv, const int* kv, int ksv, int Rh,
                                      const int* crop, const uint8_t* flip, int th, int tw,
                                      const float* mean3, const float* std3, float* norm,
                                      float* raw, uint8_t* u8, void* stream) {
    TCAM_REQUIRE(frames && B > 0 && Hin > 0 && Win > 0 && bh && kh && bv && kv);
    TCAM_REQUIRE(ksh > 0 && ksv > 0 && th > 0 && tw > 0 && th <= Rh && tw <= Rw);
    TCAM_REQUIRE(norm || raw || u8);
    TCAM_REQUIRE(!norm || (mean3 && std3));
    FrameArgs a{};
    a.in = frames;
    a.Hin = Hin;
    a.Win = Win;
    a.bh = bh;
    a.kh = kh;
    a.ksh = ksh;
    a.bv = bv;
    a.kv = kv;
    a.ksv = ksv;
    a.crop = crop;
    a.flip = flip;
    a.B = B;
    a.th = th;
    a.tw = tw;
    for (int c = 0; c < 3; ++c) {
        a.mean[c] = mean3 ? mean3[c] : 0.f;
        a.stdv[c] = std3 ? std3[c] : 1.f;
    }
    a.norm = norm;
    a.raw = raw;
    a.u8 = u8;
    const long n = (long)B * th * tw;
    frames_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(a);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
