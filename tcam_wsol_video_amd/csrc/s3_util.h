// S3-layout helpers shared by the S3 kernels (s3.hip, train.hip): a group of 8
// channels is 48 bytes [hi x8][mid x8][lo x8] bf16, value = (hi + mid) + lo exactly.
#pragma once
#include "common.h"

namespace s3 {

struct G8 {
    float v[8];
};

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// 48-byte group at p -> 8 fp32 values
__device__ __forceinline__ G8 load_g8(const uint8_t* p) {
    const uint4 h = *reinterpret_cast<const uint4*>(p);
    const uint4 m = *reinterpret_cast<const uint4*>(p + 16);
    const uint4 l = *reinterpret_cast<const uint4*>(p + 32);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, mw[4] = {m.x, m.y, m.z, m.w},
                   lw[4] = {l.x, l.y, l.z, l.w};
    G8 g;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        g.v[2 * i] = (bf_lo(hw[i]) + bf_lo(mw[i])) + bf_lo(lw[i]);
        g.v[2 * i + 1] = (bf_hi(hw[i]) + bf_hi(mw[i])) + bf_hi(lw[i]);
    }
    return g;
}

__device__ __forceinline__ uint32_t bfbits(float x) {
    return __builtin_bit_cast(uint16_t, (__bf16)x);
}

// split 8 fp32 into the 48-byte group at p (x = hi + mid + lo exactly)
__device__ __forceinline__ void store_g8(uint8_t* p, const G8& g) {
    uint32_t hw[4], mw[4], lw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t hh[2], mm[2], ll[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float x = g.v[2 * i + e];
            hh[e] = bfbits(x);
            const float r1 = x - __uint_as_float(hh[e] << 16);
            mm[e] = bfbits(r1);
            ll[e] = bfbits(r1 - __uint_as_float(mm[e] << 16));
        }
        hw[i] = hh[0] | (hh[1] << 16);
        mw[i] = mm[0] | (mm[1] << 16);
        lw[i] = ll[0] | (ll[1] << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    *reinterpret_cast<uint4*>(p + 16) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
    *reinterpret_cast<uint4*>(p + 32) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}


}  // namespace s3

// S2 layout (the f16x3 inference path, conv_x6.hip FmtF16): a group of 8 channels is
// 32 bytes [h x8][l x8] fp16, value = h + l (h = rne_f16(x), l = rne_f16(x - h): 11 + 11
// significand bits; |x| <= 65504, see include/tcam_hip.h).
namespace s2 {

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float h_lo(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
}
__device__ __forceinline__ float h_hi(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
}
__device__ __forceinline__ uint32_t hbits(float x) {
    return __builtin_bit_cast(uint16_t, (_Float16)x);
}

// x = h + l (two fp16 bit patterns)
__device__ __forceinline__ void split2(float x, uint32_t& h, uint32_t& l) {
    const _Float16 hh = (_Float16)x;
    h = __builtin_bit_cast(uint16_t, hh);
    l = hbits(x - (float)hh);
}

__device__ __forceinline__ s3::G8 load_g8(const uint8_t* p) {
    const uint4 h = *reinterpret_cast<const uint4*>(p);
    const uint4 l = *reinterpret_cast<const uint4*>(p + 16);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, lw[4] = {l.x, l.y, l.z, l.w};
    s3::G8 g;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        g.v[2 * i] = h_lo(hw[i]) + h_lo(lw[i]);
        g.v[2 * i + 1] = h_hi(hw[i]) + h_hi(lw[i]);
    }
    return g;
}

__device__ __forceinline__ void store_g8(uint8_t* p, const s3::G8& g) {
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t hh[2], ll[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) split2(g.v[2 * i + e], hh[e], ll[e]);
        hw[i] = hh[0] | (hh[1] << 16);
        lw[i] = ll[0] | (ll[1] << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    *reinterpret_cast<uint4*>(p + 16) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

}  // namespace s2

// S1 layout (the AMP training path, conv_x6.hip FmtH1): a group of 8 channels is 16 bytes
// [h x8] fp16 — autocast's fp16 activation (h = rne_f16(x); beyond 65504 -> inf, which the
// loss scaler's non-finite check catches, as torch.cuda.amp.GradScaler does).
namespace s1 {

__device__ __forceinline__ s3::G8 load_g8(const uint8_t* p) {
    const uint4 h = *reinterpret_cast<const uint4*>(p);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
    s3::G8 g;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        g.v[2 * i] = s2::h_lo(hw[i]);
        g.v[2 * i + 1] = s2::h_hi(hw[i]);
    }
    return g;
}

__device__ __forceinline__ void store_g8(uint8_t* p, const s3::G8& g) {
    uint32_t hw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) hw[i] = s2::hbits(g.v[2 * i]) | (s2::hbits(g.v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
}

}  // namespace s1

// Layout traits for the kernels written once over both activation layouts.
struct LayS3 {
    static constexpr int GB = 48;
    static __device__ __forceinline__ s3::G8 load(const uint8_t* p) { return s3::load_g8(p); }
    static __device__ __forceinline__ void store(uint8_t* p, const s3::G8& g) { s3::store_g8(p, g); }
};
struct LayS2 {
    static constexpr int GB = 32;
    static __device__ __forceinline__ s3::G8 load(const uint8_t* p) { return s2::load_g8(p); }
    static __device__ __forceinline__ void store(uint8_t* p, const s3::G8& g) { s2::store_g8(p, g); }
};
struct LayS1 {
    static constexpr int GB = 16;
    static __device__ __forceinline__ s3::G8 load(const uint8_t* p) { return s1::load_g8(p); }
    static __device__ __forceinline__ void store(uint8_t* p, const s3::G8& g) { s1::store_g8(p, g); }
};
