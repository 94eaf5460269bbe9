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
