// Shared helpers for the TCAM gfx950 kernels.  Written for CDNA4 only:
// 64-lane wavefronts, fp32 MFMA, 160 KiB LDS per CU.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tcam_hip.h"

#define TCAM_CHECK_LAUNCH()                         \
    do {                                            \
        hipError_t e_ = hipGetLastError();          \
        if (e_ != hipSuccess) return (int)e_;       \
    } while (0)

#define TCAM_REQUIRE(cond) \
    do {                   \
        if (!(cond)) return TCAM_E_ARG; \
    } while (0)

static inline hipStream_t as_stream(void* s) { return (hipStream_t)s; }

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Launch timing of the convolutions (bench.py's roofline, tcam_timer_arm): the armed events
// are bound to the conv kernels' own dispatches (hipExtLaunchKernelGGL), start to the first
// launch of a call and stop to every launch, so timing adds no marker packets between kernels.
extern hipEvent_t g_timer_start, g_timer_stop;

template <class K, class... A>
static inline void timed_launch(K kern, dim3 grid, dim3 block, hipStream_t st, A... args) {
    hipEvent_t s = g_timer_start;
    g_timer_start = nullptr;
    hipExtLaunchKernelGGL(kern, grid, block, 0, st, s, g_timer_stop, 0, args...);
}

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ReLU with torch's NaN semantics (relu(NaN) = NaN; fmaxf would return 0): a NaN anywhere
// in the forward reaches the loss, as in the reference, so its non-finite-loss skip
// (learning/train_wsol.py:1181) sees it.
__device__ __forceinline__ float relu_nan(float v) { return v < 0.f ? 0.f : v; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
