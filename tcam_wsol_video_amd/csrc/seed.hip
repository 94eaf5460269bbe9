// TCAM pseudo-label seeding on gfx950: one 1024-thread workgroup per frame.
//
// Replaces the per-sample Python loop of
//   TCAMSeeder.forward               dlib/cams/tcam_seeding.py:187-258
//   _OneSample / _SFG / _SBG         tcam_seeding.py:409-563
//   GetRoiSingleCam.__call__ / get_thresh (skimage 0.17.2 Otsu, measure.label)
//                                    tcam_seeding.py:303-406
// and kornia 0.6.4 erosion / dilation (all-ones kernel, geodesic border).
//
// Every per-pixel set (blobs, ROI, candidates, seeds) lives in LDS as a bitmap
// built 64 pixels at a time with one wave ballot; the cam stays in HBM/L2 and is
// streamed once per pass.  Order statistics are block radix selects:
//   * the stable top-n of torch.sort (ties -> lower raster index first) =
//     the n-th largest orderable key T, every key > T, then the first
//     (n - #{> T}) keys == T in raster order (word popcount scan);
//   * multinomial(p, k, replacement=False) = topk(p / q, k), q ~ Exp(1)
//     (torch's no-replacement path), with q from a counter-based Philox4x32-10
//     keyed by (pixel, frame, offset; seed) — reproducible per (seed, offset).
// 4-connected labelling (ROI_LARGEST / ROI_H_DENSITY) is a lock-free union-find
// (atomicMin, root = smallest raster index = skimage's label order) in a
// per-frame int32 workspace.
// All float arithmetic restating numpy / torch runs with contraction off.
#pragma clang fp contract(off)

#include "common.h"

namespace {

constexpr int SEED_THREADS = 1024;
constexpr int SEED_WAVES = SEED_THREADS / 64;
constexpr int SEED_MAX_HW = 320 * 320;
constexpr int N_BITMAPS = 6;

enum { BM_ROI = 0, BM_A, BM_B, BM_FG, BM_BG, BM_T };

struct SeedArgs {
    const float* cam;        // (B, HW) fp32
    const uint8_t* roi_in;   // (B, HW) 0/1 or NULL
    int32_t* seeds;          // (B, HW) or NULL
    uint8_t* roi_out;        // (B, HW) or NULL
    float* th_out;           // (B,) or NULL
    int32_t* bbox_out;       // (B, 4) or NULL
    int32_t* ws_label;       // (B, HW)
    int32_t* ws_area;        // (B, HW)
    unsigned long long* ws_key;  // (B, HW): fixed-point cam sums, then sample keys
    int H, W;
    int seed_tech;           // 0 uniform, 1 weighted
    int min_, max_;
    float max_p, min_p;
    int fg_erode_k, fg_erode_iter, ksz;
    int ignore_idx;
    int roi_method;          // 0 all, 1 high density, 2 largest
    double p_min_area_roi;
    int use_roi;
    double thresh;           // < 0: Otsu; else GetRoiSingleCam(thresh=...)
    const double* thresh_b;  // (B,) per-frame thresholds (< 0 or NaN: Otsu) or NULL
    unsigned long long seed, offset;
    int roi_only;            // 1: GetRoiSingleCam (no flat-frame exit, no seeds)
};

struct Smem {
    int hist[256];
    double w1[256], w2[256], c1[256], c2[256];
    float edges[257];
    int wi[SEED_WAVES];
    unsigned long long wu[SEED_WAVES];
    double wd[SEED_WAVES];
    float wf[SEED_WAVES * 2];
    int scan[SEED_WAVES];
    int bcast_i[4];
    unsigned long long bcast_u[2];
    float bcast_f[2];
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint32_t get_bit(const uint32_t* bm, int p) {
    return (bm[p >> 5] >> (p & 31)) & 1u;
}

__device__ __forceinline__ int ld_label(const int32_t* L, int p) {
    return __hip_atomic_load(L + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int ld_i32(const int32_t* P, int p) {
    return __hip_atomic_load(P + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_u64(const unsigned long long* P, int p) {
    return __hip_atomic_load(P + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Build a bitmap 64 pixels per wave-iteration from a predicate (no atomics).
template <class F>
__device__ __forceinline__ void build_bitmap(uint32_t* bm, int HW, F pred) {
    for (int base = wave_id() * 64; base < HW; base += SEED_THREADS) {
        int p = base + lane_id();
        bool v = (p < HW) && pred(p);
        unsigned long long m = __ballot(v);
        if (lane_id() == 0) {
            bm[base >> 5] = (uint32_t)m;
            bm[(base >> 5) + 1] = (uint32_t)(m >> 32);
        }
    }
}

__device__ int block_sum_i(Smem& s, int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane_id() == 0) s.wi[wave_id()] = v;
    __syncthreads();
    int t = 0;
    for (int i = 0; i < SEED_WAVES; ++i) t += s.wi[i];
    return t;
}

__device__ unsigned long long block_max_u64(Smem& s, unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    __syncthreads();
    if (lane_id() == 0) s.wu[wave_id()] = v;
    __syncthreads();
    unsigned long long t = 0;
    for (int i = 0; i < SEED_WAVES; ++i) t = s.wu[i] > t ? s.wu[i] : t;
    return t;
}

__device__ unsigned long long block_min_u64(Smem& s, unsigned long long v) {
    return ~block_max_u64(s, ~v);
}

// (max key, then min index) over doubles >= 0 / indices; returns the index (-1: none).
__device__ int block_argmax_d(Smem& s, double key, int idx) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        double k2 = __shfl_xor(key, o, 64);
        int i2 = __shfl_xor(idx, o, 64);
        if (k2 > key || (k2 == key && (unsigned)i2 < (unsigned)idx)) {
            key = k2;
            idx = i2;
        }
    }
    __syncthreads();
    if (lane_id() == 0) {
        s.wd[wave_id()] = key;
        s.wi[wave_id()] = idx;
    }
    __syncthreads();
    double bk = s.wd[0];
    int bi = s.wi[0];
    for (int i = 1; i < SEED_WAVES; ++i) {
        if (s.wd[i] > bk || (s.wd[i] == bk && (unsigned)s.wi[i] < (unsigned)bi)) {
            bk = s.wd[i];
            bi = s.wi[i];
        }
    }
    return bi;
}

// Exclusive block scan of one int per thread.
__device__ int block_exscan(Smem& s, int v, int* total) {
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane_id() >= o) x += y;
    }
    __syncthreads();
    if (lane_id() == 63) s.scan[wave_id()] = x;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int i = 0; i < SEED_WAVES; ++i) {
        if (i < wave_id()) pre += s.scan[i];
        tot += s.scan[i];
    }
    *total = tot;
    return pre + x - v;
}

// dst |= the first m set bits (raster order) of src (words 0..NW).
__device__ void take_first_bits(Smem& s, uint32_t* dst, const uint32_t* src, int NW, int m) {
    const int per = (NW + SEED_THREADS - 1) / SEED_THREADS;
    const int w0 = threadIdx.x * per;
    int cnt = 0;
    for (int j = 0; j < per; ++j)
        if (w0 + j < NW) cnt += __popc(src[w0 + j]);
    int tot;
    int pre = block_exscan(s, cnt, &tot);
    for (int j = 0; j < per; ++j) {
        int w = w0 + j;
        if (w >= NW) break;
        uint32_t bits = src[w];
        int c = __popc(bits);
        if (pre >= m) break;
        if (pre + c > m) {
            uint32_t keep = 0;
            for (int r = m - pre; r > 0; --r) {
                uint32_t low = bits & (0u - bits);
                keep |= low;
                bits ^= low;
            }
            bits = keep;
            c = m - pre;
        }
        dst[w] |= bits;
        pre += c;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t ord32(float f) {
    uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Histogram add of an 8-bit digit; one LDS add per wave when the active lanes agree.
__device__ __forceinline__ void hist_add(int* hist, bool act, int digit) {
    unsigned long long am = __ballot(act);
    if (am == 0) return;
    int lead = __shfl(digit, __ffsll((long long)am) - 1, 64);
    unsigned long long same = __ballot(act && digit == lead);
    if (same == am) {
        if (lane_id() == __ffsll((long long)am) - 1) atomicAdd(&hist[lead], __popcll(am));
    } else if (act) {
        atomicAdd(&hist[digit], 1);
    }
}

// dst = the n largest keys (desc, ties -> lower raster index first).
// key(p) returns (active, orderable key).  Keys are 32- or 64-bit.
template <typename K, class F>
__device__ void select_top(Smem& s, uint32_t* dst, uint32_t* tmp, int HW, int NW, int n,
                           F key) {
    constexpr int NB = sizeof(K) * 8;
    K prefix = 0, himask = 0;
    int remaining = n;
    for (int shift = NB - 8; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += SEED_THREADS) s.hist[i] = 0;
        __syncthreads();
        for (int base = wave_id() * 64; base < HW; base += SEED_THREADS) {
            int p = base + lane_id();
            bool act = false;
            K k = 0;
            if (p < HW) act = key(p, k);
            act = act && ((k & himask) == prefix);
            hist_add(s.hist, act, (int)((k >> shift) & 0xFF));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int cum = 0, d = 255;
            for (; d > 0; --d) {
                if (cum + s.hist[d] >= remaining) break;
                cum += s.hist[d];
            }
            s.bcast_i[0] = d;
            s.bcast_i[1] = remaining - cum;
        }
        __syncthreads();
        prefix |= (K)s.bcast_i[0] << shift;
        himask |= (K)0xFF << shift;
        remaining = s.bcast_i[1];
        __syncthreads();
    }
    const K T = prefix;
    build_bitmap(dst, HW, [&](int p) {
        K k = 0;
        return key(p, k) && k > T;
    });
    build_bitmap(tmp, HW, [&](int p) {
        K k = 0;
        return key(p, k) && k == T;
    });
    __syncthreads();
    take_first_bits(s, dst, tmp, NW, remaining);
}

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        unsigned long long p0 = (unsigned long long)0xD2511F53u * c[0];
        unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// q ~ Exp(1) for (frame, pixel), Philox lane `lane` (0 fg, 1 bg).
__device__ __forceinline__ double exp_noise(const SeedArgs& a, int frame, int p, int lane) {
    uint32_t c[4] = {(uint32_t)p, (uint32_t)frame, (uint32_t)a.offset,
                     (uint32_t)(a.offset >> 32)};
    philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    double u = ((double)c[lane] + 0.5) * 2.3283064365386963e-10;  // 2^-32
    return -log(u);
}

// Draw k of the candidate pixels in `cand` with probabilities prob(p):
// topk(prob / q) (multinomial without replacement), ties -> lower raster index.
template <class P>
__device__ void sample(Smem& s, const SeedArgs& a, int frame, int lane, uint32_t* dst,
                       const uint32_t* cand, uint32_t* tmp, int HW, int NW, int n, int k,
                       unsigned long long* keys, P prob) {
    if (k >= n) {  // every candidate is drawn
        for (int w = threadIdx.x; w < NW; w += SEED_THREADS) dst[w] = cand[w];
        __syncthreads();
        return;
    }
    if (k == 1) {
        double best = -1.0;
        int bi = -1;
        for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
            if (!get_bit(cand, p)) continue;
            double key = (double)prob(p) / exp_noise(a, frame, p, lane);
            if (key > best) {
                best = key;
                bi = p;
            }
        }
        int sel = block_argmax_d(s, best, bi);
        for (int w = threadIdx.x; w < NW; w += SEED_THREADS) dst[w] = 0;
        __syncthreads();
        if (threadIdx.x == 0 && sel >= 0) dst[sel >> 5] |= 1u << (sel & 31);
        __syncthreads();
        return;
    }
    for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
        unsigned long long kb = 0;
        if (get_bit(cand, p)) {
            double key = (double)prob(p) / exp_noise(a, frame, p, lane);
            kb = (unsigned long long)__double_as_longlong(key);  // > 0: bit order = value order
        }
        keys[p] = kb;
    }
    __syncthreads();
    select_top<unsigned long long>(s, dst, tmp, HW, NW, k,
                                   [&](int p, unsigned long long& kk) {
                                       kk = ld_u64(keys, p);
                                       return kk != 0ull;
                                   });
}

// Separable geodesic morphology with a k x k all-ones kernel, origin (k/2, k/2):
// dst(y,x) = OP over rows [y-o, y-o+k-1] x cols [x-o, x-o+k-1] inside the image.
__device__ void morph(uint32_t* dst, uint32_t* tmp, const uint32_t* src, int H, int W, int k,
                      bool dilate) {
    const int HW = H * W, o = k / 2;
    build_bitmap(tmp, HW, [&](int p) {
        int y = p / W, x = p - y * W;
        int c0 = max(0, x - o), c1 = min(W - 1, x - o + k - 1);
        for (int c = c0; c <= c1; ++c) {
            uint32_t b = get_bit(src, y * W + c);
            if (dilate ? b : !b) return dilate;
        }
        return !dilate;
    });
    __syncthreads();
    build_bitmap(dst, HW, [&](int p) {
        int y = p / W, x = p - y * W;
        int r0 = max(0, y - o), r1 = min(H - 1, y - o + k - 1);
        for (int r = r0; r <= r1; ++r) {
            uint32_t b = get_bit(tmp, r * W + x);
            if (dilate ? b : !b) return dilate;
        }
        return !dilate;
    });
    __syncthreads();
}

__device__ int uf_find(const int32_t* L, int p) {
    int q = ld_label(L, p);
    while (q != p) {
        p = q;
        q = ld_label(L, p);
    }
    return p;
}

__device__ void uf_unite(int32_t* L, int a, int b) {
    a = uf_find(L, a);
    b = uf_find(L, b);
    while (a != b) {
        if (a < b) {
            int t = a;
            a = b;
            b = t;
        }
        int old = atomicMin(L + a, b);
        if (old == a) break;
        a = uf_find(L, old);
        b = uf_find(L, b);
    }
}

// skimage threshold_otsu(floor(cam*255)) as get_thresh (tcam_seeding.py:399-406):
// numpy 1.21.5 np.histogram(float32 image, 256 bins over [min, max]).
__device__ float otsu(Smem& s, const float* cam, int HW, float cmin, float cmax) {
    const float mn = floorf(cmin * 255.f), mx = floorf(cmax * 255.f);
    if (mn == mx) return 0.f;
    const double dmn = (double)mn, dmx = (double)mx;
    const double step = (dmx - dmn) / 256.0;
    for (int i = threadIdx.x; i <= 256; i += SEED_THREADS)
        s.edges[i] = (i == 256) ? mx : (float)((double)i * step + dmn);
    for (int i = threadIdx.x; i < 256; i += SEED_THREADS) s.hist[i] = 0;
    const float norm = (float)(256.0 / (dmx - dmn));
    __syncthreads();
    for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
        float v = floorf(cam[p] * 255.f);
        float f = (v - mn) * norm;
        int idx = (int)f;
        if (idx == 256) idx = 255;
        if (v < s.edges[idx]) --idx;
        if (v >= s.edges[idx + 1] && idx != 255) ++idx;
        atomicAdd(&s.hist[idx], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // numpy cumsum order
        double a1 = 0.0, b1 = 0.0;
        for (int i = 0; i < 256; ++i) {
            float cen = (s.edges[i] + s.edges[i + 1]) / 2.f;
            a1 += (double)s.hist[i];
            b1 += (double)s.hist[i] * (double)cen;
            s.w1[i] = a1;
            s.c1[i] = b1;
        }
        double a2 = 0.0, b2 = 0.0;
        for (int i = 255; i >= 0; --i) {
            float cen = (s.edges[i] + s.edges[i + 1]) / 2.f;
            a2 += (double)s.hist[i];
            b2 += (double)s.hist[i] * (double)cen;
            s.w2[i] = a2;
            s.c2[i] = b2;
        }
    }
    __syncthreads();
    double var = -1.0;
    int vi = 0x7fffffff;
    if (threadIdx.x < 255) {
        int i = threadIdx.x;
        double m1 = s.c1[i] / s.w1[i];
        double m2 = s.c2[i + 1] / s.w2[i + 1];
        double d = m1 - m2;
        var = (s.w1[i] * s.w2[i + 1]) * (d * d);
        vi = i;
    }
    int best = block_argmax_d(s, var, vi);
    return (s.edges[best] + s.edges[best + 1]) / 2.f;
}

__global__ __launch_bounds__(SEED_THREADS) void seeder_kernel(SeedArgs a) {
    extern __shared__ uint32_t dyn[];
    __shared__ Smem s;
    const int b = blockIdx.x;
    const int H = a.H, W = a.W, HW = H * W;
    const int NW = ((HW + 63) / 64) * 2;
    uint32_t* bm[N_BITMAPS];
    for (int i = 0; i < N_BITMAPS; ++i) bm[i] = dyn + i * NW;
    const float* cam = a.cam + (long)b * HW;
    int32_t* L = a.ws_label + (long)b * HW;
    int32_t* area = a.ws_area + (long)b * HW;
    unsigned long long* keys = a.ws_key + (long)b * HW;

    // -- flat frame: no seeds (tcam_seeding.py:455-456)
    float mn = INFINITY, mx = -INFINITY;
    for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
        float v = cam[p];
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane_id() == 0) {
        s.wf[wave_id()] = mn;
        s.wf[SEED_WAVES + wave_id()] = mx;
    }
    __syncthreads();
    mn = s.wf[0];
    mx = s.wf[SEED_WAVES];
    for (int i = 1; i < SEED_WAVES; ++i) {
        mn = fminf(mn, s.wf[i]);
        mx = fmaxf(mx, s.wf[SEED_WAVES + i]);
    }
    __syncthreads();
    if (!a.roi_only && mn == mx) {
        if (a.seeds)
            for (int p = threadIdx.x; p < HW; p += SEED_THREADS) a.seeds[(long)b * HW + p] = a.ignore_idx;
        return;
    }

    // -- ROI (GetRoiSingleCam or the caller's roi), then erosion
    bool have_roi = a.use_roi || a.roi_only;
    if (have_roi) {
        if (a.roi_in && !a.roi_only) {
            const uint8_t* r = a.roi_in + (long)b * HW;
            build_bitmap(bm[BM_ROI], HW, [&](int p) { return r[p] != 0; });
            __syncthreads();
        } else {
            double tq = a.thresh_b ? a.thresh_b[b] : a.thresh;
            float th = tq >= 0.0 ? (float)(tq * 255.0) : otsu(s, cam, HW, mn, mx);
            if (a.th_out && threadIdx.x == 0) a.th_out[b] = th;
            build_bitmap(bm[BM_A], HW, [&](int p) { return cam[p] * 255.f >= th; });
            __syncthreads();
            int x0 = 0, y0 = 0, x1 = H - 1, y1 = W - 1;  // roi_all: "not used" box
            if (a.roi_method == 0) {
                for (int w = threadIdx.x; w < NW; w += SEED_THREADS) bm[BM_ROI][w] = bm[BM_A][w];
                __syncthreads();
            } else {
                // 4-connected labels, root = smallest raster index
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
                    L[p] = get_bit(bm[BM_A], p) ? p : -1;
                    area[p] = 0;
                    keys[p] = 0ull;
                }
                __syncthreads();
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
                    if (!get_bit(bm[BM_A], p)) continue;
                    int x = p % W;
                    if (x > 0 && get_bit(bm[BM_A], p - 1)) uf_unite(L, p, p - 1);
                    if (p >= W && get_bit(bm[BM_A], p - W)) uf_unite(L, p, p - W);
                }
                __syncthreads();
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
                    if (!get_bit(bm[BM_A], p)) continue;
                    int r = uf_find(L, p);
                    // path compression to the root (an ancestor: safe under concurrent finds)
                    __hip_atomic_store(L + p, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(area + r, 1);
                    if (a.roi_method == 1) {
                        // fixed point 2^-40: integer adds commute (deterministic)
                        unsigned long long fx = (unsigned long long)(long long)(cam[p] * 1099511627776.0f);
                        atomicAdd(keys + r, fx);
                    }
                }
                __syncthreads();
                // largest: max area, first label (smallest root) on ties
                unsigned long long best = 0;
                double bd = -1.0;
                int bdi = 0x7fffffff;
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
                    if (!get_bit(bm[BM_A], p) || ld_label(L, p) != p) continue;
                    const int ar = ld_i32(area, p);
                    unsigned long long k = ((unsigned long long)ar << 32) |
                                           (0xFFFFFFFFu - (uint32_t)p);
                    best = k > best ? k : best;
                    if (a.roi_method == 1) {
                        double d = ((double)(long long)ld_u64(keys, p) / 1099511627776.0) / (double)ar;
                        if (d > bd || (d == bd && p < bdi)) {
                            bd = d;
                            bdi = p;
                        }
                    }
                }
                best = block_max_u64(s, best);
                int chosen = best ? (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull)) : -1;
                if (a.roi_method == 1 && best) {
                    int dch = block_argmax_d(s, bd, bdi);
                    double min_area = (double)HW * a.p_min_area_roi;
                    if (!((double)ld_i32(area, dch) < min_area)) chosen = dch;
                }
                if (chosen < 0) {  // no component: final_roi = blobs (empty)
                    for (int w = threadIdx.x; w < NW; w += SEED_THREADS) bm[BM_ROI][w] = 0;
                } else {
                    build_bitmap(bm[BM_ROI], HW, [&](int p) {
                        return get_bit(bm[BM_A], p) && ld_label(L, p) == chosen;
                    });
                }
                __syncthreads();
                // bbox of the single-component ROI (ext-contour boundingRect, +1 clamp)
                unsigned long long ext = ~0ull, eyt = ~0ull, exb = 0, eyb = 0;
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
                    if (!get_bit(bm[BM_ROI], p)) continue;
                    unsigned long long y = p / W, x = p % W;
                    ext = x < ext ? x : ext;
                    eyt = y < eyt ? y : eyt;
                    exb = x + 1 > exb ? x + 1 : exb;
                    eyb = y + 1 > eyb ? y + 1 : eyb;
                }
                ext = block_min_u64(s, ext);
                eyt = block_min_u64(s, eyt);
                exb = block_max_u64(s, exb);
                eyb = block_max_u64(s, eyb);
                if (exb == 0) {
                    x0 = y0 = x1 = y1 = 0;
                } else {
                    x0 = (int)ext;
                    y0 = (int)eyt;
                    x1 = min((int)exb, W - 1);
                    y1 = min((int)eyb, H - 1);
                }
            }
            if (a.bbox_out && threadIdx.x == 0) {
                a.bbox_out[b * 4 + 0] = x0;
                a.bbox_out[b * 4 + 1] = y0;
                a.bbox_out[b * 4 + 2] = x1;
                a.bbox_out[b * 4 + 3] = y1;
            }
        }
        if (a.roi_only) {
            if (a.roi_out)
                for (int p = threadIdx.x; p < HW; p += SEED_THREADS)
                    a.roi_out[(long)b * HW + p] = (uint8_t)get_bit(bm[BM_ROI], p);
            return;
        }
        for (int it = 0; it < a.fg_erode_iter; ++it)
            morph(bm[BM_ROI], bm[BM_T], bm[BM_ROI], H, W, a.fg_erode_k, false);
        if (a.roi_out)
            for (int p = threadIdx.x; p < HW; p += SEED_THREADS)
                a.roi_out[(long)b * HW + p] = (uint8_t)get_bit(bm[BM_ROI], p);
    }

    // -- foreground (_SFG, tcam_seeding.py:478-521)
    for (int w = threadIdx.x; w < NW; w += SEED_THREADS) {
        bm[BM_FG][w] = 0;
        bm[BM_BG][w] = 0;
    }
    __syncthreads();
    int n;
    if (have_roi) {
        int cnt = 0;
        for (int w = threadIdx.x; w < NW; w += SEED_THREADS) cnt += __popc(bm[BM_ROI][w]);
        int nroi = block_sum_i(s, cnt);
        n = (int)(a.max_p * (float)nroi);
    } else {
        n = (int)((double)a.max_p * (double)HW);
    }
    auto fgval = [&](int p) -> float {
        float c = cam[p];
        if (have_roi) c = c * (float)get_bit(bm[BM_ROI], p);
        return c + 1e-8f;
    };
    if (n > 0 && a.max_ > 0) {
        __syncthreads();
        select_top<uint32_t>(s, bm[BM_A], bm[BM_B], HW, NW, n, [&](int p, uint32_t& k) {
            k = ord32(fgval(p));
            return true;
        });
        int k = min(a.max_, n);
        if (a.seed_tech == 1)
            sample(s, a, b, 0, bm[BM_FG], bm[BM_A], bm[BM_B], HW, NW, n, k, keys,
                   [&](int p) { return fgval(p); });
        else
            sample(s, a, b, 0, bm[BM_FG], bm[BM_A], bm[BM_B], HW, NW, n, k, keys,
                   [&](int p) { return 1.0f; });
    }
    // -- background (_SBG, tcam_seeding.py:529-563): n smallest, uniform draw
    n = (int)((double)a.min_p * (double)H * (double)W);
    if (n > 0 && a.min_ > 0) {
        __syncthreads();
        select_top<uint32_t>(s, bm[BM_A], bm[BM_B], HW, NW, n, [&](int p, uint32_t& k) {
            k = ~ord32(cam[p] + 1e-8f);
            return true;
        });
        int k = min(a.min_, n);
        sample(s, a, b, 1, bm[BM_BG], bm[BM_A], bm[BM_B], HW, NW, n, k, keys,
               [&](int p) { return 1.0f; });
    }
    __syncthreads();
    // -- dilation, conflicts, labels (tcam_seeding.py:238-256)
    uint32_t* fg = bm[BM_FG];
    uint32_t* bg = bm[BM_BG];
    if (a.ksz > 1) {
        morph(bm[BM_A], bm[BM_T], bm[BM_FG], H, W, a.ksz, true);
        morph(bm[BM_B], bm[BM_T], bm[BM_BG], H, W, a.ksz, true);
        fg = bm[BM_A];
        bg = bm[BM_B];
    }
    int32_t* out = a.seeds + (long)b * HW;
    for (int p = threadIdx.x; p < HW; p += SEED_THREADS) {
        uint32_t f = get_bit(fg, p), g = get_bit(bg, p);
        out[p] = (f && !g) ? 1 : ((g && !f) ? 0 : a.ignore_idx);
    }
}

// ROI threshold of a stored CAM (inference_wsol.py:1107-1124 / 1144-1159):
//   full = F.interpolate(cam, (S, S), bilinear, align_corners=True)
//   th   = STOtsu(floor(full * 255))   (cams/core_seeding.py:23-56, float32 torch ops)
// One workgroup per frame; the histogram has one bin per integer value in [min, max]
// (torch.histc with max-min+1 bins over [min, max] puts each integer in its own bin).
constexpr int STOTSU_MAX_BINS = 1024;
__global__ __launch_bounds__(256) void stotsu_kernel(const float* __restrict__ cams,
                                                     float* __restrict__ th_out, int h, int w,
                                                     int S) {
    __shared__ int hist[STOTSU_MAX_BINS];
    __shared__ float red[8];
    const int b = blockIdx.x;
    const float* src = cams + (long)b * h * w;
    const float sh = S > 1 ? (float)(h - 1) / (float)(S - 1) : 0.f;
    const float sw = S > 1 ? (float)(w - 1) / (float)(S - 1) : 0.f;
    auto val = [&](int p) -> float {
        int oy = p / S, ox = p - oy * S;
        float ry = sh * (float)oy, rx = sw * (float)ox;
        int y0 = (int)ry, x0 = (int)rx;
        int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
        float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
        float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
        float v = ly0 * (lx0 * src[y0 * w + x0] + lx1 * src[y0 * w + x1]) +
                  ly1 * (lx0 * src[y1 * w + x0] + lx1 * src[y1 * w + x1]);
        return floorf(v * 255.f);
    };
    const int n = S * S;
    float mn = INFINITY, mx = -INFINITY;
    for (int p = threadIdx.x; p < n; p += 256) {
        float v = val(p);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[wid] = mn;
        red[4 + wid] = mx;
    }
    __syncthreads();
    mn = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
    mx = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
    if (mn == mx) {  // bad egg: STOtsu returns min
        if (threadIdx.x == 0) th_out[b] = mn;
        return;
    }
    const int nb = (int)(mx - mn + 1.f);
    if (nb > STOTSU_MAX_BINS || !(mx - mn < 1e9f)) {
        if (threadIdx.x == 0) th_out[b] = NAN;
        return;
    }
    for (int i = threadIdx.x; i < nb; i += 256) hist[i] = 0;
    __syncthreads();
    for (int p = threadIdx.x; p < n; p += 256) atomicAdd(&hist[(int)(val(p) - mn)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        // float32 as torch: cumsums of integers < 2^24 are exact in any order
        float W = 0.f, Cs = 0.f;
        for (int i = 0; i < nb; ++i) {
            W += (float)hist[i];
            Cs += (float)hist[i] * (mn + (float)i);
        }
        float w1 = 0.f, c1 = 0.f, best = -1.f;
        int bi = 0;
        for (int i = 0; i < nb - 1; ++i) {
            w1 += (float)hist[i];
            c1 += (float)hist[i] * (mn + (float)i);
            float w2 = W - w1, c2 = Cs - c1;   // suffix sums from i + 1 (exact)
            float m1 = c1 / w1, m2 = c2 / w2;
            float d = m1 - m2;
            float var = (w1 * w2) * (d * d);
            if (var > best) {
                best = var;
                bi = i;
            }
        }
        th_out[b] = mn + (float)bi;
    }
}

__device__ __forceinline__ float nan_to_num01(float v) {
    if (v != v) return 0.f;
    if (isinf(v)) return v > 0.f ? 1.f : 0.f;
    return v;
}

// prepare_std_cams_disq (learning/train_wsol.py:417-432): nan_to_num(0, 1, 0),
// F.interpolate(bilinear, align_corners=False) to the image size, nan_to_num.
__global__ __launch_bounds__(256) void prepare_cams_kernel(const float* __restrict__ in,
                                                           float* __restrict__ out, int h,
                                                           int w, int Ho, int Wo) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= Ho * Wo) return;
    const float* src = in + (long)b * h * w;
    const float sh = (float)h / (float)Ho, sw = (float)w / (float)Wo;
    int oy = p / Wo, ox = p - oy * Wo;
    float ry = fmaxf(sh * ((float)oy + 0.5f) - 0.5f, 0.f);
    float rx = fmaxf(sw * ((float)ox + 0.5f) - 0.5f, 0.f);
    int y0 = (int)ry, x0 = (int)rx;
    int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    float ly1 = ry - (float)y0, ly0 = 1.f - ly1;
    float lx1 = rx - (float)x0, lx0 = 1.f - lx1;
    float v = ly0 * (lx0 * nan_to_num01(src[y0 * w + x0]) + lx1 * nan_to_num01(src[y0 * w + x1])) +
              ly1 * (lx0 * nan_to_num01(src[y1 * w + x0]) + lx1 * nan_to_num01(src[y1 * w + x1]));
    out[(long)b * Ho * Wo + p] = nan_to_num01(v);
}

}  // namespace

extern "C" int tcam_stotsu_roi_thresh(const float* cams, int B, int h, int w, int S,
                                      float* th_out, void* stream) {
    TCAM_REQUIRE(cams && th_out && B > 0 && h > 0 && w > 0 && S > 0);
    stotsu_kernel<<<B, 256, 0, as_stream(stream)>>>(cams, th_out, h, w, S);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_prepare_std_cams(const float* cams, float* out, int B, int h, int w,
                                     int Ho, int Wo, void* stream) {
    TCAM_REQUIRE(cams && out && B > 0 && h > 0 && w > 0 && Ho > 0 && Wo > 0);
    dim3 grid(cdiv((long)Ho * Wo, 256), B);
    prepare_cams_kernel<<<grid, 256, 0, as_stream(stream)>>>(cams, out, h, w, Ho, Wo);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" size_t tcam_seeder_ws_bytes(int B, int H, int W) {
    return (size_t)B * H * W * (4 + 4 + 8);
}

static int launch_seeder(SeedArgs& a, int B, void* ws, size_t ws_bytes, void* stream) {
    const long HW = (long)a.H * a.W;
    TCAM_REQUIRE(a.cam && B > 0 && a.H > 0 && a.W > 0 && HW <= SEED_MAX_HW);
    TCAM_REQUIRE(ws && ws_bytes >= tcam_seeder_ws_bytes(B, a.H, a.W));
    char* w = (char*)ws;
    a.ws_key = (unsigned long long*)w;
    a.ws_label = (int32_t*)(w + (size_t)B * HW * 8);
    a.ws_area = (int32_t*)(w + (size_t)B * HW * 12);
    const int NW = (int)(((HW + 63) / 64) * 2);
    size_t lds = (size_t)N_BITMAPS * NW * 4;
    seeder_kernel<<<B, SEED_THREADS, lds, as_stream(stream)>>>(a);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_tcam_seeder(const float* cams, const uint8_t* roi, int32_t* seeds, int B,
                                int H, int W, int seed_tech, int min_, int max_, float max_p,
                                float min_p, int fg_erode_k, int fg_erode_iter, int ksz,
                                int ignore_idx, int roi_method, double p_min_area_roi,
                                int use_roi, unsigned long long seed,
                                unsigned long long offset, uint8_t* roi_out, float* th_out,
                                void* ws, size_t ws_bytes, void* stream) {
    TCAM_REQUIRE(seeds && seed_tech >= 0 && seed_tech <= 1 && min_ >= 0 && max_ >= 0);
    TCAM_REQUIRE(roi_method >= 0 && roi_method <= 2 && ksz >= 1 && fg_erode_iter >= 0);
    TCAM_REQUIRE(fg_erode_iter == 0 || fg_erode_k >= 1);
    TCAM_REQUIRE(max_p >= 0.f && max_p <= 1.f && min_p >= 0.f && min_p <= 1.f);
    SeedArgs a = {};
    a.cam = cams;
    a.roi_in = roi;
    a.seeds = seeds;
    a.roi_out = roi_out;
    a.th_out = th_out;
    a.H = H;
    a.W = W;
    a.seed_tech = seed_tech;
    a.min_ = min_;
    a.max_ = max_;
    a.max_p = max_p;
    a.min_p = min_p;
    a.fg_erode_k = fg_erode_k;
    a.fg_erode_iter = fg_erode_iter;
    a.ksz = ksz;
    a.ignore_idx = ignore_idx;
    a.roi_method = roi_method;
    a.p_min_area_roi = p_min_area_roi;
    a.use_roi = use_roi;
    a.thresh = -1.0;
    a.seed = seed;
    a.offset = offset;
    a.roi_only = 0;
    return launch_seeder(a, B, ws, ws_bytes, stream);
}

extern "C" int tcam_get_roi(const float* cams, int B, int H, int W, int roi_method,
                            double p_min_area_roi, double thresh, const double* thresh_b,
                            uint8_t* roi_out,
                            int32_t* bbox_out, float* th_out, void* ws, size_t ws_bytes,
                            void* stream) {
    TCAM_REQUIRE(roi_out && roi_method >= 0 && roi_method <= 2);
    SeedArgs a = {};
    a.cam = cams;
    a.roi_out = roi_out;
    a.bbox_out = bbox_out;
    a.th_out = th_out;
    a.H = H;
    a.W = W;
    a.roi_method = roi_method;
    a.p_min_area_roi = p_min_area_roi;
    a.use_roi = 1;
    a.thresh = thresh;
    a.thresh_b = thresh_b;
    a.roi_only = 1;
    a.ksz = 1;
    return launch_seeder(a, B, ws, ws_bytes, stream);
}
