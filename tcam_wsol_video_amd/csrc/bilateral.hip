// Permutohedral-lattice bilateral filter for gfx950 — the device replacement of
// the reference's SWIG CRF filters
//   bilateralfilter_batch       crf/crfwrapper/bilateralfilter/bilateralfilter.cpp:4-55
//   colorbilateralfilter_batch  crf/crfwrapper/colorbilateralfilter/colorbilateralfilter.cpp:4-54
// over the lattice of crf/crfwrapper/bilateralfilter/permutohedral.cpp:105-571
// (Adams et al. 2010, Krähenbühl's variant; the x86-64 build takes the SSE branch,
// which is the one restated here).
//
// Output is BIT-IDENTICAL to the reference on the same inputs:
//   * lattice coordinates, ranks and barycentric weights use the reference's fp32
//     operation sequence with contraction off (no FMA), round-to-nearest-even;
//   * the splat sum of a lattice vertex is accumulated sequentially in increasing
//     point order — the reference's order — by gathering the vertex's entries
//     after a STABLE sort of (vertex, entry) pairs that starts in point order;
//   * blur and slice are per-vertex / per-point in the reference's order.
// Vertex numbering differs from the reference's hash order (and between runs), but
// no output depends on it.
//
// Lattice keys: d coordinates, all congruent to the vertex remainder r mod (d+1),
// packed exactly into one 64-bit word (r, (k_i - r)/(d+1)); the hash-table slot
// holding a key IS its vertex id, so insertion is a single lock-free CAS.
//
// Pipeline per call (N images of P = H*W points, E = N*P*(d+1) entries):
//   lattice  (point)   elevate, simplex, barycentric, insert d+1 keys
//   compact  (slot)    dense vertex ids per image
//   remap    (entry)   sort key = image vertex id
//   sort               stable LSD radix sort of (vertex, entry)   [hipCUB]
//   segments (entry)   [begin, end) of every vertex in the sorted entries
//   splat    (vertex)  sequential gather in point order, all K channels
//   blur x(d+1) (vertex) v + 0.5 (n1 + n2) along each lattice axis
//   slice    (point)   sum_r (w_r * alpha) * v, then out (N, K, H, W)
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr uint64_t kEmpty = ~0ull;   // remainder field 7: never a valid key
constexpr int kMaxK = 8;             // channels per call (TCAM uses K = 2)
constexpr int kBlock = 256;

struct Geo {
    int N, K, H, W, P, D;
    long E;        // entries = N * P * (D + 1)
    long Vcap;     // vertex capacity per image = (P + 1) * (D + 1)
    int logCap;    // hash slots per image = 2^logCap >= 2 * Vcap
    int sortBits;  // bits of N * Vcap
};

inline Geo make_geo(int N, int K, int H, int W, int D) {
    Geo g;
    g.N = N; g.K = K; g.H = H; g.W = W; g.P = H * W; g.D = D;
    g.E = (long)N * g.P * (D + 1);
    g.Vcap = (long)(g.P + 1) * (D + 1);
    g.logCap = 1;
    while ((1l << g.logCap) < 2 * g.Vcap) ++g.logCap;
    g.sortBits = 1;
    while ((1l << g.sortBits) < (long)N * g.Vcap) ++g.sortBits;
    return g;
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout (offsets in bytes; every block 256-B aligned).
struct Ws {
    size_t hdr, slot, cid, vslot, eslot, skey, sval, skey2, sval2, bary, seg_b, seg_e, v0,
        v1, tmp, total;
    size_t tmp_bytes;
};

Ws make_ws(const Geo& g, size_t sort_tmp) {
    Ws w;
    size_t o = 0;
    const long cap = 1l << g.logCap;
    w.hdr = o;   o += al(sizeof(int) * (g.N + 64));
    w.slot = o;  o += al(sizeof(uint64_t) * g.N * cap);
    w.cid = o;   o += al(sizeof(int) * g.N * cap);
    w.vslot = o; o += al(sizeof(int) * g.N * g.Vcap);
    w.eslot = o; o += al(sizeof(int) * g.E);
    w.skey = o;  o += al(sizeof(uint32_t) * g.E);
    w.sval = o;  o += al(sizeof(uint32_t) * g.E);
    w.skey2 = o; o += al(sizeof(uint32_t) * g.E);
    w.sval2 = o; o += al(sizeof(uint32_t) * g.E);
    w.bary = o;  o += al(sizeof(float) * g.E);
    w.seg_b = o; o += al(sizeof(int) * g.N * g.Vcap);
    w.seg_e = o; o += al(sizeof(int) * g.N * g.Vcap);
    w.v0 = o;    o += al(sizeof(float) * g.N * g.Vcap * g.K);
    w.v1 = o;    o += al(sizeof(float) * g.N * g.Vcap * g.K);
    w.tmp = o;   o += al(sort_tmp);
    w.tmp_bytes = sort_tmp;
    w.total = o;
    return w;
}

// Bits per packed quotient: d = 5 -> 12 (|key| <= 12287), d <= 4 -> 15 (all shorts).
template <int D> struct KeyBits { static constexpr int B = D == 5 ? 12 : 15; };

// Sets *err when a quotient does not fit (the key is then not representable).
template <int D>
__device__ __forceinline__ uint64_t pack_key(const int (&k)[D], int r, int* err) {
    constexpr int B = KeyBits<D>::B;
    constexpr int bias = 1 << (B - 1);
    uint64_t w = (uint64_t)r;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const int q = (k[i] - r) / (D + 1) + bias;   // exact: k[i] == r (mod d+1)
        if (q < 0 || q >= (1 << B)) *err = 1;
        w |= (uint64_t)(q & ((1 << B) - 1)) << (3 + B * i);
    }
    return w;
}

template <int D>
__device__ __forceinline__ void unpack_key(uint64_t w, int (&k)[D], int& r) {
    constexpr int B = KeyBits<D>::B;
    constexpr int bias = 1 << (B - 1);
    r = (int)(w & 7);
#pragma unroll
    for (int i = 0; i < D; ++i)
        k[i] = ((int)((w >> (3 + B * i)) & ((1u << B) - 1)) - bias) * (D + 1) + r;
}

__device__ __forceinline__ uint32_t hash_slot(uint64_t w, int logCap) {
    w ^= w >> 31;
    w *= 0x9E3779B97F4A7C15ull;
    w ^= w >> 29;
    return (uint32_t)(w >> (64 - logCap));
}

__device__ __forceinline__ int table_insert(uint64_t* tab, int logCap, uint64_t key) {
    const uint32_t mask = (1u << logCap) - 1;
    uint32_t h = hash_slot(key, logCap);
    while (true) {
        uint64_t cur = __hip_atomic_load(tab + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == kEmpty) cur = atomicCAS((unsigned long long*)(tab + h), kEmpty, key);
        if (cur == kEmpty || cur == key) return (int)h;
        h = (h + 1) & mask;
    }
}

// Read-only probe (the table is complete: launched after the insert kernel).
__device__ __forceinline__ int table_find(const uint64_t* tab, int logCap, uint64_t key) {
    const uint32_t mask = (1u << logCap) - 1;
    uint32_t h = hash_slot(key, logCap);
    while (true) {
        const uint64_t cur = tab[h];
        if (cur == key) return (int)h;
        if (cur == kEmpty) return -1;
        h = (h + 1) & mask;
    }
}

struct LatticeArgs {
    const float* img;      // (N, 3, H, W)
    float inv_xy_div;      // sigma_xy  (features divide, as the reference)
    float rgb_div;         // sigma_rgb
    float sf[5];           // scale_factor[i] (host-computed as permutohedral.cpp:164-166)
    float inv_dp1, dp1;    // 1.0f / (d+1), d+1
    uint64_t* slot;
    int* eslot;
    uint32_t* sval;
    float* bary;
    int* err;
    int xy;                // 1: (x, y, r, g, b) features; 0: colour planes only
};

// One thread per point (plus one virtual zero-feature point per image when P % 4 != 0:
// the SSE init pads the last block of 4 with zero features and inserts their keys,
// permutohedral.cpp:171-175, 258-264).
template <int D>
__global__ __launch_bounds__(kBlock) void lattice_kernel(LatticeArgs a, Geo g) {
#pragma clang fp contract(off)
    const int extra = (g.P % 4) ? 1 : 0;
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const int per = g.P + extra;
    if (t >= (long)g.N * per) return;
    const int n = (int)(t / per);
    const int p = (int)(t - (long)n * per);
    const bool real = p < g.P;

    float f[D];
    if (real) {
        const float* im = a.img + (long)n * 3 * g.P + p;
        if (a.xy) {
            const int y = p / g.W, x = p - y * g.W;
            f[0] = (float)x / a.inv_xy_div;
            if (D > 1) f[1] = (float)y / a.inv_xy_div;
#pragma unroll
            for (int c = 2; c < D; ++c) f[c] = im[(long)(c - 2) * g.P] / a.rgb_div;
        } else {
#pragma unroll
            for (int c = 0; c < D; ++c) f[c] = im[(long)c * g.P] / a.rgb_div;
        }
    } else {
#pragma unroll
        for (int c = 0; c < D; ++c) f[c] = 0.f;
    }

    // Elevate (permutohedral.cpp:181-189).
    float el[D + 1];
    float sm = 0.f;
#pragma unroll
    for (int j = D; j > 0; --j) {
        const float cf = f[j - 1] * a.sf[j - 1];
        el[j] = sm - (float)j * cf;
        sm += cf;
    }
    el[0] = sm;
    // Closest 0-coloured point (192-203): cvtps_epi32 = round half to even.
    float rem0[D + 1];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i <= D; ++i) {
        const float v = rintf(a.inv_dp1 * el[i]);
        rem0[i] = v * a.dp1;
        sum += v;
    }
    // Ranks (206-215).
    float rank[D + 1];
#pragma unroll
    for (int i = 0; i <= D; ++i) rank[i] = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const float di = el[i] - rem0[i];
#pragma unroll
        for (int j = i + 1; j <= D; ++j) {
            const float dj = el[j] - rem0[j];
            const float c = di < dj ? 1.f : 0.f;
            rank[i] += c;
            rank[j] += 1.f - c;
        }
    }
    // Back onto the plane (218-224).
#pragma unroll
    for (int i = 0; i <= D; ++i) {
        rank[i] += sum;
        const float add = rank[i] < 0.f ? a.dp1 : 0.f;
        const float sub = rank[i] >= a.dp1 ? a.dp1 : 0.f;
        rank[i] += add - sub;
        rem0[i] += add - sub;
    }
    // Barycentric coordinates (227-243), accumulated in the reference order.
    float b[D + 2];
#pragma unroll
    for (int i = 0; i < D + 2; ++i) b[i] = 0.f;
#pragma unroll
    for (int i = 0; i <= D; ++i) {
        const float v = (el[i] - rem0[i]) * a.inv_dp1;
        const int pp = (int)((float)D - rank[i]);
#pragma unroll
        for (int q = 0; q <= D; ++q) {
            if (q == pp) b[q] += v;
            if (q == pp) b[q + 1] -= v;
        }
    }
    b[0] += 1.f + b[D + 1];

    int lerr = 0;
    const long ebase = ((long)n * g.P + p) * (D + 1);
    uint64_t* tab = a.slot + ((long)n << g.logCap);
    // Vertices (249-256): key_i = rem0_i + canonical[r][rank_i].
#pragma unroll
    for (int r = 0; r <= D; ++r) {
        int k[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int rk = (int)rank[i];
            const int canon = rk <= D - r ? r : r - (D + 1);
            k[i] = (int)(short)(rem0[i] + (float)canon);
        }
        const uint64_t key = pack_key<D>(k, r, &lerr);
        const int h = table_insert(tab, g.logCap, key);
        if (real) {
            a.eslot[ebase + r] = h;
            a.sval[ebase + r] = (uint32_t)(ebase + r);
            a.bary[ebase + r] = b[r];
        }
    }
    if (lerr) atomicOr(a.err, 1);
}

// Dense vertex ids: cid[slot] and vslot[id] per image; M[n] = vertex count.
__global__ __launch_bounds__(kBlock) void compact_kernel(const uint64_t* slot, int* cid,
                                                         int* vslot, int* M, Geo g) {
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const long cap = 1l << g.logCap;
    if (t >= (long)g.N * cap) return;
    if (slot[t] == kEmpty) return;
    const int n = (int)(t >> g.logCap);
    const int c = atomicAdd(M + n, 1);
    cid[t] = c;
    vslot[(long)n * g.Vcap + c] = (int)(t & (cap - 1));
}

__global__ __launch_bounds__(kBlock) void remap_kernel(const int* eslot, const int* cid,
                                                       uint32_t* skey, Geo g) {
    const long e = (long)blockIdx.x * kBlock + threadIdx.x;
    if (e >= g.E) return;
    const int n = (int)(e / ((long)g.P * (g.D + 1)));
    const long s = ((long)n << g.logCap) + eslot[e];
    skey[e] = (uint32_t)((long)n * g.Vcap + cid[s]);
}

__global__ __launch_bounds__(kBlock) void segments_kernel(const uint32_t* skey2, int* seg_b,
                                                          int* seg_e, Geo g) {
    const long i = (long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= g.E) return;
    const uint32_t k = skey2[i];
    if (i == 0 || skey2[i - 1] != k) seg_b[k] = (int)i;
    if (i == g.E - 1 || skey2[i + 1] != k) seg_e[k] = (int)(i + 1);
}

// values[v][k] = sum over the vertex's entries, in point order, of bary * in[k][p]
// (permutohedral.cpp:413-421: values[o] += w * val, no fusion).
__global__ __launch_bounds__(kBlock) void splat_kernel(const float* in, const uint32_t* sval2,
                                                       const float* bary, const int* seg_b,
                                                       const int* seg_e, const int* M,
                                                       float* vals, Geo g) {
#pragma clang fp contract(off)
    const long v = (long)blockIdx.x * kBlock + threadIdx.x;
    if (v >= (long)g.N * g.Vcap) return;
    const int n = (int)(v / g.Vcap);
    const int c = (int)(v - (long)n * g.Vcap);
    if (c >= M[n]) return;
    float acc[kMaxK];
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) acc[k] = 0.f;
    const int i0 = seg_b[v], i1 = seg_e[v];
    const int dp1 = g.D + 1;
    const float* inn = in + (long)n * g.K * g.P;
    const long pbase = (long)n * g.P;
    for (int i = i0; i < i1; ++i) {
        const uint32_t e = sval2[i];
        const float w = bary[e];
        const int p = (int)(e / dp1 - pbase);
#pragma unroll
        for (int k = 0; k < kMaxK; ++k)
            if (k < g.K) acc[k] += w * inn[(long)k * g.P + p];
    }
#pragma unroll
    for (int k = 0; k < kMaxK; ++k)
        if (k < g.K) vals[v * g.K + k] = acc[k];
}

// One blur pass along lattice axis j (permutohedral.cpp:425-441).
template <int D>
__global__ __launch_bounds__(kBlock) void blur_kernel(const uint64_t* slot, const int* cid,
                                                      const int* vslot, const int* M,
                                                      const float* old, float* nw, int j,
                                                      Geo g) {
#pragma clang fp contract(off)
    const long v = (long)blockIdx.x * kBlock + threadIdx.x;
    if (v >= (long)g.N * g.Vcap) return;
    const int n = (int)(v / g.Vcap);
    const int c = (int)(v - (long)n * g.Vcap);
    if (c >= M[n]) return;
    const uint64_t* tab = slot + ((long)n << g.logCap);
    const int* cidn = cid + ((long)n << g.logCap);
    int k[D], r;
    unpack_key<D>(tab[vslot[v]], k, r);
    int k1[D], k2[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        k1[i] = k[i] - 1;
        k2[i] = k[i] + 1;
        if (i == j) {
            k1[i] = k[i] + D;
            k2[i] = k[i] - D;
        }
    }
    const int r1 = r == 0 ? D : r - 1;   // n1 lies on remainder r-1, n2 on r+1 (mod d+1)
    const int r2 = r == D ? 0 : r + 1;
    int bad1 = 0, bad2 = 0;   // a neighbour outside the packable range is not in the table
    const uint64_t key1 = pack_key<D>(k1, r1, &bad1);
    const uint64_t key2 = pack_key<D>(k2, r2, &bad2);
    const int h1 = bad1 ? -1 : table_find(tab, g.logCap, key1);
    const int h2 = bad2 ? -1 : table_find(tab, g.logCap, key2);
    const long base = (long)n * g.Vcap;
    const long o1 = h1 >= 0 ? base + cidn[h1] : -1;
    const long o2 = h2 >= 0 ? base + cidn[h2] : -1;
#pragma unroll
    for (int q = 0; q < kMaxK; ++q) {
        if (q < g.K) {
            const float a = o1 >= 0 ? old[o1 * g.K + q] : 0.f;
            const float b = o2 >= 0 ? old[o2 * g.K + q] : 0.f;
            nw[v * g.K + q] = old[v * g.K + q] + 0.5f * (a + b);
        }
    }
}

// out[n][k][p] = sum_r (bary_r * alpha) * vals[vertex_r][k]   (permutohedral.cpp:446-456).
template <int D>
__global__ __launch_bounds__(kBlock) void slice_kernel(const uint32_t* skey, const float* bary,
                                                       const float* vals, float alpha,
                                                       float* out, Geo g) {
#pragma clang fp contract(off)
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (long)g.N * g.P) return;
    const int n = (int)(t / g.P);
    const int p = (int)(t - (long)n * g.P);
    float acc[kMaxK];
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r <= D; ++r) {
        const long e = t * (D + 1) + r;
        const float w = bary[e] * alpha;
        const long v = skey[e];
#pragma unroll
        for (int k = 0; k < kMaxK; ++k)
            if (k < g.K) acc[k] += w * vals[v * g.K + k];
    }
#pragma unroll
    for (int k = 0; k < kMaxK; ++k)
        if (k < g.K) out[((long)n * g.K + k) * g.P + p] = acc[k];
}

size_t sort_tmp_bytes(const Geo& g) {
    size_t b = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)g.E, 0, g.sortBits,
                                           (hipStream_t)0) != hipSuccess)
        return 0;
    return b;
}

bool valid_dims(int N, int K, int H, int W, int D) {
    if (N <= 0 || K <= 0 || K > kMaxK || H <= 0 || W <= 0) return false;
    if (D < 1 || D > 5) return false;
    const Geo g = make_geo(N, K, H, W, D);
    // Entry and vertex indices are 32-bit.
    return g.E < (1l << 31) && (long)N * g.Vcap < (1l << 31) && g.sortBits <= 32 &&
           ((long)N << g.logCap) < (1l << 31);
}

// The reference's per-lattice constants (permutohedral.cpp:160-166, 444): computed in
// double and rounded to float exactly as the SSE init does.
void lattice_constants(int D, float* sf, float* alpha) {
    const float inv_std_dev = (float)(std::sqrt(2.0 / 3.0) * (D + 1));
    for (int i = 0; i < D; ++i)
        sf[i] = (float)(1.0 / std::sqrt((double)((i + 2) * (i + 1))) * (double)inv_std_dev);
    *alpha = 1.0f / (1 + powf(2, -D));
}

template <int D>
int run(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
        const Geo& g, float s_rgb, float s_xy, int xy, hipStream_t st) {
    const size_t tmp = sort_tmp_bytes(g);
    if (tmp == 0) return TCAM_E_ARG;
    const Ws w = make_ws(g, tmp);
    if (!ws || ws_bytes < w.total) return TCAM_E_NOMEM;
    char* base = (char*)ws;
    int* M = (int*)(base + w.hdr);
    int* err = M + g.N;
    uint64_t* slot = (uint64_t*)(base + w.slot);
    int* cid = (int*)(base + w.cid);
    int* vslot = (int*)(base + w.vslot);
    int* eslot = (int*)(base + w.eslot);
    uint32_t* skey = (uint32_t*)(base + w.skey);
    uint32_t* sval = (uint32_t*)(base + w.sval);
    uint32_t* skey2 = (uint32_t*)(base + w.skey2);
    uint32_t* sval2 = (uint32_t*)(base + w.sval2);
    float* bary = (float*)(base + w.bary);
    int* seg_b = (int*)(base + w.seg_b);
    int* seg_e = (int*)(base + w.seg_e);
    float* v0 = (float*)(base + w.v0);
    float* v1 = (float*)(base + w.v1);
    const long cap = 1l << g.logCap;

    hipError_t e;
    if ((e = hipMemsetAsync(M, 0, sizeof(int) * (g.N + 64), st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(slot, 0xff, sizeof(uint64_t) * g.N * cap, st)) != hipSuccess)
        return e;

    LatticeArgs a;
    a.img = images;
    a.inv_xy_div = s_xy;
    a.rgb_div = s_rgb;
    float alpha;
    lattice_constants(D, a.sf, &alpha);
    a.inv_dp1 = 1.0f / (D + 1);
    a.dp1 = (float)(D + 1);
    a.slot = slot;
    a.eslot = eslot;
    a.sval = sval;
    a.bary = bary;
    a.err = err;
    a.xy = xy;
    const long npts = (long)g.N * (g.P + ((g.P % 4) ? 1 : 0));
    lattice_kernel<D><<<cdiv(npts, kBlock), kBlock, 0, st>>>(a, g);
    TCAM_CHECK_LAUNCH();
    compact_kernel<<<cdiv((long)g.N * cap, kBlock), kBlock, 0, st>>>(slot, cid, vslot, M, g);
    TCAM_CHECK_LAUNCH();
    remap_kernel<<<cdiv(g.E, kBlock), kBlock, 0, st>>>(eslot, cid, skey, g);
    TCAM_CHECK_LAUNCH();
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(base + w.tmp, tb, skey, skey2, sval, sval2,
                                                (int)g.E, 0, g.sortBits, st)) != hipSuccess)
        return e;
    // Vertices without entries (the virtual point's) keep the empty segment [0, 0).
    if ((e = hipMemsetAsync(seg_b, 0, sizeof(int) * g.N * g.Vcap, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(seg_e, 0, sizeof(int) * g.N * g.Vcap, st)) != hipSuccess) return e;
    segments_kernel<<<cdiv(g.E, kBlock), kBlock, 0, st>>>(skey2, seg_b, seg_e, g);
    TCAM_CHECK_LAUNCH();
    const long nv = (long)g.N * g.Vcap;
    splat_kernel<<<cdiv(nv, kBlock), kBlock, 0, st>>>(ins, sval2, bary, seg_b, seg_e, M, v0,
                                                      g);
    TCAM_CHECK_LAUNCH();
    float* cur = v0;
    float* nxt = v1;
    for (int j = 0; j <= D; ++j) {
        blur_kernel<D><<<cdiv(nv, kBlock), kBlock, 0, st>>>(slot, cid, vslot, M, cur, nxt, j,
                                                            g);
        TCAM_CHECK_LAUNCH();
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    slice_kernel<D><<<cdiv((long)g.N * g.P, kBlock), kBlock, 0, st>>>(skey, bary, cur, alpha,
                                                                       outs, g);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

int dispatch(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
             int N, int K, int H, int W, int D, float s_rgb, float s_xy, int xy, void* stream) {
    if (!valid_dims(N, K, H, W, D) || !images || !ins || !outs) return TCAM_E_ARG;
    if (!(s_rgb > 0.f) || (xy && !(s_xy > 0.f))) return TCAM_E_ARG;
    const Geo g = make_geo(N, K, H, W, D);
    hipStream_t st = as_stream(stream);
    switch (D) {
        case 1: return run<1>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st);
        case 2: return run<2>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st);
        case 3: return run<3>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st);
        case 4: return run<4>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st);
        default: return run<5>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st);
    }
}

size_t ws_bytes_for(int N, int K, int H, int W, int D) {
    if (!valid_dims(N, K, H, W, D)) return 0;
    const Geo g = make_geo(N, K, H, W, D);
    const size_t tmp = sort_tmp_bytes(g);
    if (tmp == 0) return 0;
    return make_ws(g, tmp).total;
}

// Host-compat path: H2D -> filter -> D2H on the null stream, temporaries freed.
void host_compat(float* images, float* ins, float* outs, int N, int K, int H, int W, int D,
                 float s_rgb, float s_xy, int xy) {
    const size_t P = (size_t)H * W;
    const size_t wsb = ws_bytes_for(N, K, H, W, D);
    if (wsb == 0) return;
    float *di = nullptr, *dn = nullptr, *dout = nullptr;
    void* ws = nullptr;
    if (hipMalloc(&di, sizeof(float) * N * 3 * P) == hipSuccess &&
        hipMalloc(&dn, sizeof(float) * N * K * P) == hipSuccess &&
        hipMalloc(&dout, sizeof(float) * N * K * P) == hipSuccess &&
        hipMalloc(&ws, wsb) == hipSuccess &&
        hipMemcpy(di, images, sizeof(float) * N * 3 * P, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dn, ins, sizeof(float) * N * K * P, hipMemcpyHostToDevice) == hipSuccess &&
        dispatch(di, dn, dout, ws, wsb, N, K, H, W, D, s_rgb, s_xy, xy, nullptr) == TCAM_OK)
        (void)hipMemcpy(outs, dout, sizeof(float) * N * K * P, hipMemcpyDeviceToHost);
    (void)hipFree(di);
    (void)hipFree(dn);
    (void)hipFree(dout);
    (void)hipFree(ws);
}

}  // namespace

extern "C" size_t tcam_bilateral_ws_bytes(int N, int K, int H, int W, int dim) {
    return ws_bytes_for(N, K, H, W, dim);
}

extern "C" int tcam_bilateral_batch(const float* images, const float* ins, float* outs, void* ws,
                                    size_t ws_bytes, int N, int K, int H, int W, float s_rgb,
                                    float s_xy, void* stream) {
    return dispatch(images, ins, outs, ws, ws_bytes, N, K, H, W, 5, s_rgb, s_xy, 1, stream);
}

extern "C" int tcam_colorbilateral_batch(const float* images, const float* ins, float* outs,
                                         void* ws, size_t ws_bytes, int N, int K, int H, int W,
                                         float s_rgb, int dim, void* stream) {
    if (dim < 1 || dim > 3) return TCAM_E_ARG;
    return dispatch(images, ins, outs, ws, ws_bytes, N, K, H, W, dim, s_rgb, 1.f, 0, stream);
}

extern "C" int tcam_bilateral_status(const void* ws, int N, int* status) {
    if (!ws || N <= 0 || !status) return TCAM_E_ARG;
    // err lives right after M[N] in the header block.
    return (int)hipMemcpy(status, (const int*)ws + N, sizeof(int), hipMemcpyDeviceToHost);
}

extern "C" void bilateralfilter_batch(float* images, int len_images, float* ins, int len_ins,
                                      float* outs, int len_outs, int N, int K, int H, int W,
                                      float sigmargb, float sigmaxy) {
    (void)len_images; (void)len_ins; (void)len_outs;
    host_compat(images, ins, outs, N, K, H, W, 5, sigmargb, sigmaxy, 1);
}

extern "C" void colorbilateralfilter_batch(float* images, int len_images, float* ins,
                                           int len_ins, float* outs, int len_outs, int N,
                                           int K, int H, int W, float sigmargb, int DIM) {
    (void)len_images; (void)len_ins; (void)len_outs;
    if (DIM < 1 || DIM > 3) return;
    host_compat(images, ins, outs, N, K, H, W, DIM, sigmargb, 1.f, 0);
}

// ------------------------------------------------------------- CRF loss
// DenseCRFLossFunction.forward / backward (crf/dense_crf_loss.py:33-77):
//   loss = -sum(seg * AS) / N          grad_seg = -2 * g * AS / N
// Deterministic two-stage reduction: per-block partial sums (fixed order) into
// part[], then one block sums the partials in index order.
namespace {
constexpr int kRedBlock = 256;
constexpr int kRedGrid = 1024;

__global__ __launch_bounds__(kRedBlock) void energy_partial_kernel(const float* seg,
                                                                   const float* as, long n,
                                                                   float* part) {
    float acc = 0.f;
    for (long i = (long)blockIdx.x * kRedBlock + threadIdx.x; i < n;
         i += (long)kRedGrid * kRedBlock)
        acc += seg[i] * as[i];
    acc = wave_sum(acc);
    __shared__ float red[kRedBlock / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kRedBlock / 64; ++w) s += red[w];
        part[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(kRedBlock) void energy_final_kernel(const float* part,
                                                                 float neg_inv_n, float* loss) {
    float acc = 0.f;
    for (int i = threadIdx.x; i < kRedGrid; i += kRedBlock) acc += part[i];
    acc = wave_sum(acc);
    __shared__ float red[kRedBlock / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kRedBlock / 64; ++w) s += red[w];
        loss[0] = s * neg_inv_n;
    }
}

__global__ __launch_bounds__(kRedBlock) void crf_grad_kernel(const float* as, const float* g,
                                                             float scale, float* grad, long n) {
    const long i = (long)blockIdx.x * kRedBlock + threadIdx.x;
    if (i >= n) return;
    grad[i] = scale * g[0] * as[i];
}
}  // namespace

extern "C" size_t tcam_crf_energy_ws_bytes(void) { return sizeof(float) * kRedGrid; }

extern "C" int tcam_crf_energy(const float* seg, const float* as, long n, int N, float* loss,
                               float* ws, void* stream) {
    TCAM_REQUIRE(seg && as && loss && ws && n > 0 && N > 0);
    hipStream_t st = as_stream(stream);
    energy_partial_kernel<<<kRedGrid, kRedBlock, 0, st>>>(seg, as, n, ws);
    TCAM_CHECK_LAUNCH();
    energy_final_kernel<<<1, kRedBlock, 0, st>>>(ws, -1.0f / (float)N, loss);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_crf_grad(const float* as, const float* grad_out, long n, int N, float* grad,
                             void* stream) {
    TCAM_REQUIRE(as && grad_out && grad && n > 0 && N > 0);
    crf_grad_kernel<<<cdiv(n, kRedBlock), kRedBlock, 0, as_stream(stream)>>>(
        as, grad_out, -2.0f / (float)N, grad, n);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
