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
// packed exactly into one 64-bit word (r + 1, (k_i - r)/(d+1)); 0 = empty slot.  The
// global hash-table slot holding a key is the vertex's identity (sort key n * Cap + slot),
// so no counter is ever shared: same-address atomics serialise at ~0.3 us each on this
// chip, and a per-image vertex counter or a CAS storm on a hot vertex costs milliseconds.
//
// Pipeline per call (N images of P = H*W points; P' = P + 1 when P % 4 != 0, the extra
// point being the SSE init's zero-feature padding, permutohedral.cpp:171-175, 258-264,
// whose vertices exist in the reference lattice; its entries carry the value 0, which
// adds +-0 at the end of each of its vertices' sums and changes nothing):
//   lattice  (point)    elevate, simplex, barycentric: keys + weights of E = N P' (d+1)
//                       entries, entry e = (n P' + p)(d+1) + r
//   dedupe   (tile)     4096 consecutive keys of an image deduplicated in an LDS table
//   merge    (image)    the tiles' distinct keys merged in an LDS table, each vertex then
//                       inserted once in the global table (lock-free CAS)
//   remap    (entry)    sort key = n * Cap + slot
//   sort                stable LSD radix sort of (vertex key, entry)          [hipCUB]
//   vertices (sorted)   run starts -> dense vertex ids, first entries, slot -> id (two
//                       passes over entry tiles around a scan of the tile counts)
//   products (entry)    bary * in, in sorted order
//   splat    (vertex)   sequential sum of the vertex's products (= point order)
//   blur x(d+1) (vertex) v + 0.5 (n1 + n2) along each lattice axis
//   slice    (point)    sum_r (w_r * alpha) * v, then out (N, K, H, W)
//   clear    (vertex)   empties the used table slots: the table is left all-zero
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr uint64_t kEmpty = 0;       // valid keys carry r + 1 >= 1 in their low bits
constexpr int kMaxK = 8;             // channels per call (TCAM uses K = 2)
constexpr int kBlock = 256;
constexpr int kInsBlock = 1024;
constexpr int kTileKeys = 4096;      // keys deduplicated together (one block)
constexpr int kLdsSlots = 8192;      // LDS dedupe table (64-bit keys) per block
constexpr int kPersist = 2048;       // blocks of the grid-stride per-vertex kernels
constexpr int kVBlock = 1024, kVPer = 8;   // vertex-boundary passes: threads, entries each
constexpr int kVTile = kVBlock * kVPer;

struct Geo {
    int N, K, H, W, P, D;
    int Pv;        // points per image incl. the virtual one
    long E;        // entries = N * Pv * (D + 1)
    int logCap;    // hash slots per image = 2^logCap >= 1.25 * Pv * (D + 1)
    int sortBits;  // bits of N << logCap
    long tiles;    // dedupe tiles per image
};

inline Geo make_geo(int N, int K, int H, int W, int D) {
    Geo g;
    g.N = N; g.K = K; g.H = H; g.W = W; g.P = H * W; g.D = D;
    g.Pv = g.P + ((g.P % 4) ? 1 : 0);
    g.E = (long)N * g.Pv * (D + 1);
    const long per = (long)g.Pv * (D + 1);
    // load factor <= 0.8 even if every entry were its own vertex (a CAM image has ~1 % of
    // that): linear probing stays short and a probe for an absent key meets an empty slot.
    // At 224^2 this is 2^19 slots, so 32 images sort on 24-bit keys: three 8-bit radix passes
    // (rocPRIM's onesweep digit on gfx950) instead of four for 2x the entries' bound
    g.logCap = 13;
    while ((1l << g.logCap) < per + per / 4) ++g.logCap;
    g.sortBits = g.logCap;
    while ((1l << g.sortBits) < ((long)N << g.logCap)) ++g.sortBits;
    g.tiles = (per + kTileKeys - 1) / kTileKeys;
    return g;
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout (offsets in bytes; every block 256-B aligned).  `slot` must be zero
// before the first call; every call leaves it zero.
struct Ws {
    size_t hdr, slot, cid, ekey, ukey, nuniq, lidx, uslot, skey, sval, skey2, sval2, bary,
        prod, vkey, vcnt, voff, v0, v1, tmp, total;
    size_t tmp_bytes;
};

Ws make_ws(const Geo& g, size_t tmp_bytes) {
    Ws w;
    size_t o = 0;
    const long cap = 1l << g.logCap;
    const long tk = (long)g.N * g.tiles * kTileKeys;
    w.hdr = o;   o += al(sizeof(int) * 64);                 // [0] err, [1] vertex count,
                                                            // [2] merge parts by fallback
    w.slot = o;  o += al(sizeof(uint64_t) * g.N * cap);
    w.cid = o;   o += al(sizeof(int) * g.N * cap);
    w.ekey = o;  o += al(sizeof(uint64_t) * g.E);
    w.ukey = o;  o += al(sizeof(uint64_t) * tk);
    w.nuniq = o; o += al(sizeof(int) * g.N * g.tiles);
    w.lidx = o;  o += al(sizeof(int) * tk);
    w.uslot = o; o += al(sizeof(int) * tk);
    w.skey = o;  o += al(sizeof(uint32_t) * g.E);
    w.sval = o;  o += al(sizeof(uint32_t) * g.E);
    w.skey2 = o; o += al(sizeof(uint32_t) * g.E);
    w.sval2 = o; o += al(sizeof(uint32_t) * g.E);
    w.bary = o;  o += al(sizeof(float) * g.E);
    w.prod = o;  o += al(sizeof(float) * g.E * g.K);
    w.vkey = o;  o += al(sizeof(uint32_t) * g.E);           // vertex -> n * Cap + slot
    w.vcnt = o;  o += al(sizeof(int) * 2 * ((g.E + kVTile - 1) / kVTile));   // tile counts, scan
    w.voff = o;  o += al(sizeof(int) * (g.E + 1));
    w.v0 = o;    o += al(sizeof(float) * g.E * g.K);
    w.v1 = o;    o += al(sizeof(float) * g.E * g.K);
    w.tmp = o;   o += al(tmp_bytes);
    w.tmp_bytes = tmp_bytes;
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
    uint64_t w = (uint64_t)(r + 1);
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
    r = (int)(w & 7) - 1;
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

// Global insert.  A slot changes at most once while a call runs (EMPTY -> key), so a
// plain (possibly stale, cached) probe is exact whenever it shows a key; only an EMPTY
// observation needs the CAS, whose return value is the slot's true content.
__device__ __forceinline__ int table_insert(uint64_t* tab, int logCap, uint64_t key) {
    const uint32_t mask = (1u << logCap) - 1;
    uint32_t h = hash_slot(key, logCap);
    while (true) {
        uint64_t cur = tab[h];
        if (cur == kEmpty) cur = atomicCAS((unsigned long long*)(tab + h), kEmpty, key);
        if (cur == kEmpty || cur == key) return (int)h;
        h = (h + 1) & mask;
    }
}

// Read-only probe (the table is complete: launched after the insert kernels).
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
    float xy_div;          // sigma_xy  (features divide, as the reference)
    float rgb_div;         // sigma_rgb
    float sf[5];           // scale_factor[i] (host-computed as permutohedral.cpp:164-166)
    float inv_dp1, dp1;    // 1.0f / (d+1), d+1
    uint32_t* sval;
    float* bary;
    int* err;
    int xy;                // 1: (x, y, r, g, b) features; 0: colour planes only
};

// Lattice point of one feature vector: the d+1 packed vertex keys and barycentric weights,
// in the reference's fp32 operation order (permutohedral.cpp:177-256, SSE branch).
template <int D>
__device__ __forceinline__ void point_lattice(const float (&f)[D], const LatticeArgs& a,
                                              uint64_t (&key)[D + 1], float (&bw)[D + 1],
                                              int* lerr) {
#pragma clang fp contract(off)
    // Elevate (181-189).
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
        key[r] = pack_key<D>(k, r, lerr);
        bw[r] = b[r];
    }
}

// Keys and weights of every entry (the virtual point's weights are stored too; its input
// value is 0).
template <int D>
__global__ __launch_bounds__(kBlock) void lattice_kernel(LatticeArgs a, uint64_t* ekey, Geo g) {
#pragma clang fp contract(off)
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (long)g.N * g.Pv) return;
    const int n = (int)(t / g.Pv);
    const int p = (int)(t - (long)n * g.Pv);
    float f[D];
    if (p < g.P) {
        const float* im = a.img + (long)n * 3 * g.P + p;
        if (a.xy) {
            const int y = p / g.W, x = p - y * g.W;
            f[0] = (float)x / a.xy_div;
            if (D > 1) f[1] = (float)y / a.xy_div;
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
    uint64_t key[D + 1];
    float bw[D + 1];
    int lerr = 0;
    point_lattice<D>(f, a, key, bw, &lerr);
    const long ebase = t * (D + 1);
#pragma unroll
    for (int r = 0; r <= D; ++r) {
        ekey[ebase + r] = key[r];
        a.sval[ebase + r] = (uint32_t)(ebase + r);
        a.bary[ebase + r] = bw[r];
    }
    if (lerr) atomicOr(a.err, 1);
}

// The tile's (<= kTileKeys) distinct keys, listed in ukey[tile][0, nuniq); each key
// records its index in that list.
__global__ __launch_bounds__(kInsBlock) void dedupe_kernel(const uint64_t* ekey, uint64_t* ukey,
                                                           int* nuniq, int* lidx, Geo g) {
    __shared__ uint64_t lkey[kLdsSlots];
    __shared__ int lpos[kLdsSlots];    // index of the LDS entry in the tile's list
    __shared__ int wsum[kInsBlock / 64];
    const long per_img = (long)g.Pv * (g.D + 1);
    const int n = (int)(blockIdx.x / g.tiles);
    const long k0 = (long)(blockIdx.x - n * g.tiles) * kTileKeys;
    for (int i = threadIdx.x; i < kLdsSlots; i += kInsBlock) lkey[i] = kEmpty;
    __syncthreads();
    constexpr int per = kTileKeys / kInsBlock;
    int where[per];
#pragma unroll
    for (int q = 0; q < per; ++q) {
        const long k = k0 + q * kInsBlock + threadIdx.x;
        where[q] = -1;
        if (k >= per_img) continue;
        const uint64_t key = ekey[(long)n * per_img + k];
        uint32_t h = hash_slot(key, 13);
        while (true) {   // <= kTileKeys distinct keys in 2x as many slots: terminates
            uint64_t cur = lkey[h];
            if (cur == kEmpty) cur = atomicCAS((unsigned long long*)&lkey[h], kEmpty, key);
            if (cur == kEmpty || cur == key) break;
            h = (h + 1) & (kLdsSlots - 1);
        }
        where[q] = (int)h;
    }
    __syncthreads();
    // Block-wide compaction of the occupied LDS slots into the tile's list.
    constexpr int sper = kLdsSlots / kInsBlock;
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < sper; ++q) cnt += lkey[threadIdx.x * sper + q] != kEmpty;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int c = incl - cnt;
    int tot = 0;
    for (int w = 0; w < kInsBlock / 64; ++w) {
        if (w < wv) c += wsum[w];
        tot += wsum[w];
    }
    uint64_t* uk = ukey + (long)blockIdx.x * kTileKeys;
#pragma unroll
    for (int q = 0; q < sper; ++q) {
        const int sl = threadIdx.x * sper + q;
        const uint64_t k = lkey[sl];
        if (k != kEmpty) {
            uk[c] = k;
            lpos[sl] = c++;
        }
    }
    if (threadIdx.x == 0) nuniq[blockIdx.x] = tot;
    __syncthreads();
    int* li = lidx + (long)blockIdx.x * kTileKeys;
#pragma unroll
    for (int q = 0; q < per; ++q)
        if (where[q] >= 0) li[q * kInsBlock + threadIdx.x] = lpos[where[q]];
}

// Image-level dedupe of the tiles' distinct keys, then ONE global insert per vertex.
// A vertex occurs in ~13 tiles of its image (TCAM sigmas, 224^2: ~40 k tile-distinct keys
// for ~3 k vertices per image), so inserting every tile's list globally costs ~13 probes
// of the same hot slots per vertex across the chip; here kMergeParts workgroups per image
// (each owning the keys of one hash part) merge the image's tile lists in an LDS table
// first.  A part with more than kMergeFill distinct keys (a table too full to probe
// cheaply) falls back to inserting its tile-distinct keys globally, the previous scheme
// (exact either way: the global slot is the vertex id).
constexpr int kMergeSlots = 12288;                    // LDS keys (96 KiB) + slots (48 KiB)
constexpr int kMergeFill = kMergeSlots * 3 / 4;
constexpr int kMergeParts = 8;

__device__ __forceinline__ uint64_t merge_mix(uint64_t w) {
    w ^= w >> 33;
    w *= 0xC2B2AE3D27D4EB4Full;
    w ^= w >> 29;
    return w;
}
__device__ __forceinline__ uint32_t merge_hash(uint64_t w) {
    return (uint32_t)((merge_mix(w) >> 32) % kMergeSlots);
}
__device__ __forceinline__ int merge_part(uint64_t w) {
    return (int)(merge_mix(w) & (kMergeParts - 1));
}

constexpr int kMergeTiles = 2048;   // tiles per image listed in LDS (224^2: 74)

__global__ __launch_bounds__(kInsBlock) void merge_kernel(const uint64_t* ukey, const int* nuniq,
                                                          int* uslot, uint64_t* slot,
                                                          int* nfallback, Geo g) {
    __shared__ uint64_t mkey[kMergeSlots];
    __shared__ int mslot[kMergeSlots];   // the global slot of each occupied LDS slot
    __shared__ int pre[kMergeTiles + 1]; // prefix of the image's tile list lengths
    __shared__ int fill, over;
    const int n = blockIdx.x / kMergeParts, part = blockIdx.x % kMergeParts;
    uint64_t* tab = slot + ((long)n << g.logCap);
    const long t0 = (long)n * g.tiles;
    const int nt = (int)min<long>(g.tiles, kMergeTiles);
    for (int i = threadIdx.x; i < kMergeSlots; i += kInsBlock) mkey[i] = kEmpty;
    if (threadIdx.x == 0) {
        fill = 0;
        over = g.tiles > kMergeTiles;   // (never at TCAM sizes) take the fallback
        int acc = 0;
        for (int t = 0; t < nt; ++t) {
            pre[t] = acc;
            acc += nuniq[t0 + t];
        }
        pre[nt] = acc;
    }
    __syncthreads();
    const int total = pre[nt];
    // item j of the image's concatenated tile lists -> its ukey index
    auto item = [&](int j) {
        int lo = 0, hi = nt;                 // pre[lo] <= j < pre[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (pre[mid] <= j) lo = mid; else hi = mid;
        }
        return (t0 + lo) * kTileKeys + (j - pre[lo]);
    };
    // pass 1: this part's keys of the image into the LDS table (loads 4 ahead)
    for (int j0 = 0; j0 < total && !over; j0 += 4 * kInsBlock) {
        uint64_t keys[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kInsBlock + threadIdx.x;
            keys[u] = j < total ? ukey[item(j)] : kEmpty;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t key = keys[u];
            if (key == kEmpty || merge_part(key) != part || over) continue;
            uint32_t h = merge_hash(key);
            while (true) {
                uint64_t cur = mkey[h];
                if (cur == kEmpty) {
                    cur = atomicCAS((unsigned long long*)&mkey[h], kEmpty, key);
                    if (cur == kEmpty && atomicAdd(&fill, 1) >= kMergeFill) over = 1;
                }
                if (cur == kEmpty || cur == key) break;
                if (++h == kMergeSlots) h = 0;
            }
        }
    }
    __syncthreads();
    if (over) {
        // fallback: this part's tile-distinct keys inserted globally one by one (the
        // previous scheme; counted in header word 2)
        if (threadIdx.x == 0) atomicAdd(nfallback, 1);
        for (long t = t0; t < t0 + g.tiles; ++t) {
            const int nu = nuniq[t];
            for (int i = threadIdx.x; i < nu; i += kInsBlock) {
                const uint64_t key = ukey[t * kTileKeys + i];
                if (merge_part(key) == part)
                    uslot[t * kTileKeys + i] = table_insert(tab, g.logCap, key);
            }
        }
        return;
    }
    // pass 2: each distinct key once into the global table
    for (int i = threadIdx.x; i < kMergeSlots; i += kInsBlock) {
        const uint64_t key = mkey[i];
        if (key != kEmpty) mslot[i] = table_insert(tab, g.logCap, key);
    }
    __syncthreads();
    // pass 3: the global slot of each of this part's tile-distinct keys
    for (int j0 = 0; j0 < total; j0 += 4 * kInsBlock) {
        uint64_t keys[4];
        long idx[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kInsBlock + threadIdx.x;
            idx[u] = j < total ? item(j) : -1;
            keys[u] = idx[u] >= 0 ? ukey[idx[u]] : kEmpty;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t key = keys[u];
            if (key == kEmpty || merge_part(key) != part) continue;
            uint32_t h = merge_hash(key);
            while (mkey[h] != key)
                if (++h == kMergeSlots) h = 0;
            uslot[idx[u]] = mslot[h];
        }
    }
}

__global__ __launch_bounds__(kBlock) void remap_kernel(const int* lidx, const int* uslot,
                                                       uint32_t* skey, Geo g) {
    const long e = (long)blockIdx.x * kBlock + threadIdx.x;
    if (e >= g.E) return;
    const long per_img = (long)g.Pv * (g.D + 1);
    const int n = (int)(e / per_img);
    const long k = e - n * per_img;
    const long tb = (n * g.tiles + k / kTileKeys) * kTileKeys;
    const int s = uslot[tb + lidx[tb + (k % kTileKeys)]];
    skey[e] = (uint32_t)(((long)n << g.logCap) + s);
}

// Vertices of the sorted entries (a vertex starts where the sort key changes), in two passes
// over tiles of kVTile entries: per-tile run-start counts, then — after a scan of the counts —
// each run start's dense vertex id: vkey[v] (n * Cap + slot), voff[v] (its first sorted
// entry), cid[slot] = v, and voff[nv] = E, *nv.  (Replaces a run-length encode, a scan over
// every entry and a slot -> id pass.)
__global__ __launch_bounds__(kVBlock) void vcount_kernel(const uint32_t* __restrict__ sk, long E,
                                                         int* __restrict__ tcnt) {
    __shared__ int red[kVBlock / 64];
    const int tid = threadIdx.x;
    const long i0 = (long)blockIdx.x * kVTile + (long)tid * kVPer;
    int c = 0;
#pragma unroll
    for (int q = 0; q < kVPer; ++q) {
        const long i = i0 + q;
        if (i < E && (i == 0 || sk[i] != sk[i - 1])) ++c;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kVBlock / 64; ++w) t += red[w];
        tcnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kVBlock) void vassign_kernel(const uint32_t* __restrict__ sk, long E,
                                                          const int* __restrict__ tscan,
                                                          int* __restrict__ nv,
                                                          uint32_t* __restrict__ vkey,
                                                          int* __restrict__ voff,
                                                          int* __restrict__ cid) {
    __shared__ int wsum[kVBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long i0 = (long)blockIdx.x * kVTile + (long)tid * kVPer;
    uint32_t k[kVPer];
    bool head[kVPer];
    int c = 0;
    uint32_t prev = (i0 > 0 && i0 - 1 < E) ? sk[i0 - 1] : 0u;
#pragma unroll
    for (int q = 0; q < kVPer; ++q) {
        const long i = i0 + q;
        k[q] = i < E ? sk[i] : 0u;
        head[q] = i < E && (i == 0 || k[q] != prev);
        c += head[q];
        prev = k[q];
    }
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int v = tscan[blockIdx.x] + incl - c;
    for (int q = 0; q < w; ++q) v += wsum[q];
#pragma unroll
    for (int q = 0; q < kVPer; ++q) {
        const long i = i0 + q;
        if (head[q]) {
            vkey[v] = k[q];
            voff[v] = (int)i;
            cid[k[q]] = v;
            ++v;
        }
        if (i == E - 1) {
            *nv = v;
            voff[v] = (int)E;
        }
    }
}

// Splat, in two exact steps (permutohedral.cpp:413-421: values[o] += w * val, no fusion):
//   products  (sorted entry)  prod[i][k] = bary[e] * in[k][p(e)]   (the same fp32 product)
//   splat     (vertex)        values[v][k] = 0 + prod[i0][k] + prod[i0+1][k] + ...
// The serial sum streams its vertex's contiguous products, so its loads do not depend on
// each other or on the sum and pipeline freely.
__global__ __launch_bounds__(kBlock) void products_kernel(const float* in, const uint32_t* sval2,
                                                          const float* bary, float* prod, Geo g) {
#pragma clang fp contract(off)
    const long i = (long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= g.E) return;
    const uint32_t e = sval2[i];
    const float w = bary[e];
    const long pt = e / (g.D + 1);          // n * Pv + p
    const int n = (int)(pt / g.Pv);
    const int p = (int)(pt - (long)n * g.Pv);
    const float* src = in + (long)n * g.K * g.P + p;
#pragma unroll
    for (int k = 0; k < kMaxK; ++k)
        if (k < g.K) prod[i * g.K + k] = w * (p < g.P ? src[(long)k * g.P] : 0.f);
}

template <int K>
__global__ __launch_bounds__(kBlock) void splat_kernel(const float* prod, const int* voff,
                                                       const int* nv, float* vals) {
#pragma clang fp contract(off)
    const int nvert = *nv;
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < nvert; v += gridDim.x * kBlock) {
        const int i0 = voff[v], i1 = voff[v + 1];
        float acc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = 0.f;
        const float* pp = prod + (long)i0 * K;
        int i = i0;
        for (; i + 4 <= i1; i += 4, pp += 4 * K) {
            float t[4][K];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k) t[u][k] = pp[u * K + k];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k) acc[k] += t[u][k];
        }
        for (; i < i1; ++i, pp += K)
#pragma unroll
            for (int k = 0; k < K; ++k) acc[k] += pp[k];
#pragma unroll
        for (int k = 0; k < K; ++k) vals[(long)v * K + k] = acc[k];
    }
}

// One blur pass along lattice axis j (permutohedral.cpp:425-441).
template <int D, int K>
__global__ __launch_bounds__(kBlock) void blur_kernel(const uint64_t* slot, const int* cid,
                                                      const uint32_t* vkey, const int* nv,
                                                      const float* old, float* nw, int j,
                                                      Geo g) {
#pragma clang fp contract(off)
    const int nvert = *nv;
    const uint32_t mask = (1u << g.logCap) - 1;
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < nvert; v += gridDim.x * kBlock) {
        const uint32_t vk = vkey[v];
        const long tbase = (long)(vk >> g.logCap) << g.logCap;   // image n's table
        const uint64_t* tab = slot + tbase;
        int k[D], r;
        unpack_key<D>(tab[vk & mask], k, r);
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
        const long o1 = h1 >= 0 ? cid[tbase + h1] : -1;
        const long o2 = h2 >= 0 ? cid[tbase + h2] : -1;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const float a = o1 >= 0 ? old[o1 * K + q] : 0.f;
            const float b = o2 >= 0 ? old[o2 * K + q] : 0.f;
            nw[(long)v * K + q] = old[(long)v * K + q] + 0.5f * (a + b);
        }
    }
}

// out[n][k][p] = sum_r (bary_r * alpha) * vals[vertex_r][k]   (permutohedral.cpp:446-456).
template <int D, int K>
__global__ __launch_bounds__(kBlock) void slice_kernel(const uint32_t* skey, const int* cid,
                                                       const float* bary, const float* vals,
                                                       float alpha, float* out, Geo g) {
#pragma clang fp contract(off)
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (long)g.N * g.P) return;
    const int n = (int)(t / g.P);
    const int p = (int)(t - (long)n * g.P);
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.f;
    const long ebase = ((long)n * g.Pv + p) * (D + 1);
#pragma unroll
    for (int r = 0; r <= D; ++r) {
        const float w = bary[ebase + r] * alpha;
        const long v = cid[skey[ebase + r]];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += w * vals[v * K + k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) out[((long)n * K + k) * g.P + p] = acc[k];
}

// Leaves the table all-zero for the next call: clears exactly the slots this call used.
__global__ __launch_bounds__(kBlock) void clear_kernel(uint64_t* slot, const uint32_t* vkey,
                                                       const int* nv) {
    const int n = *nv;
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < n; v += gridDim.x * kBlock)
        slot[vkey[v]] = kEmpty;
}

size_t tmp_bytes_for(const Geo& g) {
    size_t a = 0, b = 0, c = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)g.E, 0, g.sortBits,
                                           (hipStream_t)0) != hipSuccess)
        return 0;
    const int nt = (int)((g.E + kVTile - 1) / kVTile);
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int*)nullptr, (int*)nullptr, nt,
                                         (hipStream_t)0) != hipSuccess)
        return 0;
    return std::max(a, std::max(b, c));
}

bool valid_dims(int N, int K, int H, int W, int D) {
    if (N <= 0 || K <= 0 || K > kMaxK || H <= 0 || W <= 0) return false;
    if (D < 1 || D > 5) return false;
    if ((long)H * W > (1l << 26)) return false;
    const Geo g = make_geo(N, K, H, W, D);
    // Entry indices and vertex keys are 32-bit.
    return g.E < (1l << 31) && g.sortBits <= 32;
}

// The reference's per-lattice constants (permutohedral.cpp:160-166, 444): computed in
// double and rounded to float exactly as the SSE init does.
void lattice_constants(int D, float* sf, float* alpha) {
    const float inv_std_dev = (float)(std::sqrt(2.0 / 3.0) * (D + 1));
    for (int i = 0; i < D; ++i)
        sf[i] = (float)(1.0 / std::sqrt((double)((i + 2) * (i + 1))) * (double)inv_std_dev);
    *alpha = 1.0f / (1 + powf(2, -D));
}

constexpr int kBoth = 0, kPrepare = 1, kApply = 2;

template <int D, int K>
int apply(const float* ins, float* outs, void* ws, const Geo& g, hipStream_t st);

// Phase 1 (depends on the images only): lattice, dedupe, merge, sort, vertices; then (phase
// kBoth) phase 2.  A caller may run phase 1 ahead, e.g. on a side stream while the network
// producing the values runs, and phase 2 later (tcam_bilateral_prepare / _apply).
template <int D, int K>
int run(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
        const Geo& g, float s_rgb, float s_xy, int xy, hipStream_t st, int phase) {
    const size_t tmpb = tmp_bytes_for(g);
    if (tmpb == 0) return TCAM_E_ARG;
    const Ws w = make_ws(g, tmpb);
    if (!ws || ws_bytes < w.total) return TCAM_E_NOMEM;
    char* base = (char*)ws;
    int* hdr = (int*)(base + w.hdr);
    int* err = hdr;
    int* nv = hdr + 1;
    uint64_t* slot = (uint64_t*)(base + w.slot);
    int* cid = (int*)(base + w.cid);
    uint64_t* ekey = (uint64_t*)(base + w.ekey);
    uint64_t* ukey = (uint64_t*)(base + w.ukey);
    int* nuniq = (int*)(base + w.nuniq);
    int* lidx = (int*)(base + w.lidx);
    int* uslot = (int*)(base + w.uslot);
    uint32_t* skey = (uint32_t*)(base + w.skey);
    uint32_t* sval = (uint32_t*)(base + w.sval);
    uint32_t* skey2 = (uint32_t*)(base + w.skey2);
    uint32_t* sval2 = (uint32_t*)(base + w.sval2);
    float* bary = (float*)(base + w.bary);
    float* prod = (float*)(base + w.prod);
    uint32_t* vkey = (uint32_t*)(base + w.vkey);
    int* vcnt = (int*)(base + w.vcnt);
    int* voff = (int*)(base + w.voff);
    float* v0 = (float*)(base + w.v0);
    float* v1 = (float*)(base + w.v1);
    void* tmp = base + w.tmp;

    hipError_t e;
    if ((e = hipMemsetAsync(hdr, 0, sizeof(int) * 64, st)) != hipSuccess) return e;
    LatticeArgs a;
    a.img = images;
    a.xy_div = s_xy;
    a.rgb_div = s_rgb;
    float alpha;
    lattice_constants(D, a.sf, &alpha);
    a.inv_dp1 = 1.0f / (D + 1);
    a.dp1 = (float)(D + 1);
    a.sval = sval;
    a.bary = bary;
    a.err = err;
    a.xy = xy;
    lattice_kernel<D><<<cdiv((long)g.N * g.Pv, kBlock), kBlock, 0, st>>>(a, ekey, g);
    TCAM_CHECK_LAUNCH();
    const int ntiles = (int)(g.N * g.tiles);
    dedupe_kernel<<<ntiles, kInsBlock, 0, st>>>(ekey, ukey, nuniq, lidx, g);
    TCAM_CHECK_LAUNCH();
    merge_kernel<<<g.N * kMergeParts, kInsBlock, 0, st>>>(ukey, nuniq, uslot, slot, hdr + 2, g);
    TCAM_CHECK_LAUNCH();
    remap_kernel<<<cdiv(g.E, kBlock), kBlock, 0, st>>>(lidx, uslot, skey, g);
    TCAM_CHECK_LAUNCH();
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, skey, skey2, sval, sval2, (int)g.E, 0,
                                                g.sortBits, st)) != hipSuccess)
        return e;
    const int nvt = (int)((g.E + kVTile - 1) / kVTile);
    int* tcnt = vcnt;
    int* tscan = vcnt + nvt;
    vcount_kernel<<<nvt, kVBlock, 0, st>>>(skey2, g.E, tcnt);
    TCAM_CHECK_LAUNCH();
    tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, tcnt, tscan, nvt, st)) != hipSuccess)
        return e;
    vassign_kernel<<<nvt, kVBlock, 0, st>>>(skey2, g.E, tscan, nv, vkey, voff, cid);
    TCAM_CHECK_LAUNCH();
    if (phase == kPrepare) return TCAM_OK;
    return apply<D, K>(ins, outs, ws, g, st);
}

// Phase 2 (depends on the values): products, splat, blur, slice, clear.  Consumes the
// lattice phase 1 left in `ws` (once: the clear empties the table again).
template <int D, int K>
int apply(const float* ins, float* outs, void* ws, const Geo& g, hipStream_t st) {
    const Ws w = make_ws(g, tmp_bytes_for(g));
    char* base = (char*)ws;
    int* hdr = (int*)(base + w.hdr);
    int* nv = hdr + 1;
    uint64_t* slot = (uint64_t*)(base + w.slot);
    int* cid = (int*)(base + w.cid);
    uint32_t* skey = (uint32_t*)(base + w.skey);
    uint32_t* sval2 = (uint32_t*)(base + w.sval2);
    float* bary = (float*)(base + w.bary);
    float* prod = (float*)(base + w.prod);
    uint32_t* vkey = (uint32_t*)(base + w.vkey);
    int* voff = (int*)(base + w.voff);
    float* v0 = (float*)(base + w.v0);
    float* v1 = (float*)(base + w.v1);
    float sf[5], alpha;
    lattice_constants(D, sf, &alpha);
    products_kernel<<<cdiv(g.E, kBlock), kBlock, 0, st>>>(ins, sval2, bary, prod, g);
    TCAM_CHECK_LAUNCH();
    splat_kernel<K><<<kPersist, kBlock, 0, st>>>(prod, voff, nv, v0);
    TCAM_CHECK_LAUNCH();
    float* cur = v0;
    float* nxt = v1;
    for (int j = 0; j <= D; ++j) {
        blur_kernel<D, K><<<kPersist, kBlock, 0, st>>>(slot, cid, vkey, nv, cur, nxt, j, g);
        TCAM_CHECK_LAUNCH();
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    slice_kernel<D, K><<<cdiv((long)g.N * g.P, kBlock), kBlock, 0, st>>>(skey, cid, bary, cur,
                                                                          alpha, outs, g);
    TCAM_CHECK_LAUNCH();
    clear_kernel<<<kPersist, kBlock, 0, st>>>(slot, vkey, nv);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <int D>
int run_k(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
          const Geo& g, float s_rgb, float s_xy, int xy, hipStream_t st, int phase) {
    switch (g.K) {
#define RUN_K(KK) \
        case KK: return phase == kApply ? apply<D, KK>(ins, outs, ws, g, st) \
                                        : run<D, KK>(images, ins, outs, ws, ws_bytes, g, s_rgb, \
                                                     s_xy, xy, st, phase);
        RUN_K(1) RUN_K(2) RUN_K(3) RUN_K(4) RUN_K(5) RUN_K(6) RUN_K(7) RUN_K(8)
#undef RUN_K
        default: return TCAM_E_ARG;
    }
}

int dispatch(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
             int N, int K, int H, int W, int D, float s_rgb, float s_xy, int xy, void* stream,
             int phase = kBoth) {
    if (!valid_dims(N, K, H, W, D)) return TCAM_E_ARG;
    if (phase != kApply && !images) return TCAM_E_ARG;
    if (phase != kPrepare && (!ins || !outs)) return TCAM_E_ARG;
    if (!(s_rgb > 0.f) || (xy && !(s_xy > 0.f))) return TCAM_E_ARG;
    const Geo g = make_geo(N, K, H, W, D);
    if (!ws || ws_bytes < make_ws(g, tmp_bytes_for(g)).total) return TCAM_E_NOMEM;
    hipStream_t st = as_stream(stream);
    switch (D) {
#define RUN_D(DD) \
        case DD: return run_k<DD>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st, phase);
        RUN_D(1) RUN_D(2) RUN_D(3) RUN_D(4)
#undef RUN_D
        default: return run_k<5>(images, ins, outs, ws, ws_bytes, g, s_rgb, s_xy, xy, st, phase);
    }
}

size_t ws_bytes_for(int N, int K, int H, int W, int D) {
    if (!valid_dims(N, K, H, W, D)) return 0;
    const Geo g = make_geo(N, K, H, W, D);
    const size_t tmpb = tmp_bytes_for(g);
    if (tmpb == 0) return 0;
    return make_ws(g, tmpb).total;
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
        hipMalloc(&ws, wsb) == hipSuccess && hipMemset(ws, 0, wsb) == hipSuccess &&
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

extern "C" int tcam_bilateral_prepare(const float* images, void* ws, size_t ws_bytes, int N,
                                      int K, int H, int W, float s_rgb, float s_xy,
                                      void* stream) {
    return dispatch(images, nullptr, nullptr, ws, ws_bytes, N, K, H, W, 5, s_rgb, s_xy, 1,
                    stream, kPrepare);
}

extern "C" int tcam_bilateral_apply(const float* ins, float* outs, void* ws, size_t ws_bytes,
                                    int N, int K, int H, int W, float s_rgb, float s_xy,
                                    void* stream) {
    return dispatch(nullptr, ins, outs, ws, ws_bytes, N, K, H, W, 5, s_rgb, s_xy, 1, stream,
                    kApply);
}

extern "C" int tcam_colorbilateral_batch(const float* images, const float* ins, float* outs,
                                         void* ws, size_t ws_bytes, int N, int K, int H, int W,
                                         float s_rgb, int dim, void* stream) {
    if (dim < 1 || dim > 3) return TCAM_E_ARG;
    return dispatch(images, ins, outs, ws, ws_bytes, N, K, H, W, dim, s_rgb, 1.f, 0, stream);
}

extern "C" int tcam_bilateral_status(const void* ws, int N, int* status) {
    if (!ws || N <= 0 || !status) return TCAM_E_ARG;
    // err is the first word of the header block.
    return (int)hipMemcpy(status, ws, sizeof(int), hipMemcpyDeviceToHost);
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
