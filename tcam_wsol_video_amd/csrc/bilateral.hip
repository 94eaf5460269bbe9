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
//     point order — the reference's order (permutohedral.cpp:413-421);
//   * blur and slice are per-vertex / per-point in the reference's order.
// Vertex numbering differs from the reference's hash order (and between runs), but
// no output depends on it.
//
// Lattice keys: d coordinates, all congruent to the vertex remainder r mod (d+1),
// packed exactly into one 64-bit word (r + 1, (k_i - r)/(d+1)); 0 = empty slot.  The
// global hash-table slot holding a key is the vertex's identity.
//
// Runs.  Neighbouring pixels mostly share their simplex: along a row the vertex of
// remainder r changes every few to tens of pixels (TCAM sigmas: a lattice cell spans
// ~25 pixels of x).  A wave holds 64 consecutive points of one image; for each r, the
// lanes where the vertex changes (shuffle compare) start a PIECE (head point, length
// <= 64).  Only piece heads probe the global hash table, and the vertex sums are formed
// from pieces: a vertex's entries in point order are its pieces in point order, each a
// contiguous stretch of points.  So the stable sort that groups entries by vertex sorts
// pieces — ~10-25x fewer items than entries — not entries.
//
// Pipeline per call (N images of P = H*W points; P' = P + 1 when P % 4 != 0, the extra
// point being the SSE init's zero-feature padding, permutohedral.cpp:171-175, 258-264,
// whose vertices exist in the reference lattice; its entries carry the value 0, which
// adds +-0 at the end of each of its vertices' sums and changes nothing):
//   lattice   (point, wave)  elevate, simplex, barycentric; per r the wave's pieces: heads
//                            insert their key (lock-free CAS), every entry gets its vertex
//                            slot; pieces (slot key, point << 6 | len - 1) listed per wave;
//                            the block's histogram of sort digit 0
//   sort      LSD radix sort of the pieces by (image, slot), 8-bit digits, stable: per
//             pass a block histogram, a scan (hipCUB), a stable scatter (per-wave digit
//             ranks by ballots, wave offsets through LDS).  The piece count is known on the
//             device only, so the grids cover the capacity and idle blocks exit: no host
//             synchronisation.  Pass 1 reads the lattice blocks' per-wave lists directly.
//   vertices  (sorted piece)  run starts -> dense vertex id, start offset, slot -> id
//   splat     (vertex)   sequential sum of bary * in over the vertex's pieces' points
//   blur x(d+1) (vertex) v + 0.5 (n1 + n2) along each lattice axis
//   slice     (point)    sum_r (w_r * alpha) * v, then out (N, K, H, W)
//   clear     (vertex)   empties the used table slots: the table is left all-zero
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr uint64_t kEmpty = 0;       // valid keys carry r + 1 >= 1 in their low bits
constexpr int kMaxK = 8;             // channels per call (TCAM uses K = 2)
constexpr int kBlock = 256;
constexpr int kPersist = 2048;       // blocks of the grid-stride per-vertex kernels
constexpr int kLatWaves = 16;        // waves per lattice block (= one pass-1 sort tile)
constexpr int kLatBlock = 64 * kLatWaves;
constexpr int kSortBlock = 1024;
constexpr int kSortWaves = kSortBlock / 64;
constexpr int kSortTile = 8 * kSortBlock;    // items per dense sort tile (8 rounds)
constexpr int kVtxPer = kSortTile / kSortBlock;
constexpr int kLenBits = 6;          // piece value: point << 6 | (length - 1), length <= 64
constexpr long kMaxPoints = 1l << (32 - kLenBits);   // points (incl. virtual) per launch

struct Geo {
    int N, K, H, W, P, D;
    int Pv;        // points per image incl. the virtual one
    long E;        // entries = N * Pv * (D + 1)
    int logCap;    // hash slots per image = 2^logCap >= 1.25 * Pv * (D + 1)
    int sortBits;  // bits of N << logCap
    int passes;    // 8-bit LSD passes
    int nwav;      // waves (64 points) per image
    long NWV;      // waves per call
    int G1;        // lattice blocks = pass-1 tiles
    long Mc;       // piece capacity: NWV * 64 * (D + 1)
    int Gd;        // dense sort tiles over Mc
};

inline Geo make_geo(int N, int K, int H, int W, int D) {
    Geo g;
    g.N = N; g.K = K; g.H = H; g.W = W; g.P = H * W; g.D = D;
    g.Pv = g.P + ((g.P % 4) ? 1 : 0);
    g.E = (long)N * g.Pv * (D + 1);
    const long per = (long)g.Pv * (D + 1);
    // load factor <= 0.8 even if every entry were its own vertex: linear probing ends, and a
    // table_find of an absent key meets an empty slot
    g.logCap = 13;
    while ((1l << g.logCap) < per + per / 4) ++g.logCap;
    g.sortBits = g.logCap;
    while ((1l << g.sortBits) < ((long)N << g.logCap)) ++g.sortBits;
    g.passes = (g.sortBits + 7) / 8;
    g.nwav = (g.Pv + 63) / 64;
    g.NWV = (long)N * g.nwav;
    g.G1 = (int)((g.NWV + kLatWaves - 1) / kLatWaves);
    g.Mc = g.NWV * 64 * (D + 1);
    g.Gd = (int)((g.Mc + kSortTile - 1) / kSortTile);
    return g;
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout (offsets in bytes; every block 256-B aligned).  `slot` must be zero
// before the first call; every call leaves it zero.
struct Ws {
    size_t hdr, slot, cid, skey, bary, wcnt, pk0, pv0, pk1, pv1, pk2, pv2, hist, hscan, tcnt,
        tscan, vstart, vkey, v0, v1, tmp, total;
    size_t tmp_bytes;
};

Ws make_ws(const Geo& g, size_t tmp_bytes) {
    Ws w;
    size_t o = 0;
    const long cap = 1l << g.logCap;
    const long hn = 256l * std::max<long>(g.G1, g.Gd);
    w.hdr = o;    o += al(sizeof(int) * 64);    // [0] err, [1] vertices, [2] pieces
    w.slot = o;   o += al(sizeof(uint64_t) * g.N * cap);
    w.cid = o;    o += al(sizeof(int) * g.N * cap);
    w.skey = o;   o += al(sizeof(uint32_t) * g.E);      // entry -> n * Cap + slot
    w.bary = o;   o += al(sizeof(float) * g.E);
    w.wcnt = o;   o += al(sizeof(int) * g.NWV);          // pieces per wave
    w.pk0 = o;    o += al(sizeof(uint32_t) * g.Mc);      // per-wave piece lists
    w.pv0 = o;    o += al(sizeof(uint32_t) * g.Mc);
    w.pk1 = o;    o += al(sizeof(uint32_t) * g.Mc);      // sort ping-pong
    w.pv1 = o;    o += al(sizeof(uint32_t) * g.Mc);
    w.pk2 = o;    o += al(sizeof(uint32_t) * g.Mc);
    w.pv2 = o;    o += al(sizeof(uint32_t) * g.Mc);
    w.hist = o;   o += al(sizeof(int) * hn);
    w.hscan = o;  o += al(sizeof(int) * hn);
    w.tcnt = o;   o += al(sizeof(int) * g.Gd);
    w.tscan = o;  o += al(sizeof(int) * g.Gd);
    w.vstart = o; o += al(sizeof(int) * (g.Mc + 1));     // vertex -> first sorted piece
    w.vkey = o;   o += al(sizeof(uint32_t) * g.Mc);      // vertex -> n * Cap + slot
    w.v0 = o;     o += al(sizeof(float) * g.Mc * g.K);
    w.v1 = o;     o += al(sizeof(float) * g.Mc * g.K);
    w.tmp = o;    o += al(tmp_bytes);
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

struct RunArgs {
    uint64_t* slot;     // hash tables, N x 2^logCap
    uint32_t* skey;     // entry -> n * Cap + slot
    uint32_t* pk;       // per-wave piece lists: key n * Cap + slot
    uint32_t* pv;       //                       point << 6 | (length - 1)
    int* wcnt;          // pieces per wave
    int* hist;          // pass-1 digit histogram, digit-major (256 x G1)
};

// Keys, weights, vertex slots and pieces of 64 consecutive points per wave (see the
// header).  Lanes past the image's last point (incl. the virtual one) are inactive.
template <int D>
__global__ __launch_bounds__(kLatBlock) void lattice_runs_kernel(LatticeArgs a, RunArgs ra,
                                                                 Geo g) {
#pragma clang fp contract(off)
    __shared__ int lh[256];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 256; i += kLatBlock) lh[i] = 0;
    __syncthreads();
    const long wv = (long)blockIdx.x * kLatWaves + (tid >> 6);
    const bool wvalid = wv < g.NWV;
    int n = 0, p = 0;
    if (wvalid) {
        n = (int)(wv / g.nwav);
        p = (int)(wv - (long)n * g.nwav) * 64 + lane;
    }
    const bool act = wvalid && p < g.Pv;
    float f[D];
    if (act && p < g.P) {
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
    const uint64_t am = __ballot(act);
    const int nact = __popcll(am);          // active lanes are a prefix of the wave
    const uint64_t lt = (1ull << lane) - 1;
    const uint64_t le = lt | (1ull << lane);
    uint64_t* tab = ra.slot + ((long)n << g.logCap);
    const long pt = (long)n * g.Pv + p;
    const long ebase = pt * (D + 1);
    const long rbase = wv * 64 * (D + 1);
    const uint32_t nbase = (uint32_t)((long)n << g.logCap);
    int woff = 0;
#pragma unroll
    for (int r = 0; r <= D; ++r) {
        const uint64_t k = key[r];
        const uint64_t kp = __shfl(k, lane > 0 ? lane - 1 : 0, 64);
        const bool head = act && (lane == 0 || k != kp);
        const uint64_t hm = __ballot(head);
        int s = 0;
        if (head) s = table_insert(tab, g.logCap, k);
        const uint64_t upto = hm & le;               // this lane's piece starts at the
        const int hl = upto ? 63 - __clzll(upto) : 0;  // highest head at or below it
        const int sl = __shfl(s, hl, 64);
        if (act) {
            ra.skey[ebase + r] = nbase + (uint32_t)sl;
            a.bary[ebase + r] = bw[r];
        }
        if (head) {
            const uint64_t above = hm & ~le;
            const int nxt = above ? __ffsll((long long)above) - 1 : nact;
            const int pos = woff + __popcll(hm & lt);
            const uint32_t k32 = nbase + (uint32_t)s;
            ra.pk[rbase + pos] = k32;
            ra.pv[rbase + pos] = (uint32_t)(pt << kLenBits) | (uint32_t)(nxt - lane - 1);
            atomicAdd(&lh[k32 & 255u], 1);
        }
        woff += __popcll(hm);
    }
    if (wvalid && lane == 0) ra.wcnt[wv] = woff;
    if (act && lerr) atomicOr(a.err, 1);
    __syncthreads();
    for (int d = tid; d < 256; d += kLatBlock) ra.hist[(long)d * g.G1 + blockIdx.x] = lh[d];
}

// Piece count of the call: the last bin of the scanned pass-1 histogram plus its count.
__device__ __forceinline__ long piece_count(const int* hscan, const int* hist, int G) {
    const long last = 255l * G + G - 1;
    return (long)hscan[last] + hist[last];
}

struct SortArgs {
    const uint32_t* ik;
    const uint32_t* iv;
    uint32_t* ok;
    uint32_t* ov;
    const int* hscan;   // scanned digit histogram of this pass (256 x G, digit-major)
    const int* wcnt;    // pass 1: pieces per wave (items = the lattice block's wave lists)
    int* hdr;           // pass 1 writes the piece count to hdr[2]; later passes read it
    const int* hist1;   // pass 1: its raw histogram (for the count)
    int G, shift;
    long NWV, R;        // waves, per-wave list stride
};

// Stable scatter of one LSD pass.  Items of tile b in order: round j, wave w, lane l hold
// item j * 1024 + 64 w + l.  A lane's rank among its wave's lanes of the same digit comes
// from 8 ballots; wave offsets per digit and the running offsets of the tile live in LDS
// (two count buffers alternate between rounds, so each round needs two barriers).
__global__ __launch_bounds__(kSortBlock) void sort_scatter_kernel(SortArgs s) {
    __shared__ int run[256];
    __shared__ int wc[2][kSortWaves][256];
    __shared__ int wpre[kLatWaves + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b = blockIdx.x;
    const bool sparse = s.wcnt != nullptr;
    long t0 = 0;
    int tn = 0;
    if (sparse) {
        if (tid == 0) {
            int acc = 0;
            for (int q = 0; q < kLatWaves; ++q) {
                wpre[q] = acc;
                const long wv = (long)b * kLatWaves + q;
                acc += wv < s.NWV ? s.wcnt[wv] : 0;
            }
            wpre[kLatWaves] = acc;
            if (b == 0) s.hdr[2] = (int)piece_count(s.hscan, s.hist1, s.G);
        }
    } else {
        const long M = __builtin_amdgcn_readfirstlane(s.hdr[2]);
        t0 = (long)b * kSortTile;
        if (t0 >= M) return;
        tn = (int)min<long>(kSortTile, M - t0);
    }
    if (tid < 256) run[tid] = s.hscan[(long)tid * s.G + b];
    for (int i = tid; i < 2 * kSortWaves * 256; i += kSortBlock) (&wc[0][0][0])[i] = 0;
    __syncthreads();
    if (sparse) tn = wpre[kLatWaves];
    tn = __builtin_amdgcn_readfirstlane(tn);
    const int nround = (tn + kSortBlock - 1) / kSortBlock;
    for (int j = 0; j < nround; ++j) {
        const int t = j * kSortBlock + tid;
        const bool valid = t < tn;
        uint32_t k = 0, v = 0;
        if (valid) {
            long src;
            if (sparse) {
                int q = 0;
                while (q + 1 < kLatWaves && wpre[q + 1] <= t) ++q;
                src = ((long)b * kLatWaves + q) * s.R + (t - wpre[q]);
            } else {
                src = t0 + t;
            }
            k = s.ik[src];
            v = s.iv[src];
        }
        const int d = (int)((k >> s.shift) & 255u);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool on = (d >> bit) & 1;
            const uint64_t bb = __ballot(on);
            peers &= on ? bb : ~bb;
        }
        const int rank = __popcll(peers & ((1ull << lane) - 1));
        const int buf = j & 1;
        if (valid && rank == 0) wc[buf][w][d] = __popcll(peers);
        __syncthreads();
        if (tid < 256) {   // digit tid: wave offsets of this round; clear the other buffer
            int acc = run[tid];
#pragma unroll
            for (int q = 0; q < kSortWaves; ++q) {
                const int c = wc[buf][q][tid];
                wc[buf][q][tid] = acc;
                acc += c;
                wc[buf ^ 1][q][tid] = 0;
            }
            run[tid] = acc;
        }
        __syncthreads();
        if (valid) {
            const int pos = wc[buf][w][d] + rank;
            s.ok[pos] = k;
            s.ov[pos] = v;
        }
    }
}

// Digit histogram of a dense pass (tiles past the piece count write zeros).
__global__ __launch_bounds__(kSortBlock) void sort_hist_kernel(const uint32_t* ik, const int* hdr,
                                                               int G, int shift, int* hist) {
    __shared__ int lh[256];
    const int tid = threadIdx.x, b = blockIdx.x;
    if (tid < 256) lh[tid] = 0;
    __syncthreads();
    const long M = __builtin_amdgcn_readfirstlane(hdr[2]);
    const long t0 = (long)b * kSortTile;
    const long t1 = min<long>(t0 + kSortTile, M);
    for (long t = t0 + tid; t < t1; t += kSortBlock) atomicAdd(&lh[(ik[t] >> shift) & 255u], 1);
    __syncthreads();
    if (tid < 256) hist[(long)tid * G + b] = lh[tid];
}

// Vertices of the sorted pieces: a vertex starts where the key changes.  Tile counts ...
__global__ __launch_bounds__(kSortBlock) void vertex_count_kernel(const uint32_t* sk,
                                                                  const int* hdr, int* tcnt) {
    __shared__ int red[kSortWaves];
    const int tid = threadIdx.x, b = blockIdx.x;
    const long M = __builtin_amdgcn_readfirstlane(hdr[2]);
    const long i0 = (long)b * kSortTile + (long)tid * kVtxPer;
    int c = 0;
#pragma unroll
    for (int q = 0; q < kVtxPer; ++q) {
        const long i = i0 + q;
        if (i < M && (i == 0 || sk[i] != sk[i - 1])) ++c;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int s = 0;
        for (int w = 0; w < kSortWaves; ++w) s += red[w];
        tcnt[b] = s;
    }
}

// ... then the dense vertex ids in sorted order: vstart[v], vkey[v], cid[slot] = v, the
// vertex count (hdr[1]) and vstart[count] = M.
__global__ __launch_bounds__(kSortBlock) void vertex_kernel(const uint32_t* sk, const int* tscan,
                                                            int* hdr, int* vstart, uint32_t* vkey,
                                                            int* cid) {
    __shared__ int wsum[kSortWaves];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, b = blockIdx.x;
    const long M = __builtin_amdgcn_readfirstlane(hdr[2]);
    const long i0 = (long)b * kSortTile + (long)tid * kVtxPer;
    if ((long)b * kSortTile >= M) return;
    uint32_t k[kVtxPer];
    int c = 0;
    uint32_t prev = i0 > 0 && i0 - 1 < M ? sk[i0 - 1] : 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < kVtxPer; ++q) {
        const long i = i0 + q;
        k[q] = i < M ? sk[i] : 0u;
        if (i < M && (i == 0 || k[q] != prev)) ++c;
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
    int v = tscan[b] + incl - c;
    for (int q = 0; q < w; ++q) v += wsum[q];
    prev = i0 > 0 && i0 - 1 < M ? sk[i0 - 1] : 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < kVtxPer; ++q) {
        const long i = i0 + q;
        if (i < M && (i == 0 || k[q] != prev)) {
            vstart[v] = (int)i;
            vkey[v] = k[q];
            cid[k[q]] = v;
            ++v;
        }
        if (i == M - 1) {
            hdr[1] = v;
            vstart[v] = (int)M;
        }
        prev = k[q];
    }
}

// Splat (permutohedral.cpp:413-421: values[o] += w * val, no fusion): the vertex's pieces in
// point order, each a stretch of consecutive points of remainder r.
template <int D, int K>
__global__ __launch_bounds__(kBlock) void splat_kernel(const uint64_t* slot, const int* vstart,
                                                       const uint32_t* vkey, const uint32_t* pv,
                                                       const float* bary, const float* in,
                                                       const int* hdr, float* vals, Geo g) {
#pragma clang fp contract(off)
    const int nvert = hdr[1];
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < nvert; v += gridDim.x * kBlock) {
        const uint32_t vk = vkey[v];
        const int r = (int)(slot[vk] & 7) - 1;
        const int n = (int)(vk >> g.logCap);
        const long pbase = (long)n * g.Pv;
        const float* src = in + (long)n * K * g.P;
        float acc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = 0.f;
        const int i1 = vstart[v + 1];
        for (int i = vstart[v]; i < i1; ++i) {
            const uint32_t val = pv[i];
            const long pt = val >> kLenBits;
            const int len = (int)(val & ((1u << kLenBits) - 1)) + 1;
            const float* bw = bary + pt * (D + 1) + r;
            const int p0 = (int)(pt - pbase);
            int q = 0;
            for (; q + 4 <= len; q += 4) {
                float t[4][K];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float wq = bw[(long)(q + u) * (D + 1)];
                    const int p = p0 + q + u;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        t[u][k] = wq * (p < g.P ? src[(long)k * g.P + p] : 0.f);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < K; ++k) acc[k] += t[u][k];
            }
            for (; q < len; ++q) {
                const float wq = bw[(long)q * (D + 1)];
                const int p = p0 + q;
#pragma unroll
                for (int k = 0; k < K; ++k) acc[k] += wq * (p < g.P ? src[(long)k * g.P + p] : 0.f);
            }
        }
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
    size_t a = 0;
    const long hn = 256l * std::max<long>(g.G1, g.Gd);
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int*)nullptr, (int*)nullptr, (int)hn,
                                         (hipStream_t)0) != hipSuccess)
        return 0;
    return std::max<size_t>(a, 256);
}

// points per launch (test hook tcam_bilateral_set_max_points lowers it to exercise the
// image-chunked dispatch at small sizes)
long g_max_points = kMaxPoints;

bool valid_geo(int N, int K, int H, int W, int D) {
    if (N <= 0 || K <= 0 || K > kMaxK || H <= 0 || W <= 0) return false;
    if (D < 1 || D > 5) return false;
    if ((long)H * W > (1l << 26)) return false;
    const Geo g = make_geo(N, K, H, W, D);
    // 32-bit entry / piece indices and keys, piece values point << 6
    return g.Mc < (1l << 31) && g.sortBits <= 32 && (long)N * g.Pv < g_max_points;
}

// Images per launch: the largest batch whose pieces and points fit the 32-bit encodings
// (the filter is per image, so consecutive launches over image chunks are exact).
int chunk_images(int N, int K, int H, int W, int D) {
    int lo = 0, hi = N;
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (valid_geo(mid, K, H, W, D)) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// The reference's per-lattice constants (permutohedral.cpp:160-166, 444): computed in
// double and rounded to float exactly as the SSE init does.
void lattice_constants(int D, float* sf, float* alpha) {
    const float inv_std_dev = (float)(std::sqrt(2.0 / 3.0) * (D + 1));
    for (int i = 0; i < D; ++i)
        sf[i] = (float)(1.0 / std::sqrt((double)((i + 2) * (i + 1))) * (double)inv_std_dev);
    *alpha = 1.0f / (1 + powf(2, -D));
}

// g: this launch's images; w: the workspace layout of the largest launch of the call (every
// launch of a call uses the same slot-table region, which each leaves all-zero)
template <int D, int K>
int run(const float* images, const float* ins, float* outs, void* ws, const Ws& w,
        const Geo& g, float s_rgb, float s_xy, int xy, hipStream_t st) {
    char* base = (char*)ws;
    int* hdr = (int*)(base + w.hdr);
    uint64_t* slot = (uint64_t*)(base + w.slot);
    int* cid = (int*)(base + w.cid);
    uint32_t* skey = (uint32_t*)(base + w.skey);
    float* bary = (float*)(base + w.bary);
    int* wcnt = (int*)(base + w.wcnt);
    uint32_t* pk[3] = {(uint32_t*)(base + w.pk0), (uint32_t*)(base + w.pk1),
                       (uint32_t*)(base + w.pk2)};
    uint32_t* pv[3] = {(uint32_t*)(base + w.pv0), (uint32_t*)(base + w.pv1),
                       (uint32_t*)(base + w.pv2)};
    int* hist = (int*)(base + w.hist);
    int* hscan = (int*)(base + w.hscan);
    int* tcnt = (int*)(base + w.tcnt);
    int* tscan = (int*)(base + w.tscan);
    int* vstart = (int*)(base + w.vstart);
    uint32_t* vkey = (uint32_t*)(base + w.vkey);
    float* v0 = (float*)(base + w.v0);
    float* v1 = (float*)(base + w.v1);
    void* tmp = base + w.tmp;

    hipError_t e;
    LatticeArgs a;
    a.img = images;
    a.xy_div = s_xy;
    a.rgb_div = s_rgb;
    float alpha;
    lattice_constants(D, a.sf, &alpha);
    a.inv_dp1 = 1.0f / (D + 1);
    a.dp1 = (float)(D + 1);
    a.bary = bary;
    a.err = hdr;
    a.xy = xy;
    RunArgs ra{slot, skey, pk[0], pv[0], wcnt, hist};
    lattice_runs_kernel<D><<<g.G1, kLatBlock, 0, st>>>(a, ra, g);
    TCAM_CHECK_LAUNCH();
    // radix sort of the pieces by (image, slot): pass 1 from the per-wave lists
    size_t tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, hist, hscan, 256 * g.G1, st)) !=
        hipSuccess)
        return e;
    SortArgs sa;
    sa.ik = pk[0]; sa.iv = pv[0]; sa.ok = pk[1]; sa.ov = pv[1];
    sa.hscan = hscan; sa.wcnt = wcnt; sa.hdr = hdr; sa.hist1 = hist;
    sa.G = g.G1; sa.shift = 0; sa.NWV = g.NWV; sa.R = 64l * (D + 1);
    sort_scatter_kernel<<<g.G1, kSortBlock, 0, st>>>(sa);
    TCAM_CHECK_LAUNCH();
    int cur = 1;
    for (int ps = 1; ps < g.passes; ++ps) {
        const int nxt = cur == 1 ? 2 : 1;
        sort_hist_kernel<<<g.Gd, kSortBlock, 0, st>>>(pk[cur], hdr, g.Gd, 8 * ps, hist);
        TCAM_CHECK_LAUNCH();
        tb = w.tmp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, hist, hscan, 256 * g.Gd, st)) !=
            hipSuccess)
            return e;
        SortArgs sd;
        sd.ik = pk[cur]; sd.iv = pv[cur]; sd.ok = pk[nxt]; sd.ov = pv[nxt];
        sd.hscan = hscan; sd.wcnt = nullptr; sd.hdr = hdr; sd.hist1 = nullptr;
        sd.G = g.Gd; sd.shift = 8 * ps; sd.NWV = 0; sd.R = 0;
        sort_scatter_kernel<<<g.Gd, kSortBlock, 0, st>>>(sd);
        TCAM_CHECK_LAUNCH();
        cur = nxt;
    }
    // vertices
    vertex_count_kernel<<<g.Gd, kSortBlock, 0, st>>>(pk[cur], hdr, tcnt);
    TCAM_CHECK_LAUNCH();
    tb = w.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, tcnt, tscan, g.Gd, st)) != hipSuccess)
        return e;
    vertex_kernel<<<g.Gd, kSortBlock, 0, st>>>(pk[cur], tscan, hdr, vstart, vkey, cid);
    TCAM_CHECK_LAUNCH();
    splat_kernel<D, K><<<kPersist, kBlock, 0, st>>>(slot, vstart, vkey, pv[cur], bary, ins, hdr,
                                                    v0, g);
    TCAM_CHECK_LAUNCH();
    int* nv = hdr + 1;
    float* vc = v0;
    float* vn = v1;
    for (int j = 0; j <= D; ++j) {
        blur_kernel<D, K><<<kPersist, kBlock, 0, st>>>(slot, cid, vkey, nv, vc, vn, j, g);
        TCAM_CHECK_LAUNCH();
        float* t = vc;
        vc = vn;
        vn = t;
    }
    slice_kernel<D, K><<<cdiv((long)g.N * g.P, kBlock), kBlock, 0, st>>>(skey, cid, bary, vc,
                                                                          alpha, outs, g);
    TCAM_CHECK_LAUNCH();
    clear_kernel<<<kPersist, kBlock, 0, st>>>(slot, vkey, nv);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

template <int D>
int run_k(const float* images, const float* ins, float* outs, void* ws, const Ws& w,
          const Geo& g, float s_rgb, float s_xy, int xy, hipStream_t st) {
    switch (g.K) {
#define RUN_K(KK) \
        case KK: return run<D, KK>(images, ins, outs, ws, w, g, s_rgb, s_xy, xy, st);
        RUN_K(1) RUN_K(2) RUN_K(3) RUN_K(4) RUN_K(5) RUN_K(6) RUN_K(7) RUN_K(8)
#undef RUN_K
        default: return TCAM_E_ARG;
    }
}

int dispatch(const float* images, const float* ins, float* outs, void* ws, size_t ws_bytes,
             int N, int K, int H, int W, int D, float s_rgb, float s_xy, int xy, void* stream) {
    if (!images || !ins || !outs) return TCAM_E_ARG;
    if (!(s_rgb > 0.f) || (xy && !(s_xy > 0.f))) return TCAM_E_ARG;
    const int nc = chunk_images(N, K, H, W, D);
    if (nc <= 0) return TCAM_E_ARG;
    hipStream_t st = as_stream(stream);
    const Geo gl = make_geo(nc, K, H, W, D);
    const size_t tmpb = tmp_bytes_for(gl);
    if (tmpb == 0) return TCAM_E_ARG;
    const Ws w = make_ws(gl, tmpb);
    if (!ws || ws_bytes < w.total) return TCAM_E_NOMEM;
    // header: [0] range error (kept over the chunks), [1] vertices, [2] pieces (last chunk)
    hipError_t e;
    if ((e = hipMemsetAsync(ws, 0, sizeof(int) * 64, st)) != hipSuccess) return e;
    const long P = (long)H * W;
    for (int n0 = 0; n0 < N; n0 += nc) {
        const int nb = std::min(nc, N - n0);
        const Geo g = make_geo(nb, K, H, W, D);
        const float* im = images + (long)n0 * 3 * P;
        const float* in = ins + (long)n0 * K * P;
        float* out = outs + (long)n0 * K * P;
        int rc;
        switch (D) {
            case 1: rc = run_k<1>(im, in, out, ws, w, g, s_rgb, s_xy, xy, st); break;
            case 2: rc = run_k<2>(im, in, out, ws, w, g, s_rgb, s_xy, xy, st); break;
            case 3: rc = run_k<3>(im, in, out, ws, w, g, s_rgb, s_xy, xy, st); break;
            case 4: rc = run_k<4>(im, in, out, ws, w, g, s_rgb, s_xy, xy, st); break;
            default: rc = run_k<5>(im, in, out, ws, w, g, s_rgb, s_xy, xy, st); break;
        }
        if (rc != TCAM_OK) return rc;
    }
    return TCAM_OK;
}

size_t ws_bytes_for(int N, int K, int H, int W, int D) {
    const int nc = chunk_images(N, K, H, W, D);
    if (nc <= 0) return 0;
    const Geo g = make_geo(nc, K, H, W, D);
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

extern "C" int tcam_colorbilateral_batch(const float* images, const float* ins, float* outs,
                                         void* ws, size_t ws_bytes, int N, int K, int H, int W,
                                         float s_rgb, int dim, void* stream) {
    if (dim < 1 || dim > 3) return TCAM_E_ARG;
    return dispatch(images, ins, outs, ws, ws_bytes, N, K, H, W, dim, s_rgb, 1.f, 0, stream);
}

extern "C" int tcam_bilateral_set_max_points(long n) {
    g_max_points = n > 0 && n < kMaxPoints ? n : kMaxPoints;
    return TCAM_OK;
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
