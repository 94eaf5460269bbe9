// CAM -> bbox on the GPU: a batched, exact replacement of
// compute_bboxes_from_scoremaps (metrics/wsol_metrics.py:127-197) with
// multi_contour_eval=False, i.e. for every threshold level L the box of
//   max(cv2.findContours(u8 > L, RETR_TREE, CHAIN_APPROX_SIMPLE), key=contourArea)
// followed by BoxEvaluator.accumulate (wsol_metrics.py:295-370).
//
// OpenCV semantics reproduced (contours.cpp, Suzuki-Abe border following on
// a zero-padded copy; contourArea = shoelace over the chain vertices):
//  * foreground is 8-connected, background 4-connected;
//  * the outer contour of a component C encloses C plus its holes, and its
//    shoelace area through pixel centres equals, summed over every 2x2
//    window of pixel centres, 1 if all four pixels lie in fill(C), 1/2 if
//    exactly three do, 0 otherwise;
//  * fill(C) of the top-level components are the 8-connected components of
//    {psi > L}, psi = grayscale hole-fill of u8 (min over 4-paths from the
//    image border of the max along the path);
//  * hole contours and contours nested in holes never win the max (strictly
//    smaller than their enclosing outer contour, and listed after it);
//  * ties between top-level contours resolve to the first in OpenCV's list
//    order = the LAST discovered in raster order = the largest raster index
//    of the component's first pixel;
//  * boundingRect of the outer contour = bbox of C.
// The oracle (oracle/contours.c, a restatement of the border follower) pins
// this characterisation on random images in tests/test_bbox_oracle.py.
//
// Kernels:
//  fill_kernel   one workgroup per frame: vmax = max(u8); psi by alternating
//                row/column min-max sweeps to the fixpoint; histogram of psi
//                -> the distinct levels (F_L only changes where psi = L + 1).
//  level_kernel  one workgroup per (frame, chunk of distinct levels): psi in
//                registers, per-level bitmap in LDS, block-based union-find
//                (2x2 pixel blocks, 8-connectivity), run-based window-area
//                accumulation into root slots, argmax with OpenCV's tie
//                order, bbox.
//  expand_kernel copies each canonical level's box to the levels it stands
//                for.
//  accumulate    one thread per (frame, tau): IoU vs GT (+1 inclusive
//                convention, fp64) and the BoxEvaluator counters.
#include "common.h"

namespace {

constexpr int MAXH = 256, MAXW = 256;
constexpr int MAXP = 260;                 // padded row pitch in bytes (pitch_of(256))
constexpr uint32_t INACT = 0xFFFFFFFFu;
constexpr int NTB = 1024;

__host__ __device__ inline int pitch_of(int W) {
    int d = (W + 3) / 4;
    if ((d & 1) == 0) d += 1;  // odd dword pitch: conflict-free column walks
    return 4 * d;
}

// Block-wide reductions over NTB threads (16 waves).
__device__ inline int block_max_i(int v, int* red) {
    v = wave_max_i(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = red[0];
        for (int i = 1; i < NTB / 64; ++i) m = max(m, red[i]);
        red[NTB / 64] = m;
    }
    __syncthreads();
    return red[NTB / 64];
}
__device__ inline int block_min_i(int v, int* red) {
    return -block_max_i(-v, red);
}

// ---------------------------------------------------------------- fill
__global__ __launch_bounds__(NTB) void fill_kernel(const uint8_t* __restrict__ cam_u8,
                                                   uint8_t* __restrict__ psi_out,
                                                   int32_t* __restrict__ vmax_out,
                                                   int32_t* __restrict__ canon,
                                                   int32_t* __restrict__ lev_list,
                                                   int32_t* __restrict__ nlev, int H, int W) {
    __shared__ uint8_t img[MAXH * MAXP];
    __shared__ uint8_t psi[MAXH * MAXP];
    __shared__ int red[NTB / 64 + 1];
    __shared__ int hist[257];
    __shared__ int changed;
    const int b = blockIdx.x;
    const int P = pitch_of(W);
    const uint8_t* src = cam_u8 + (long)b * H * W;
    int vm = 0;
    for (int i = threadIdx.x; i < H * W; i += NTB) {
        int y = i / W, x = i - y * W;
        uint8_t v = src[i];
        img[y * P + x] = v;
        psi[y * P + x] = 255;
        vm = max(vm, (int)v);
    }
    vm = block_max_i(vm, red);
    if (threadIdx.x == 0) vmax_out[b] = vm;
    // psi(p) = max(u8(p), min over 4-neighbours psi(q)), outside = -1.
    // Row sweeps (thread per row) alternate with column sweeps (thread per
    // column); each thread only reads/writes its own line, values only
    // decrease, and the loop stops after a full cycle without change.
    for (;;) {
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        int ch = 0;
        if (threadIdx.x < H) {
            uint8_t* row = psi + threadIdx.x * P;
            const uint8_t* irow = img + threadIdx.x * P;
            int prev = -1;
            for (int x = 0; x < W; ++x) {
                int cur = row[x];
                int nv = max((int)irow[x], min(cur, prev));
                if (nv != cur) { row[x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
            prev = -1;
            for (int x = W - 1; x >= 0; --x) {
                int cur = row[x];
                int nv = max((int)irow[x], min(cur, prev));
                if (nv != cur) { row[x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
        }
        __syncthreads();
        if (threadIdx.x < W) {
            const int x = threadIdx.x;
            int prev = -1;
            for (int y = 0; y < H; ++y) {
                int cur = psi[y * P + x];
                int nv = max((int)img[y * P + x], min(cur, prev));
                if (nv != cur) { psi[y * P + x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
            prev = -1;
            for (int y = H - 1; y >= 0; --y) {
                int cur = psi[y * P + x];
                int nv = max((int)img[y * P + x], min(cur, prev));
                if (nv != cur) { psi[y * P + x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
        }
        if (ch) changed = 1;  // benign same-value race
        __syncthreads();
        if (!changed) break;
        __syncthreads();
    }
    uint8_t* dst = psi_out + (long)b * H * W;
    for (int i = threadIdx.x; i < 257; i += NTB) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < H * W; i += NTB) {
        int y = i / W, x = i - y * W;
        const uint8_t v = psi[y * P + x];
        dst[i] = v;
        atomicAdd(&hist[v], 1);
    }
    __syncthreads();
    // F_L = {psi > L} only changes at L = v - 1 for psi values v present:
    // compute boxes for those levels only; canon[L] names the level whose
    // F (and box) equals F_L (max(psi) = vmax, so every L < vmax maps).
    if (threadIdx.x == 0) {
        int n = 0, next = vm - 1;
        for (int L = vm - 1; L >= 0; --L) {
            if (hist[L + 1] > 0) next = L;
            canon[b * 256 + L] = next;
        }
        for (int L = 0; L < vm; ++L)
            if (hist[L + 1] > 0) lev_list[b * 256 + n++] = L;
        nlev[b] = n;
    }
}

// --------------------------------------------------------------- levels
// One workgroup per (frame, chunk of distinct levels).  psi is held in
// registers (32 pixels = 8 packed dwords per bitmap word, <= 2 words per
// thread); each level builds the bitmap F = {psi > L} in LDS, labels 2x2
// pixel blocks with a lock-free union-find (atomicMin hooks toward the
// smaller index; in a 2x2 block all foreground pixels are 8-connected, so
// block labels are pixel labels), then reuses each ROOT's label slot as its
// area accumulator (flag bit 31 marks a root slot).
constexpr int LMAXH = 256, LMAXW = 256;
constexpr int LWPR = LMAXW / 32;                 // bitmap words per row (max)
constexpr int LMAXNB = (LMAXH / 2) * (LMAXW / 2);
constexpr uint32_t RFLAG = 0x80000000u;
constexpr uint32_t NOKEY = RFLAG | 0x7FFFFFFFu;  // non-candidate root slot
constexpr int LEVEL_CHUNKS = 16;

__device__ inline uint32_t find_root(const volatile uint32_t* lab, uint32_t x) {
    uint32_t p = lab[x];
    while (p != x) {
        x = p;
        p = lab[x];
    }
    return x;
}

__device__ inline void unite(uint32_t* lab, uint32_t a, uint32_t b) {
    for (;;) {
        a = find_root(lab, a);
        b = find_root(lab, b);
        if (a == b) return;
        if (a > b) { uint32_t t = a; a = b; b = t; }
        uint32_t old = atomicMin(&lab[b], a);
        if (old == b) return;
        b = old;
    }
}

struct LevelCtx {
    const uint32_t* bm;  // bitmap, H x wpr words
    int H, W, wpr, BW;
    __device__ inline int bit(int y, int x) const {
        if ((unsigned)y >= (unsigned)H || (unsigned)x >= (unsigned)W) return 0;
        return (bm[y * wpr + (x >> 5)] >> (x & 31)) & 1;
    }
    // 2 bits (x, x+1) of row y, x even.
    __device__ inline int pair(int y, int x) const {
        if ((unsigned)y >= (unsigned)H || (unsigned)x >= (unsigned)W) return 0;
        return (bm[y * wpr + (x >> 5)] >> (x & 31)) & 3;
    }
    __device__ inline uint32_t word(int y, int j) const {
        if ((unsigned)y >= (unsigned)H || (unsigned)j >= (unsigned)wpr) return 0u;
        return bm[y * wpr + j];
    }
};

__device__ inline uint32_t root_of(const uint32_t* lab, uint32_t b) {
    uint32_t v = lab[b];
    return (v & RFLAG) ? b : v;
}

__global__ __launch_bounds__(NTB) void level_kernel(const uint8_t* __restrict__ psi_g,
                                                    const int32_t* __restrict__ vmax,
                                                    const int32_t* __restrict__ lev_list,
                                                    const int32_t* __restrict__ nlev,
                                                    int32_t* __restrict__ boxes, int H, int W) {
    __shared__ uint32_t bm[LMAXH * LWPR];
    __shared__ uint32_t lab[LMAXNB];
    __shared__ int red[4 * (NTB / 64) + 4];

    const int b = blockIdx.x / LEVEL_CHUNKS;
    const int chunk = blockIdx.x % LEVEL_CHUNKS;
    const int nl = nlev[b];
    if (chunk >= nl) return;
    const int wpr = (W + 31) / 32;
    const int NW = H * wpr;
    const int BW = (W + 1) / 2, BH = (H + 1) / 2, NB = BH * BW;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // psi of this thread's bitmap words -> registers (8 packed dwords/word).
    uint32_t pv[2][8];
    const uint8_t* src = psi_g + (long)b * H * W;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int w = tid + q * NTB;
#pragma unroll
        for (int d = 0; d < 8; ++d) pv[q][d] = 0u;
        if (w < NW) {
            const int y = w / wpr, x0 = (w - y * wpr) * 32;
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int x = x0 + 4 * d + e;
                    if (x < W) v |= (uint32_t)src[y * W + x] << (8 * e);
                }
                pv[q][d] = v;
            }
        }
    }
    LevelCtx cx{bm, H, W, wpr, BW};

    for (int li = chunk; li < nl; li += LEVEL_CHUNKS) {
        const int L = lev_list[b * 256 + li];
        int32_t* box = boxes + ((long)b * 256 + L) * 4;
        // 1. bitmap F = {psi > L}.
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int w = tid + q * NTB;
            if (w < NW) {
                uint32_t bits = 0;
#pragma unroll
                for (int d = 0; d < 8; ++d)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        bits |= (uint32_t)(((pv[q][d] >> (8 * e)) & 255u) > (uint32_t)L) << (4 * d + e);
                bm[w] = bits;
            }
        }
        __syncthreads();
        // 2. block activity.
        for (int i = tid; i < NB; i += NTB) {
            const int by = i / BW, x = 2 * (i - by * BW), y = 2 * by;
            lab[i] = (cx.pair(y, x) | cx.pair(y + 1, x)) ? (uint32_t)i : INACT;
        }
        __syncthreads();
        // 3. union with the left, top-left, top and top-right blocks.
        for (int i = tid; i < NB; i += NTB) {
            if (lab[i] == INACT) continue;
            const int by = i / BW, bx = i - by * BW, y = 2 * by, x = 2 * bx;
            const int top = cx.pair(y, x);             // bit0 = (y,x), bit1 = (y,x+1)
            const int left = (top & 1) | cx.bit(y + 1, x);
            if (bx > 0 && left && (cx.bit(y, x - 1) | cx.bit(y + 1, x - 1))) unite(lab, i, i - 1);
            if (by > 0) {
                if (top && cx.pair(y - 1, x)) unite(lab, i, i - BW);
                if (bx > 0 && (top & 1) && cx.bit(y - 1, x - 1)) unite(lab, i, i - BW - 1);
                if (bx + 1 < BW && (top & 2) && cx.bit(y - 1, x + 2)) unite(lab, i, i - BW + 1);
            }
        }
        __syncthreads();
        // 4. flatten, then 5. turn root slots into area accumulators.
        for (int i = tid; i < NB; i += NTB)
            if (lab[i] != INACT) lab[i] = find_root(lab, i);
        __syncthreads();
        for (int i = tid; i < NB; i += NTB)
            if (lab[i] == (uint32_t)i) lab[i] = RFLAG;
        __syncthreads();
        // 6. window areas in half units: per 32-window strip, windows with
        // >= 3 pixels in F form runs; one run = one component (adjacent
        // windows share two pixels, at least one of them in F).
        {
            const int nsj = (W + 1 + 31) / 32;   // strips per window row (wx in [-1, W-1])
            const int nstrips = (H + 1) * nsj;
            for (int st = tid; st < nstrips; st += NTB) {
                const int wy = st / nsj - 1, j = st % nsj;
                // window wx = 32j - 1 + i covers pixels x = 32j - 1 + i, 32j + i
                const uint32_t t0 = cx.word(wy, j), t1 = cx.word(wy + 1, j);
                const uint32_t tp = cx.word(wy, j - 1), bp = cx.word(wy + 1, j - 1);
                const uint32_t tl = (t0 << 1) | (tp >> 31), tr = t0;
                const uint32_t bl = (t1 << 1) | (bp >> 31), br = t1;
                uint32_t m3 = (tl & tr & (bl | br)) | (bl & br & (tl | tr));
                const uint32_t m4 = tl & tr & bl & br;
                const int nvalid = W + 1 - 32 * j;          // windows in this strip
                if (nvalid < 32) m3 &= (1u << nvalid) - 1u;
                while (m3) {
                    const int s0 = __builtin_ctz(m3);
                    const uint32_t rest = ~(m3 >> s0);
                    const int len = rest ? __builtin_ctz(rest) : 32 - s0;
                    const uint32_t run = (len >= 32 ? 0xFFFFFFFFu : ((1u << len) - 1u)) << s0;
                    const uint32_t contrib = __builtin_popcount(run) + __builtin_popcount(m4 & run);
                    // an F pixel of window s0
                    const int wx = 32 * j - 1 + s0;
                    int py, px;
                    if ((tl >> s0) & 1) { py = wy; px = wx; }
                    else if ((tr >> s0) & 1) { py = wy; px = wx + 1; }
                    else if ((bl >> s0) & 1) { py = wy + 1; px = wx; }
                    else { py = wy + 1; px = wx + 1; }
                    const uint32_t r = root_of(lab, (py >> 1) * BW + (px >> 1));
                    atomicAdd(&lab[r], contrib);
                    m3 &= ~run;
                }
            }
        }
        __syncthreads();
        // 7. max area over roots.
        int ma = -1;
        for (int i = tid; i < NB; i += NTB) {
            const uint32_t v = lab[i];
            if (v != INACT && (v & RFLAG)) ma = max(ma, (int)(v & ~RFLAG));
        }
        ma = block_max_i(ma, red);
        // 8. candidates (area == max) get a key slot; others NOKEY.
        for (int i = tid; i < NB; i += NTB) {
            const uint32_t v = lab[i];
            if (v != INACT && (v & RFLAG))
                lab[i] = ((int)(v & ~RFLAG) == ma) ? (RFLAG | 0x7FFFFFFEu) : NOKEY;
        }
        __syncthreads();
        // 9. key = 1 + raster index of the component's first pixel.
        for (int i = tid; i < NB; i += NTB) {
            if (lab[i] == INACT) continue;
            const uint32_t r = root_of(lab, i);
            if (lab[r] == NOKEY) continue;
            const int by = i / BW, x = 2 * (i - by * BW), y = 2 * by;
            const int top = cx.pair(y, x);
            int k;
            if (top & 1) k = y * W + x;
            else if (top & 2) k = y * W + x + 1;
            else if (cx.bit(y + 1, x)) k = (y + 1) * W + x;
            else k = (y + 1) * W + x + 1;
            atomicMin(&lab[r], RFLAG | (uint32_t)(k + 1));
        }
        __syncthreads();
        // 10. winner = candidate with the largest key (first in OpenCV's list).
        int best = 0;
        for (int i = tid; i < NB; i += NTB) {
            const uint32_t v = lab[i];
            if (v != INACT && (v & RFLAG) && v != NOKEY) best = max(best, (int)(v & ~RFLAG));
        }
        best = block_max_i(best, red);
        const int fp = best - 1;
        const uint32_t wroot = root_of(lab, ((fp / W) >> 1) * BW + ((fp % W) >> 1));
        // 11. bbox of the winner (4 reductions in one pass).
        int x0 = W, y0 = H, x1 = -1, y1 = -1;
        for (int i = tid; i < NB; i += NTB) {
            if (lab[i] == INACT || root_of(lab, i) != wroot) continue;
            const int by = i / BW, x = 2 * (i - by * BW), y = 2 * by;
            const int top = cx.pair(y, x), bot = cx.pair(y + 1, x);
            if (top | bot) {
                x0 = min(x0, ((top | bot) & 1) ? x : x + 1);
                x1 = max(x1, ((top | bot) & 2) ? x + 1 : x);
                y0 = min(y0, top ? y : y + 1);
                y1 = max(y1, bot ? y + 1 : y);
            }
        }
        x0 = wave_min_i(x0); y0 = wave_min_i(y0);
        x1 = wave_max_i(x1); y1 = wave_max_i(y1);
        if (lane == 0) {
            red[4 * wid + 0] = x0; red[4 * wid + 1] = y0;
            red[4 * wid + 2] = x1; red[4 * wid + 3] = y1;
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < NTB / 64; ++w) {
                x0 = min(x0, red[4 * w + 0]); y0 = min(y0, red[4 * w + 1]);
                x1 = max(x1, red[4 * w + 2]); y1 = max(y1, red[4 * w + 3]);
            }
            box[0] = x0;
            box[1] = y0;
            box[2] = min(x1 + 1, W - 1);  // boundingRect x + w, clamped (wsol_metrics.py:175-178)
            box[3] = min(y1 + 1, H - 1);
        }
        __syncthreads();
    }
}

// Fill the rows of non-canonical levels from their canonical level.
__global__ void expand_kernel(const int32_t* __restrict__ canon, const int32_t* __restrict__ vmax,
                              int32_t* __restrict__ boxes, int B) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * 256) return;
    const int b = i / 256, L = i % 256;
    if (L >= vmax[b]) return;
    const int c = canon[b * 256 + L];
    if (c == L) return;
    const int32_t* s = boxes + ((long)b * 256 + c) * 4;
    int32_t* d = boxes + ((long)b * 256 + L) * 4;
    d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = s[3];
}

// ------------------------------------------------------------ accumulate
__global__ void accumulate_kernel(const int32_t* __restrict__ boxes,
                                  const int32_t* __restrict__ vmax, const double* __restrict__ taus,
                                  int T, const int32_t* __restrict__ gt,
                                  const int32_t* __restrict__ ngt, int G,
                                  const int32_t* __restrict__ top1,
                                  const int32_t* __restrict__ top5,
                                  const double* __restrict__ iou_thr, int n_iou,
                                  int32_t* __restrict__ counters, double* __restrict__ best_iou,
                                  int B) {
    long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (long)B * T) return;
    const int b = (int)(id / T), i = (int)(id % T);
    const int vm = vmax[b];
    // thresh = int(threshold * np.max(scoremap_image))  (wsol_metrics.py:158)
    const int thr = (int)(taus[i] * (double)vm);
    int a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (thr < vm) {
        const int32_t* bx = boxes + ((long)b * 256 + thr) * 4;
        a0 = bx[0]; a1 = bx[1]; a2 = bx[2]; a3 = bx[3];
    }
    // calculate_multiple_iou (wsol_metrics.py:77-124), max over GT boxes.
    double best = 0.0;
    const int ng = ngt[b];
    for (int g = 0; g < ng; ++g) {
        const int32_t* q = gt + ((long)b * G + g) * 4;
        long mnx = max(a0, q[0]), mny = max(a1, q[1]);
        long mxx = min(a2, q[2]), mxy = min(a3, q[3]);
        long inter = max(0L, mxx - mnx + 1) * max(0L, mxy - mny + 1);
        long area_a = (long)(a2 - a0 + 1) * (a3 - a1 + 1);
        long area_b = (long)(q[2] - q[0] + 1) * (q[3] - q[1] + 1);
        long den = area_a + area_b - inter;
        double iou = den <= 0 ? 0.0 : (double)inter / (double)den;
        if (g == 0 || iou > best) best = iou;
    }
    if (best_iou) best_iou[id] = best;
    for (int j = 0; j < n_iou; ++j) {
        if (best >= iou_thr[j]) {
            atomicAdd(&counters[(0 * n_iou + j) * T + i], 1);
            if (top1[b]) atomicAdd(&counters[(1 * n_iou + j) * T + i], 1);
            if (top5[b]) atomicAdd(&counters[(2 * n_iou + j) * T + i], 1);
        }
    }
}

}  // namespace

extern "C" size_t tcam_bbox_ws_bytes(int B, int H, int W) {
    // psi (uint8, 16-byte aligned) | canon (B x 256) | lev_list (B x 256) | nlev (B)
    size_t psi = ((size_t)B * H * W + 15) / 16 * 16;
    return psi + (size_t)B * (256 + 256 + 1) * sizeof(int32_t);
}

extern "C" int tcam_bbox_levels(const uint8_t* cam_u8, int32_t* boxes, int32_t* vmax,
                                void* ws, int B, int H, int W, void* stream) {
    TCAM_REQUIRE(cam_u8 && boxes && vmax && ws && B > 0);
    TCAM_REQUIRE(H > 0 && W > 0 && H <= MAXH && W <= MAXW && pitch_of(W) <= MAXP);
    TCAM_REQUIRE(H <= LMAXH && W <= LMAXW);
    hipStream_t st = as_stream(stream);
    uint8_t* psi = (uint8_t*)ws;
    int32_t* canon = (int32_t*)((char*)ws + ((size_t)B * H * W + 15) / 16 * 16);
    int32_t* lev_list = canon + (size_t)B * 256;
    int32_t* nlev = lev_list + (size_t)B * 256;
    fill_kernel<<<B, NTB, 0, st>>>(cam_u8, psi, vmax, canon, lev_list, nlev, H, W);
    TCAM_CHECK_LAUNCH();
    level_kernel<<<B * LEVEL_CHUNKS, NTB, 0, st>>>(psi, vmax, lev_list, nlev, boxes, H, W);
    TCAM_CHECK_LAUNCH();
    expand_kernel<<<cdiv((long)B * 256, 256), 256, 0, st>>>(canon, vmax, boxes, B);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_box_accumulate(const int32_t* boxes, const int32_t* vmax, const double* taus,
                                   int T, const int32_t* gt, const int32_t* ngt, int G,
                                   const int32_t* top1, const int32_t* top5,
                                   const double* iou_thr, int n_iou, int32_t* counters,
                                   double* best_iou, int B, void* stream) {
    TCAM_REQUIRE(boxes && vmax && taus && gt && ngt && top1 && top5 && iou_thr && counters);
    TCAM_REQUIRE(T > 0 && G > 0 && n_iou > 0 && B > 0);
    long total = (long)B * T;
    accumulate_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        boxes, vmax, taus, T, gt, ngt, G, top1, top5, iou_thr, n_iou, counters, best_iou, B);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
